"""GPU parity of the free bodies' ground friction patches (DESIGN.md §3.2.1,
mg_rigid.hip k_rigid_step1 with its persistent [MG_FP_N][nf1] record table)
against the oracle (oracle/migym_oracle.c rigid_body_step, its body cache kept
from step to step the same way), bit for bit:

  - test10's servo scene (UAV + ground vehicle per env, the patch parameters at
    Isaac Gym's defaults) under a random root teleport every frame (vehicles
    thrown at up to 50 m/s: anchors made and dropped), then one gentle teleport
    of every vehicle to 0.15 m above its rest height at rest and 40 frames in
    which they land and come to rest on their anchors;
  - ground vehicles pushed sideways through apply_rigid_body_force_tensors at
    0.5 / 0.9 / 1.1 / 1.5 mu m g (held below, sliding above), with a teleport
    of every other env half-way (the held anchors let go of a moved body).
"""
import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import scenes
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_servo_teleports_then_rest_bitexact(gym):
    n, teleports, rest = 256, 40, 40
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    acts = scenes.servo_actions(n, teleports, DEV, seed=31)
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    st = sim.model_arrays["body_state0"].copy()
    roots = sim.model_arrays["actor_root_body"]
    dof = np.zeros((0, 2), np.float32)
    gym.refresh_actor_root_state_tensor(sim)
    held_seen = 0
    for k in range(teleports + rest):
        if k < teleports:
            root[:, 3:10] = acts[k]
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            st[roots, 3:10] = acts[k].cpu().numpy()
        elif k == teleports:                   # vehicles set down at rest, yaw kept
            root[1::2, 2] = 1.4
            root[1::2, 7:13] = 0.0
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            st[roots[1::2], 2] = 1.4
            st[roots[1::2], 7:13] = 0.0
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        cf = oracle.step(p, m, st, dof, contact_cache=cc)
        got = rb.cpu().numpy()
        assert np.array_equal(got, st), "frame %d: max |diff| %g" % (k, np.abs(got - st).max())
        assert np.array_equal(ncf.cpu().numpy(), cf), "frame %d: contact force" % k
        held_seen = max(held_seen, int((cc.body[:, 0] == 2.0).sum()))
    assert held_seen >= n                      # every vehicle came to rest on two anchors
    veh = roots[1::2]
    assert np.all(np.abs(st[veh, 2] - 1.25) < 2e-3) and np.all(np.abs(st[veh, 7:10]) < 1e-2)


def test_vehicle_pushes_bitexact(gym):
    n, frames = 64, 90
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    A = sim.model_arrays
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    nb = st.shape[0]
    for _ in range(60):                      # the vehicles settle (the UAVs keep falling)
        gym.simulate(sim)
        oracle.step(p, m, st, dof, contact_cache=cc)
    mu = 0.5 * (float(A["shapes"][int(A["tmpl_body_i"][A["body_tmpl"][1]][0])][11]) + 1.0)
    force = np.zeros((nb, 3), np.float32)
    pushes = np.array([0.5, 0.9, 1.1, 1.5], np.float32)[np.arange(n) % 4]
    force[1::2, 0] = pushes * mu * 100.0 * 9.8
    force[1::2, 1] = np.where(np.arange(n) % 8 >= 4, 0.3, 0.0) * mu * 100.0 * 9.8
    ext = np.zeros((nb, 6), np.float32)
    ext[:, 0:3] = force
    ft = torch.from_numpy(force).to(DEV)
    tq = torch.zeros_like(ft)
    x0 = st[1::2, 0].copy()
    for k in range(frames):
        if k == frames // 2:                 # teleport every other vehicle 2 m sideways
            gym.refresh_actor_root_state_tensor(sim)
            sel = torch.arange(1, 2 * n, 4, device=DEV)
            root[sel, 1] += 2.0
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            st[np.arange(1, 2 * n, 4), 1] += 2.0
        assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(ft), gymtorch.unwrap_tensor(tq),
                                                  gymapi.ENV_SPACE)
        gym.simulate(sim)
        oracle.step(p, m, st, dof, ext=ext, contact_cache=cc)
    gym.refresh_rigid_body_state_tensor(sim)
    got = rb.cpu().numpy()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
    moved = np.abs(st[1::2, 0] - x0)
    assert np.all(moved[pushes < 1.0] < 2e-3) and np.all(moved[pushes > 1.0] > 0.05)
