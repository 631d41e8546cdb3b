"""test10_servo_vecenv.py's own mode, the CPU pipeline (host state tensors,
SURVEY.md §0.7, BASELINE config 2), on the device: fetch_results(sim, True)
stages the whole state in one round trip (mg_fetch_host_state) and the
refresh_*_tensor calls that follow copy from it — unless a simulate or a
state set intervened, which sends the refresh back to the device. Checked bit
for bit against the oracle every step, including a set between fetch and
refresh (the refresh must show the set's state, not the staged one)."""
import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import scenes
import oracle

pytestmark = pytest.mark.gpu


def test_cpu_pipeline_staged_refreshes_gpu(gym):
    n = 256
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    assert root.device.type == "cpu" and sim.host_stage is not None
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    roots = A["actor_root_body"]
    acts = scenes.servo_actions(n, 8, "cpu", seed=4)
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(40):
        root[:, 3:10] = acts[k % 8]
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        st[roots, 3:10] = acts[k % 8].numpy()
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        cf = oracle.step(p, m, st, dof)
        assert sim.host_stage_epoch == sim.epoch
        if k % 10 == 5:
            # a set between fetch and refresh (every root from the host tensor,
            # still holding the previous refresh, one of them moved): the
            # refresh shows the set's state, not the staged one
            root[0, 0:3] = torch.tensor([1.0, 2.0, 150.0])
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            st[roots] = root.numpy()
            assert sim.host_stage_epoch != sim.epoch
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        gym.refresh_dof_state_tensor(sim)
        assert np.array_equal(rb.numpy(), st), "step %d: rigid-body tensor" % k
        assert np.array_equal(root.numpy(), st[roots]), "step %d: root tensor" % k
        if k % 10 != 5:
            assert np.array_equal(ncf.numpy(), cf), "step %d: net contact force" % k


def test_cpu_pipeline_copy_at_set_and_set_before_fetch_gpu(gym):
    """The host root set is Isaac Gym's copy-at-set: the tensor is copied at
    the call (into the library's page-locked buffer) and read by the next
    simulate's step kernel, so overwriting the host tensor right after the set
    changes nothing. And a set between simulate and fetch_results: the staged
    state is the set's (the step's own output rows are stale then, so the
    fetch gathers). Bit for bit the oracle."""
    n = 128
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    roots = A["actor_root_body"]
    acts = scenes.servo_actions(n, 8, "cpu", seed=6)
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(24):
        root[:, 3:10] = acts[k % 8]
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        st[roots, 3:10] = acts[k % 8].numpy()
        root.fill_(float("nan"))                 # overwritten right after the set
        gym.simulate(sim)
        oracle.step(p, m, st, dof)
        if k % 6 == 3:
            # a set after the simulate and before the fetch: the staged state is the set's
            gym.refresh_actor_root_state_tensor(sim)        # (the tensor holds the state again)
            root[1, 0:3] = torch.tensor([-3.0, 4.0, 120.0])
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            st[roots] = root.numpy()
        gym.fetch_results(sim, True)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        assert np.array_equal(rb.numpy(), st), "step %d: rigid-body tensor" % k
        assert np.array_equal(root.numpy(), st[roots]), "step %d: root tensor" % k


@pytest.mark.parametrize("kind", ["gimbal", "pile"])
def test_cpu_pipeline_other_kernels_gpu(gym, kind):
    """The zero-copy host stage with the other step kernels: the S2 gimbal
    (k_artic_chain writes its body and DOF rows into the mapped stage itself;
    DOF targets set from a host tensor every step) and the S6 ball pile
    (k_pile_step: the fetch gathers into the mapped stage). Every step's
    refreshed host tensors equal the oracle bit for bit."""
    n, steps = 64, 30
    if kind == "gimbal":
        sim, _ = scenes.gimbal_scene(gym, n, use_gpu_pipeline=False)
    else:
        sim, _ = scenes.ball_pile_scene(gym, 8, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    assert rb.device.type == "cpu" and sim.host_stage is not None
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    st, ds = A["body_state0"].copy(), A["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    tg = scenes.gimbal_targets(n, steps, "cpu", seed=8) if kind == "gimbal" else None
    for k in range(steps):
        if tg is not None:
            t = tg[k].contiguous()
            assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(t))
            tgt[:, 0] = t.numpy()
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        oracle.step(p, m, st, ds, tgt=tgt)
        gym.refresh_rigid_body_state_tensor(sim)
        if ds.shape[0]:
            gym.refresh_dof_state_tensor(sim)
            assert np.array_equal(dof.numpy(), ds), "step %d: DOF tensor" % k
        assert np.array_equal(rb.numpy(), st), "step %d: rigid-body tensor" % k
