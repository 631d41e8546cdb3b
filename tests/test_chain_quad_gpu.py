"""GPU parity of the S2 chain kernels at the launch sizes that select each form
(mg_chain.hip mg_launch_artic_chain: four lanes per chain, k_artic_chain_q,
while na x 4 <= 65,536 lanes; one lane per chain, k_artic_chain, beyond), with
external wrenches (the EXT variants) and with chains of two and three links —
a tilted joint frame, COM offsets and a prismatic joint under gravity (NL = 2,
3) — bit for bit against oracle.step (oracle/migym_oracle.c chain_step_).
Launch sizes that end in a partly filled wave leave whole dead quads in it."""
import os

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import scenes
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _run_gimbals(gym, n, steps, seed, ext_every=0):
    sim, _ = scenes.gimbal_scene(gym, n)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    tg = scenes.gimbal_targets(n, steps, DEV, seed=seed)
    tg_h = tg.cpu().numpy()
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    nb = st.shape[0]
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    rng = np.random.RandomState(seed)
    for k in range(steps):
        assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k].contiguous()))
        ext = None
        if ext_every and k % ext_every == 0:
            ext = rng.uniform(-0.05, 0.05, (nb, 6)).astype(np.float32)
            ext[0::4] = 0.0                                  # the fixed base of each gimbal
            f = torch.from_numpy(ext[:, 0:3].copy()).to(DEV).view(n, 4, 3)
            t = torch.from_numpy(ext[:, 3:6].copy()).to(DEV).view(n, 4, 3)
            assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(f), gymtorch.unwrap_tensor(t),
                                                      gymapi.ENV_SPACE)
        gym.simulate(sim)
        tgt[:, 0] = tg_h[k]
        oracle.step(p, m, st, ds, tgt=tgt, ext=ext)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    gym.destroy_sim(sim)
    return got_d, ds, got, st


def test_gimbal_one_lane_launch_parity(gym):
    """16,448 gimbals: past the four-lane bound, the one-lane kernel in a launch
    of one resident round (257 workgroups: no LDS row staging)."""
    got_d, ds, got, st = _run_gimbals(gym, 16448, 12, seed=21)
    assert np.all(np.isfinite(got_d)) and np.abs(got_d[:, 1]).max() > 0.05
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


def test_gimbal_quad_external_wrench_parity(gym):
    """100 gimbals (400 lanes: the last wave 16 of 64 live) with random
    world-frame forces and torques on the links every third step (the EXT
    variant of the four-lane kernel: each lane's own link's wrench)."""
    got_d, ds, got, st = _run_gimbals(gym, 100, 30, seed=22, ext_every=3)
    assert np.all(np.isfinite(got_d))
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


def _chain_urdf(d, nl):
    """Fixed base, then a revolute link about a tilted axis with its COM off
    the joint, then (nl = 3) a prismatic link along the first link's x."""
    inert = ('<inertial><origin xyz="%s"/><mass value="%s"/>'
             '<inertia ixx="0.004" iyy="0.006" izz="0.003" ixy="0.0005" ixz="0" iyz="0.0002"/></inertial>')
    links = ['<link name="base"><collision><geometry><box size="0.1 0.1 0.1"/></geometry></collision></link>',
             '<link name="arm">' + inert % ("0.15 0.02 0", "0.7") + '</link>']
    joints = ['<joint name="hinge" type="revolute"><parent link="base"/><child link="arm"/>'
              '<origin xyz="0 0 0.2" rpy="0.3 -0.2 0.5"/><axis xyz="0 0.6 0.8"/>'
              '<limit lower="-2.5" upper="2.5" effort="40" velocity="6"/></joint>']
    if nl == 3:
        links.append('<link name="slider">' + inert % ("0.05 0 0.01", "0.4") + '</link>')
        joints.append('<joint name="slide" type="prismatic"><parent link="arm"/><child link="slider"/>'
                      '<origin xyz="0.3 0 0" rpy="0 0 0.4"/><axis xyz="1 0 0"/>'
                      '<limit lower="-0.2" upper="0.2" effort="60" velocity="2"/></joint>')
    name = "chain%d.urdf" % nl
    with open(os.path.join(d, name), "w") as f:
        f.write('<robot name="chain%d">' % nl + "".join(links + joints) + "</robot>")
    return name


@pytest.mark.parametrize("nl", [2, 3])
def test_short_chain_quad_parity(gym, tmp_path, nl):
    """Chains of two and three links (one and two DOFs) under gravity and PD
    drives with random targets: the four-lane kernel's NL = 2 / 3 forms, lanes
    past the last link idle in the quad; 77 instances (a partial last wave)."""
    sp = gymapi.SimParams()
    sp.dt, sp.substeps = 1.0 / 60.0, 2
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0.0, 0.0, -9.8)
    sp.physx.solver_type = 1
    sp.use_gpu_pipeline = True
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    asset = gym.load_asset(sim, str(tmp_path), _chain_urdf(str(tmp_path), nl), opts)
    n, steps = 77, 40
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 9)
        h = gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 1)), "chain", i, 1)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_POS
        props["stiffness"][:] = 80.0
        props["damping"][:] = 3.0
        gym.set_actor_dof_properties(env, h, props)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    nd = ds.shape[0]
    assert nd == n * (nl - 1)
    rng = np.random.RandomState(30 + nl)
    tgt = np.zeros((nd, 3), np.float32)
    for k in range(steps):
        if k % 8 == 0:
            tgt[:, 0] = rng.uniform(-1.0, 1.0, nd).astype(np.float32)
            if nl == 3:
                tgt[1::2, 0] *= 0.15                     # the slider's targets in metres
            assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(
                torch.from_numpy(tgt[:, 0].copy()).to(DEV)))
        gym.simulate(sim)
        oracle.step(p, m, st, ds, tgt=tgt)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    gym.destroy_sim(sim)
    assert np.all(np.isfinite(got_d)) and np.abs(got_d[:, 1]).max() > 0.05
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
