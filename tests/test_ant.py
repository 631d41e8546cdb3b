"""Floating-base articulations and the MJCF importer (SURVEY.md §8f rank 2:
assets/mjcf/nv_ant.xml as loaded by examples/apply_forces.py:67).

CPU: the importer against the reference's MJCF (when /root/reference is
present) and the repo's re-serialized copy (tools/make_ant_asset.py); oracle
KATs of the floating-base coupled step: exact discrete free fall, momentum
under internal joint torques in zero gravity, the ant settling on the ground,
the apply_forces.py vertical push. GPU: k_env_step vs the oracle bit for bit
on ant envs with random DOF efforts, random root poses and body forces.
"""
import os

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import _assets, _types, scenes
import oracle

REF_ANT = "/root/reference/assets/mjcf/nv_ant.xml"
H = 1.0 / 60.0


def test_mjcf_ant_import():
    a = _assets.load_mjcf(scenes.ASSET_ROOT, "mjcf/ant.xml", _types.AssetOptions())
    assert [b.name for b in a.bodies] == ["torso", "front_left_leg", "front_left_foot", "front_right_leg",
                                         "front_right_foot", "left_back_leg", "left_back_foot",
                                         "right_back_leg", "right_back_foot"]
    assert a.num_dofs == 8
    assert [j.name for j in a.dof_joints] == ["hip_1", "ankle_1", "hip_2", "ankle_2", "hip_3", "ankle_3",
                                              "hip_4", "ankle_4"]
    p = a.dof_props
    assert np.allclose(p["lower"][[0, 1, 3]], np.radians([-40, 30, -100]))
    assert np.allclose(p["upper"][[0, 1, 3]], np.radians([40, 100, -30]))
    assert np.allclose(p["armature"], 0.01) and np.allclose(p["damping"], 0.1)
    assert np.allclose(p["effort"], 15.0)                       # motor gear 15 x ctrlrange 1
    # torso: sphere r 0.25 + 4 capsules (r 0.08, length 0.2 sqrt 2) at density 5
    L = 0.2 * np.sqrt(2.0)
    cap = np.pi * 0.08 ** 2 * L + 4.0 / 3.0 * np.pi * 0.08 ** 3
    m_torso = 5.0 * (4.0 / 3.0 * np.pi * 0.25 ** 3 + 4 * cap)
    assert abs(a.mass_props[0].mass - m_torso) < 1e-9
    assert np.allclose(a.mass_props[1].com, [0.1, 0.1, 0.0])   # leg capsule centre
    sh = a.bodies[2].shapes[0]
    assert sh.type == _assets.CAPSULE and np.allclose(sh.size, [0.08, 0.2 * np.sqrt(2.0)])
    assert all(s.friction == 1.5 for b in a.bodies for s in b.shapes)


@pytest.mark.skipif(not os.path.exists(REF_ANT), reason="reference MJCF not present")
def test_repo_ant_matches_reference_mjcf():
    a = _assets.load_mjcf(os.path.dirname(os.path.dirname(REF_ANT)), "mjcf/nv_ant.xml", _types.AssetOptions())
    b = _assets.load_mjcf(scenes.ASSET_ROOT, "mjcf/ant.xml", _types.AssetOptions())
    assert len(a.bodies) == len(b.bodies)
    for x, y in zip(a.mass_props, b.mass_props):
        assert x.mass == y.mass and np.array_equal(x.com, y.com) and np.array_equal(x.inertia, y.inertia)
    assert (a.dof_props == b.dof_props).all()


def _model(gym, n, height=1.0, gravity=-9.81, damping=True):
    sp = scenes.ant_sim_params(False)
    sp.gravity = gymapi.Vec3(0.0, 0.0, gravity)
    opts = gymapi.AssetOptions()
    if not damping:                   # the root link's default angular damping (0.5) is an external loss
        opts.angular_damping = 0.0
        opts.linear_damping = 0.0
    sim, info = scenes.ant_scene(gym, n, use_gpu_pipeline=False, height=height, sim_params=sp, asset_options=opts)
    A = sim.build_model()
    return sim, A


def test_floating_base_free_fall_exact(gym):
    """No contacts, joints at rest mid-range: every body falls as one rigid body,
    z_n = z0 - g h^2 n (n + 1) / 2 (semi-implicit Euler), joints do not move."""
    sim, A = _model(gym, 2, height=50.0)
    p, m = sim.mg_params(), sim.mg_model()
    st, dof, pr = A["body_state0"].copy(), A["dof_state0"].copy(), A["dof_props"]
    dof[:, 0] = 0.5 * (pr[:, 5] + pr[:, 6])
    n = 60
    for _ in range(n):
        oracle.step(p, m, st, dof, props=pr)
    assert abs((50.0 - st[0, 2]) - 9.81 * H * H * n * (n + 1) / 2) < 2e-4
    assert abs(st[0, 9] + 9.81 * H * n) < 1e-4
    assert np.abs(dof[:, 1]).max() == 0.0
    assert np.allclose(st[0, 3:7], [0.0, 0.0, 0.0, 1.0]) and np.abs(st[:, 10:13]).max() < 1e-5


def test_floating_base_momentum_zero_gravity(gym):
    """Zero gravity, constant random joint efforts: the internal torques leave the
    total linear momentum ~0 (first-order integrator drift only) while the legs
    swing at ~1 rad/s."""
    sim, A = _model(gym, 1, height=50.0, gravity=0.0, damping=False)
    p, m = sim.mg_params(), sim.mg_model()
    st, dof, pr = A["body_state0"].copy(), A["dof_state0"].copy(), A["dof_props"].copy()
    dof[:, 0] = 0.5 * (pr[:, 5] + pr[:, 6])
    pr[:, 0] = 3.0                                           # DOF_MODE_EFFORT
    tgt = np.zeros((8, 3), np.float32)
    tgt[:, 2] = np.random.RandomState(0).uniform(-0.05, 0.05, 8)
    mass = A["body_mass"][:, 11]
    for _ in range(30):
        oracle.step(p, m, st, dof, tgt=tgt, props=pr)
    P = (mass[:9, None] * st[:9, 7:10]).sum(0)
    link_p = (mass[:9] * np.linalg.norm(st[:9, 7:10], axis=1)).sum()
    assert np.abs(dof[:, 1]).max() > 0.5
    assert np.linalg.norm(P) < 0.01 * link_p


def test_ant_settles_and_jumps(gym):
    """Dropped from 1 m the ants land on their legs and come to rest; the
    apply_forces.py push (300 N up + 100 N m yaw at the torso, one frame)
    lifts and spins them."""
    sim, A = _model(gym, 4)
    p, m = sim.mg_params(), sim.mg_model()
    st, dof, pr = A["body_state0"].copy(), A["dof_state0"].copy(), A["dof_props"]
    for _ in range(240):
        oracle.step(p, m, st, dof, props=pr)
    z = st[0::9, 2].copy()
    assert np.all(z > 0.25) and np.all(z < 0.6)
    assert np.all(np.abs(st[0::9, 7:9]) < 0.05)
    for b in range(st.shape[0]):                      # no body below the ground
        assert st[b, 2] > 0.0
    ext = np.zeros((st.shape[0], 6), np.float32)
    ext[0::9, 2] = 300.0
    ext[0::9, 5] = 100.0
    oracle.step(p, m, st, dof, props=pr, ext=ext)
    assert np.all(st[0::9, 9] > 1.0) and np.all(st[0::9, 12] > 1.0)
    for _ in range(10):
        oracle.step(p, m, st, dof, props=pr)
    assert np.all(st[0::9, 2] > z + 0.1)


def _ant_and_box(gym, n=1, gpu=False):
    sp = scenes.ant_sim_params(gpu)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    ant = gym.load_asset(sim, scenes.ASSET_ROOT, "mjcf/ant.xml", gymapi.AssetOptions())
    box = gym.create_box(sim, 0.2, 0.2, 0.2, gymapi.AssetOptions())
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 8)
        gym.create_actor(env, ant, gymapi.Transform(gymapi.Vec3(0, 0, 1)), "ant", i, 0)
        gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0.25 + 0.002 * i, 0, 1.4)), "box", i, 0)
    return sim


def test_floating_base_wide_env(gym):
    """D + 6 (floating base) + 6 per free body above 16 velocity slots: the ant
    (8 DOFs + root) with a free box is 20 slots and steps in the 64-lane coupled
    kernel (mg_env.hip G = 64; the oracle reduces over 64 lanes the same way):
    the box drops onto the ant. More than 32 slots (the humanoid's 27 + a box)
    is refused loudly by the oracle (the library refuses it at upload)."""
    sim = _ant_and_box(gym)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st, ds = A["body_state0"].copy(), A["dof_state0"].copy()
    for _ in range(60):
        oracle.step(p, m, st, ds, props=A["dof_props"])
    assert np.all(np.isfinite(st)) and np.all(np.isfinite(ds))
    assert st[9, 2] < 1.39 and st[9, 2] > 0.05                  # fell, onto the ant or the ground
    sp = scenes.ant_sim_params(False)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    hum = gym.load_asset(sim, scenes.ASSET_ROOT, "mjcf/humanoid.xml", gymapi.AssetOptions())
    box = gym.create_box(sim, 0.2, 0.2, 0.2, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 1)
    gym.create_actor(env, hum, gymapi.Transform(gymapi.Vec3(0, 0, 1.4)), "h", 0, 0)
    gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(1, 0, 0.2)), "box", 0, 0)
    A = sim.build_model()
    with pytest.raises(RuntimeError):
        oracle.step(sim.mg_params(), sim.mg_model(), A["body_state0"].copy(), A["dof_state0"].copy(),
                    props=A["dof_props"])


@pytest.mark.gpu
def test_ant_with_box_wide_parity_gpu(gym):
    """The ant + box envs of test_floating_base_wide_env (64 lanes per env) on
    the GPU, 64 envs x 60 frames: bit for bit the oracle."""
    import torch  # noqa: F401
    n = 64
    sim = _ant_and_box(gym, n, gpu=True)
    gym.prepare_sim(sim)
    from test_isaacgym_amd import _native as N
    assert N.lib.mg_num_coupled_envs(sim.native) == n
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    props = sim.model_arrays["dof_props"]
    for _ in range(60):
        gym.simulate(sim)
        oracle.step(p, m, st, ds, props=props)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    assert np.all(np.isfinite(got))
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


@pytest.mark.gpu
def test_ant_parity_gpu(gym):
    """64 ants with random root orientations / heights / velocities, random DOF
    positions, DOF_MODE_EFFORT with random efforts re-drawn every 20 frames and
    an apply_forces.py-style push every 40 frames: k_env_step (floating base)
    vs the oracle, 160 frames, bit for bit (rigid bodies, DOFs, contact forces)."""
    n, frames = 64, 160
    rng = np.random.RandomState(11)
    sp = scenes.ant_sim_params(True)
    sim, info = scenes.ant_scene(gym, n, sim_params=sp)
    props = gym.get_actor_dof_properties(info["envs"][0], info["actors"][0])
    props["driveMode"].fill(gymapi.DOF_MODE_EFFORT)
    for env, a in zip(info["envs"], info["actors"]):
        gym.set_actor_dof_properties(env, a, props)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    gym.refresh_actor_root_state_tensor(sim)
    r = root.cpu().numpy()
    q = rng.randn(n, 4).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    r[:, 2] = rng.uniform(0.6, 1.4, n)
    r[:, 3:7] = q
    r[:, 7:13] = rng.uniform(-1.0, 1.0, (n, 6))
    root.copy_(torch.from_numpy(r))
    gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
    A = sim.model_arrays
    pr = A["dof_props"].copy()
    lo, hi = pr[:, 5], pr[:, 6]
    d0 = (lo + (hi - lo) * rng.uniform(0.1, 0.9, len(lo))).astype(np.float32)
    ds = np.stack([d0, np.zeros_like(d0)], 1).astype(np.float32)
    dof.copy_(torch.from_numpy(ds))
    gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(dof))
    p, m = sim.mg_params(), sim.mg_model()
    # the oracle starts from the same set state: the library's state after the sets
    gym.refresh_rigid_body_state_tensor(sim)
    st = rb.cpu().numpy().copy()
    dh = ds.copy()
    nb = st.shape[0]
    tgt = np.zeros((len(d0), 3), np.float32)
    for k in range(frames):
        ext = None
        if k % 20 == 0:
            tgt[:, 2] = rng.uniform(-5.0, 5.0, len(d0)).astype(np.float32)
            gym.set_dof_actuation_force_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(tgt[:, 2].copy()).cuda()))
        if k % 40 == 39:
            f = torch.zeros((n, info["num_bodies"], 3), device="cuda")
            t = torch.zeros((n, info["num_bodies"], 3), device="cuda")
            f[:, 0, 2] = 300.0
            t[:, 0, 2] = 100.0
            gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(f), gymtorch.unwrap_tensor(t),
                                               gymapi.ENV_SPACE)
            ext = np.zeros((nb, 6), np.float32)
            ext[0::9, 2] = 300.0
            ext[0::9, 5] = 100.0
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        cf = oracle.step(p, m, st, dh, tgt=tgt, props=pr, ext=ext)
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_net_contact_force_tensor(sim)
    got, gd = rb.cpu().numpy(), dof.cpu().numpy()
    assert np.array_equal(got, st), "rb max |diff| %g" % np.abs(got - st).max()
    assert np.array_equal(gd, dh), "dof max |diff| %g" % np.abs(gd - dh).max()
    assert np.array_equal(ncf.cpu().numpy(), cf)
    assert np.all(np.isfinite(got))
    assert np.abs(gd[:, 1]).max() > 0.1                       # the legs moved


@pytest.mark.gpu
def test_floating_base_jacobian_mass_matrix_float64(gym):
    """acquire_jacobian_tensor / acquire_mass_matrix_tensor of the floating-base
    ant (examples/apply_forces.py:67's nv_ant.xml): (N, 9, 6, 14) and (N, 14, 14),
    the 6 root columns (base-origin linear velocity, then angular velocity) before
    the 8 DOFs, at random root poses and joint angles — against float64 textbook
    kinematics (tests/kinematics64.py: sum of m Jv^T Jv + Jw^T I Jw over link COM
    Jacobians), rtol 1e-4."""
    import kinematics64 as K
    n = 16
    sim, info = scenes.ant_scene(gym, n)
    gym.prepare_sim(sim)
    jac = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, "actor"))
    mm = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, "actor"))
    assert tuple(jac.shape) == (n, 9, 6, 14) and tuple(mm.shape) == (n, 14, 14)
    A = sim.model_arrays
    rng = np.random.RandomState(3)
    props = A["dof_props"][:8]
    lo, hi = props[:, 5], props[:, 6]
    q = (lo + (hi - lo) * rng.uniform(0.1, 0.9, (n, 8))).astype(np.float32)
    ds = torch.zeros((8 * n, 2), dtype=torch.float32, device="cuda:0")
    ds[:, 0] = torch.from_numpy(q.reshape(-1)).cuda()
    gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(ds))
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gym.refresh_actor_root_state_tensor(sim)
    quat = rng.normal(size=(n, 4))
    quat /= np.linalg.norm(quat, axis=1, keepdims=True)
    root[:, 3:7] = torch.from_numpy(quat.astype(np.float32)).cuda()
    root[:, 0:3] += torch.from_numpy(rng.uniform(-0.5, 0.5, (n, 3)).astype(np.float32)).cuda()
    gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
    gym.refresh_jacobian_tensors(sim)
    gym.refresh_mass_matrix_tensors(sim)
    gym.refresh_actor_root_state_tensor(sim)
    art = K.Articulation(A, 0)
    J, M, R = jac.cpu().numpy(), mm.cpu().numpy(), root.cpu().numpy()
    for e in range(n):
        fb = int(A["artic_i"][e, 0])
        base = R[e, 0:7].astype(np.float64)
        Jr = art.jacobian_fb(base, q[e].astype(np.float64))
        Mr = art.mass_matrix_fb(base, q[e].astype(np.float64), fb)
        assert np.allclose(J[e], Jr, rtol=1e-4, atol=1e-5), np.abs(J[e] - Jr).max()
        assert np.allclose(M[e], Mr, rtol=1e-4, atol=1e-4), np.abs(M[e] - Mr).max()
        assert np.allclose(M[e], M[e].T, atol=1e-5)
    gym.destroy_sim(sim)
