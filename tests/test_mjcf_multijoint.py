"""MJCF bodies with several joints:
assets/mjcf/nv_humanoid.xml:53-54 (abdomen_z + abdomen_y on lower_waist) and
:61-63 (three hips on each thigh), the default asset of examples/joint_monkey.py:35.

A body hanging by k hinges is k kernel links: k - 1 virtual (no body, no mass)
and the body's own, each hinge about its axis in the body frame as turned by
the hinges before it (MuJoCo's order), sharing one anchor — the same packing as
a ball joint's three rotations (include/migym.h MG_LINK_I_N).

CPU: the importer's counts, names, efforts and link packing against the
reference file; a two-hinge body steps exactly like the same chain written as a
URDF with a massless link between two revolute joints. GPU: k_artic_lanes and
k_env_step (the two-hinge arm swinging onto a box) bit for bit the oracle."""
import os

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
import oracle
from conftest import REFERENCE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HUMANOID_DOFS = ["abdomen_z", "abdomen_y", "abdomen_x", "right_hip_x", "right_hip_z", "right_hip_y", "right_knee",
                 "right_ankle_y", "right_ankle_x", "left_hip_x", "left_hip_z", "left_hip_y", "left_knee",
                 "left_ankle_y", "left_ankle_x", "right_shoulder1", "right_shoulder2", "right_elbow",
                 "left_shoulder1", "left_shoulder2", "left_elbow"]


def _sim(gym, gpu=False, gravity=-9.8):
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0, 0, gravity)
    sp.dt, sp.substeps = 1.0 / 60.0, 2
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 6
    sp.physx.num_velocity_iterations = 1
    sp.use_gpu_pipeline = gpu
    return gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)


def _humanoid(gym, root):
    sim = _sim(gym)
    a = gym.load_asset(sim, root, "mjcf/" + ("nv_humanoid.xml" if root != os.path.join(ROOT, "assets")
                                             else "humanoid.xml"), gymapi.AssetOptions())
    return sim, a


@pytest.mark.parametrize("where", ["repo", "reference"])
def test_nv_humanoid_loads(gym, where):
    root = os.path.join(ROOT, "assets") if where == "repo" else os.path.join(REFERENCE, "assets")
    if where == "reference" and not os.path.exists(os.path.join(root, "mjcf", "nv_humanoid.xml")):
        pytest.skip("reference tree absent")
    sim, a = _humanoid(gym, root)
    assert a is not None
    assert gym.get_asset_rigid_body_count(a) == 16 and gym.get_asset_dof_count(a) == 21
    assert gym.get_asset_dof_names(a) == HUMANOID_DOFS
    names = gym.get_asset_joint_names(a)
    assert "abdomen_z" in names and "abdomen_y" in names and names.index("abdomen_z") + 1 == names.index("abdomen_y")
    props = gym.get_asset_dof_properties(a)
    # motor gear x the <default><motor ctrlrange="-1 1"> (nv_humanoid.xml:8, :141-161)
    assert props["effort"][HUMANOID_DOFS.index("abdomen_y")] == pytest.approx(67.5)
    assert props["effort"][HUMANOID_DOFS.index("right_hip_y")] == pytest.approx(135.0)
    assert props["effort"][HUMANOID_DOFS.index("right_knee")] == pytest.approx(90.0)
    assert props["lower"][0] == pytest.approx(np.radians(-45)) and props["upper"][1] == pytest.approx(np.radians(30))
    assert props["armature"][0] == pytest.approx(0.02)          # big_stiff_joint class
    env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 1)
    gym.create_actor(env, a, gymapi.Transform(gymapi.Vec3(0, 0, 1.4)), "h", 0, 0)
    A = sim.build_model()
    li = A["tmpl_link_i"]
    # 16 bodies + 9 virtual links: abdomen 1, hips 2 + 2, ankles 1 + 1, shoulders 1 + 1
    assert li.shape[0] == 25 and int((li[:, 3] < 0).sum()) == 9
    assert sorted(li[li[:, 3] >= 0, 3].tolist()) == list(range(16))


def _two_hinge_mjcf(d):
    xml = ('<mujoco><worldbody><body name="base" pos="0 0 1.2"><geom type="box" size="0.05 0.05 0.05"/>'
           '<body name="arm" pos="0 0 -0.05"><joint name="hz" type="hinge" axis="0 0 1" pos="0 0 0"/>'
           '<joint name="hy" type="hinge" axis="0 1 0" pos="0 0 0"/>'
           '<inertial pos="0.3 0 -0.2" mass="2" diaginertia="0.02 0.03 0.04"/>'
           '<geom type="sphere" size="0.08" pos="0.3 0 -0.2" density="0"/></body></body></worldbody></mujoco>')
    with open(os.path.join(d, "two.xml"), "w") as f:
        f.write(xml)
    return "two.xml"


def _two_hinge_urdf(d):
    """The same chain as a URDF: a massless link between two revolute joints."""
    urdf = ('<robot name="two"><link name="base"><inertial><mass value="1"/><inertia ixx="0.01" iyy="0.01" '
            'izz="0.01" ixy="0" ixz="0" iyz="0"/></inertial><collision><geometry><box size="0.1 0.1 0.1"/>'
            '</geometry></collision></link>'
            '<link name="mid"><inertial><mass value="0"/><inertia ixx="0" iyy="0" izz="0" ixy="0" ixz="0" '
            'iyz="0"/></inertial></link>'
            '<link name="arm"><inertial><origin xyz="0.3 0 -0.2"/><mass value="2"/><inertia ixx="0.02" iyy="0.03" '
            'izz="0.04" ixy="0" ixz="0" iyz="0"/></inertial><collision><origin xyz="0.3 0 -0.2"/><geometry>'
            '<sphere radius="0.08"/></geometry></collision></link>'
            '<joint name="hz" type="continuous"><origin xyz="0 0 -0.05"/><axis xyz="0 0 1"/><parent link="base"/>'
            '<child link="mid"/></joint>'
            '<joint name="hy" type="continuous"><axis xyz="0 1 0"/><parent link="mid"/><child link="arm"/></joint>'
            '</robot>')
    with open(os.path.join(d, "two.urdf"), "w") as f:
        f.write(urdf)
    return "two.urdf"


def _arm_scene(gym, d, fname, n=1, gpu=False, box=False):
    sim = _sim(gym, gpu=gpu)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    asset = gym.load_asset(sim, d, fname, opts)
    cube = gym.create_box(sim, 0.2, 0.2, 0.2, gymapi.AssetOptions()) if box else None
    fixed = gymapi.AssetOptions()
    fixed.fix_base_link = True
    slab = gym.create_box(sim, 1.2, 1.2, 0.1, fixed) if box else None
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 2), 8)
        h = gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 0)), "arm", i, 0)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_NONE
        gym.set_actor_dof_properties(env, h, props)
        st = np.zeros(2, dtype=gymapi.DofState.dtype)
        st["pos"] = [0.4 + 0.01 * i, -0.3]
        st["vel"] = [1.5, 0.0]
        gym.set_actor_dof_states(env, h, st, gymapi.STATE_ALL)
        if box:
            gym.create_actor(env, cube, gymapi.Transform(gymapi.Vec3(0.25, 0.25, 0.7)), "cube", i, 0)
            gym.create_actor(env, slab, gymapi.Transform(gymapi.Vec3(0, 0, 0.55)), "slab", i, 0)
    return sim, asset


def test_two_hinge_body_matches_urdf_chain(gym, tmp_path):
    d = str(tmp_path)
    sm, am = _arm_scene(gym, d, _two_hinge_mjcf(d))
    su, au = _arm_scene(gym, d, _two_hinge_urdf(d))
    assert gym.get_asset_rigid_body_count(am) == 2 and gym.get_asset_rigid_body_count(au) == 3
    assert gym.get_asset_dof_names(am) == ["hz", "hy"] == gym.get_asset_dof_names(au)
    A, B = sm.build_model(), su.build_model()
    assert A["tmpl_link_i"][:, 3].tolist() == [0, -1, 1]
    pm, mm_ = sm.mg_params(), sm.mg_model()
    pu, mu = su.mg_params(), su.mg_model()
    sa, da = A["body_state0"].copy(), A["dof_state0"].copy()
    sb, db = B["body_state0"].copy(), B["dof_state0"].copy()
    assert np.allclose(sa[1], sb[2], atol=1e-6)              # same initial pose of the arm
    for _ in range(120):
        oracle.step(pm, mm_, sa, da)
        oracle.step(pu, mu, sb, db)
    assert np.abs(da - db).max() < 1e-4
    assert np.abs(sa[1] - sb[2]).max() < 1e-4
    assert abs(da[0, 0] - 0.4) > 0.5                          # it moved


@pytest.mark.gpu
@pytest.mark.parametrize("box", [False, True])
def test_two_hinge_parity_gpu(gym, tmp_path, box):
    """box=False: k_artic_lanes; box=True: the arm swings onto a cube on a slab
    (coupled per-env step with a virtual link)."""
    d = str(tmp_path)
    n, steps = 64, 60
    sim, _ = _arm_scene(gym, d, _two_hinge_mjcf(d), n=n, gpu=True, box=box)
    gym.prepare_sim(sim)
    from test_isaacgym_amd import _native as N
    assert (N.lib.mg_num_coupled_envs(sim.native) > 0) == box
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    for _ in range(steps):
        gym.simulate(sim)
        oracle.step(p, m, st, ds)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    assert np.all(np.isfinite(got)) and np.abs(got_d[:, 1]).max() > 0.1
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
    torch.cuda.synchronize()


def _humanoid_drop(gym, n=1, gpu=False):
    from test_isaacgym_amd import scenes
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, scenes.ant_sim_params(gpu))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    hum = gym.load_asset(sim, os.path.join(ROOT, "assets"), "mjcf/humanoid.xml", gymapi.AssetOptions())
    rng = np.random.RandomState(1)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 8)
        q = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 0, 1), float(rng.uniform(-3, 3)))
        gym.create_actor(env, hum, gymapi.Transform(gymapi.Vec3(0, 0, 1.3 + 0.05 * rng.uniform()), q), "h", i, 0)
    return sim


def test_humanoid_drop_settles(gym):
    """nv_humanoid (floating base, 21 DOFs in 25 kernel links: 27 velocity slots,
    the 64-lane coupled kernel) dropped on the ground: it falls, lands and stays
    above the ground, its state finite."""
    sim = _humanoid_drop(gym)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st, ds = A["body_state0"].copy(), A["dof_state0"].copy()
    z0 = float(st[0, 2])
    for _ in range(120):
        oracle.step(p, m, st, ds, props=A["dof_props"])
    assert np.all(np.isfinite(st)) and np.all(np.isfinite(ds))
    assert float(st[0, 2]) < z0 - 0.2                      # it fell
    assert float(st[:, 2].min()) > -0.05                    # nothing through the ground
    assert np.abs(st[:, 7:10]).max() < 5.0                  # and it is not flying apart


@pytest.mark.gpu
def test_humanoid_drop_parity_gpu(gym):
    """64 humanoids dropped on the ground, 60 frames: k_env_step<32, 64> bit for
    bit the oracle (rigid-body and DOF state)."""
    n = 64
    sim = _humanoid_drop(gym, n, gpu=True)
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
    assert np.all(np.isfinite(got)) and float(got[:, 2].min()) > -0.05
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


@pytest.mark.gpu
def test_fixed_humanoid_pd_parity_gpu(gym):
    """joint_monkey's setting (examples/joint_monkey.py:95-96: fix_base_link):
    32 fixed-base humanoids under gravity with PD drives on random targets —
    k_artic_lanes<32, 64> (25 links, 21 DOFs: one articulation per wavefront)
    bit for bit the oracle."""
    n = 32
    sim = _sim(gym, gpu=True)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    hum = gym.load_asset(sim, os.path.join(ROOT, "assets"), "mjcf/humanoid.xml", opts)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 8)
        h = gym.create_actor(env, hum, gymapi.Transform(gymapi.Vec3(0, 0, 1.5)), "h", i, 1)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_POS
        props["stiffness"][:] = 200.0
        props["damping"][:] = 10.0
        gym.set_actor_dof_properties(env, h, props)
    gym.prepare_sim(sim)
    from test_isaacgym_amd import _native as N
    assert N.lib.mg_num_coupled_envs(sim.native) == 0
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    props = sim.model_arrays["dof_props"]
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    rng = np.random.RandomState(2)
    for _ in range(40):
        tgt[:, 0] = rng.uniform(-0.6, 0.6, size=ds.shape[0]).astype(np.float32)
        assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(
            torch.from_numpy(tgt[:, 0].copy()).to("cuda:0")))
        gym.simulate(sim)
        oracle.step(p, m, st, ds, tgt=tgt, props=props)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    assert np.all(np.isfinite(got)) and np.abs(got_d[:, 1]).max() > 0.1
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


@pytest.mark.gpu
def test_humanoid_jacobian_mass_matrix_float64(gym):
    """acquire_jacobian_tensor / acquire_mass_matrix_tensor of nv_humanoid
    (floating base, 21 DOFs in 25 kernel links: more than 16 links and
    generalized velocities, the 32-lane k_artic_jac_mm_g<32>):
    (N, 16, 6, 27) and (N, 27, 27) at random root poses and joint angles against
    float64 textbook kinematics (tests/kinematics64.py), rtol 1e-4."""
    import kinematics64 as K
    n = 8
    sim = _humanoid_drop(gym, n, gpu=True)
    gym.prepare_sim(sim)
    jac = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, "h"))
    mm = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, "h"))
    assert tuple(jac.shape) == (n, 16, 6, 27) and tuple(mm.shape) == (n, 27, 27)
    A = sim.model_arrays
    rng = np.random.RandomState(4)
    props = A["dof_props"][:21]
    lo, hi = props[:, 5], props[:, 6]
    q = (lo + (hi - lo) * rng.uniform(0.1, 0.9, (n, 21))).astype(np.float32)
    ds = torch.zeros((21 * n, 2), dtype=torch.float32, device="cuda:0")
    ds[:, 0] = torch.from_numpy(q.reshape(-1)).cuda()
    gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(ds))
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gym.refresh_actor_root_state_tensor(sim)
    quat = rng.normal(size=(n, 4))
    quat /= np.linalg.norm(quat, axis=1, keepdims=True)
    root[:, 3:7] = torch.from_numpy(quat.astype(np.float32)).cuda()
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
