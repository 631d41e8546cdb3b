"""Spherical (ball) joints: test13_camera_spherical_joint.py's asset layout
(assets/urdf/dof_spherical_joint_test.urdf: a fixed base, three prismatic
joints through massless-in-URDF links, one spherical joint to a sphere), the
DOF state viewed as (num_envs, 6, 1) (test13 :266-269).

A ball joint's three DOF positions are the rotation vector (exponential
coordinates) of the child joint frame, as test13 feeds its targets
(quat2expcoord, :243-256, :298); its velocities the angular velocity in the
child frame. It is packed as three kernel links about x, y, z (two virtual: no
body, no mass; include/migym.h MG_LINK_I_N), the first turning by exp(th), and
integrated on SO(3): th <- log(exp(th) exp(h w)) — no gimbal lock. CPU tests
check the oracle's physics against the reference's own coordinate conversion,
closed-form and revolute-joint references and the conserved quantities of a
conical swing through 90 degrees (the reference holds no output of a spherical
joint's dynamics: parity with PhysX's integration is unpinned);
`-m gpu` tests check the HIP articulation kernel, the coupled per-env kernel
and the Jacobian / mass-matrix kernel against the oracle and float64
kinematics.
"""
import os

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
import oracle
from kinematics64 import Articulation

G = 9.8


def _urdf(d, name, bob_com=(0.0, 0.0, -0.5), prismatic=True, revolute_axis=None):
    """Fixed base `frame`; optionally tx/ty/tz prismatic links (test13's chain,
    no <inertial>: default 1 kg); then a spherical joint (or, with
    revolute_axis, a revolute joint) to `bob`: 5 kg, COM at bob_com, I = 0.05."""
    links = ['<link name="frame"><inertial><mass value="100"/><inertia ixx="1" iyy="1" izz="1" ixy="0" ixz="0" '
             'iyz="0"/></inertial><collision><geometry><box size="0.4 0.4 0.2"/></geometry></collision></link>']
    joints = []
    parent = "frame"
    if prismatic:
        for ax, n in (("1 0 0", "tx"), ("0 1 0", "ty"), ("0 0 1", "tz")):
            links.append('<link name="%s"/>' % n)
            joints.append('<joint name="p_%s" type="prismatic"><axis xyz="%s"/><origin xyz="%s"/><parent link="%s"/>'
                          '<child link="%s"/><limit effort="1.0" lower="-2" upper="2" velocity="0.1"/></joint>'
                          % (n, ax, "0.5 0 -0.1" if n == "tx" else "0 0 0", parent, n))
            parent = n
    c = " ".join("%g" % x for x in bob_com)
    links.append('<link name="bob"><inertial><origin xyz="%s"/><mass value="5"/><inertia ixx="0.05" iyy="0.05" '
                 'izz="0.05" ixy="0" ixz="0" iyz="0"/></inertial><collision><origin xyz="%s"/><geometry>'
                 '<sphere radius="0.1"/></geometry></collision></link>' % (c, c))
    if revolute_axis is None:
        joints.append('<joint name="ball" type="spherical"><origin xyz="0 0 0"/><parent link="%s"/><child link="bob"/>'
                      '<limit effort="1000.0" lower="-4" upper="4" velocity="100"/></joint>' % parent)
    else:
        joints.append('<joint name="hinge" type="continuous"><axis xyz="%s"/><origin xyz="0 0 0"/><parent link="%s"/>'
                      '<child link="bob"/></joint>' % (revolute_axis, parent))
    with open(os.path.join(d, name), "w") as f:
        f.write('<robot name="ball_test">' + "".join(links + joints) + "</robot>")
    return name


def _sim(gym, gravity=-G, gpu=False, dt=1.0 / 60.0, substeps=2):
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0, 0, gravity)
    sp.dt, sp.substeps = dt, substeps
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 6
    sp.physx.num_velocity_iterations = 0
    sp.use_gpu_pipeline = gpu
    return gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)


def _scene(gym, d, n, urdf, gravity=-G, gpu=False, init=None, drive=None):
    sim = _sim(gym, gravity, gpu)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    asset = gym.load_asset(sim, d, urdf, opts)
    nd = gym.get_asset_dof_count(asset)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 2), 8)
        h = gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 1.5)), "ball", i, 1)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_NONE
        if drive is not None:
            props["driveMode"][:] = gymapi.DOF_MODE_POS
            props["stiffness"][:] = drive[0]
            props["damping"][:] = drive[1]
        gym.set_actor_dof_properties(env, h, props)
        if init is not None:
            st = np.zeros(nd, dtype=gymapi.DofState.dtype)
            st["pos"] = init(i)[0]
            st["vel"] = init(i)[1]
            gym.set_actor_dof_states(env, h, st, gymapi.STATE_ALL)
    return sim, asset


def _run(sim, frames):
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    traj = []
    for _ in range(frames):
        oracle.step(p, m, st, dof)
        traj.append(st.copy())
    return st, dof, traj


def _qrot(q, v):
    x, y, z, w = q
    u = np.array([x, y, z])
    return v + 2.0 * np.cross(u, np.cross(u, v) + w * v)


# ------------------------------------------------------------------ CPU (oracle)
def test_layout_and_names(gym, tmp_path):
    sim, asset = _scene(gym, str(tmp_path), 2, _urdf(str(tmp_path), "b.urdf"))
    assert gym.get_asset_dof_count(asset) == 6 and gym.get_asset_rigid_body_count(asset) == 5
    assert gym.get_asset_dof_names(asset) == ["p_tx", "p_ty", "p_tz", "ball_0", "ball_1", "ball_2"]
    assert gym.get_asset_joint_type(asset, 3) == gymapi.JOINT_BALL
    A = sim.build_model()
    assert A["body_state0"].shape[0] == 10 and A["dof_state0"].shape[0] == 12
    li = A["tmpl_link_i"]
    assert li.tolist() == [[-1, 0, -1, 0], [0, 2, 0, 1], [1, 2, 1, 2], [2, 2, 2, 3],
                           [3, 1, 3, -1], [4, 1, 4, -1], [5, 1, 5, 4]]
    assert A["tmpl_link_f"][4:7, 7:10].tolist() == np.eye(3).tolist()


def test_mjcf_ball_joint(gym, tmp_path):
    """MJCF <joint type="ball"> (assets/mjcf/spherical_joint.xml is test13's
    commented-out alternative, :39): three rotation DOFs, the same packing."""
    xml = ('<mujoco><worldbody><body name="base" pos="0 0 1"><geom type="box" size="0.1 0.1 0.1"/>'
           '<body name="bob" pos="0 0 -0.2"><joint name="sph" type="ball" range="0 90"/>'
           '<geom type="sphere" size="0.05" pos="0 0 -0.3"/></body></body></worldbody></mujoco>')
    with open(os.path.join(str(tmp_path), "b.xml"), "w") as f:
        f.write(xml)
    sim = _sim(gym)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    asset = gym.load_asset(sim, str(tmp_path), "b.xml", opts)
    assert gym.get_asset_dof_count(asset) == 3
    assert gym.get_asset_dof_names(asset) == ["sph_0", "sph_1", "sph_2"]
    assert not gym.get_asset_dof_properties(asset)["hasLimits"].any()
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 2), 1)
    gym.create_actor(env, asset, gymapi.Transform(), "b", 0, 1)
    A = sim.build_model()
    assert A["tmpl_link_i"][:, 3].tolist() == [0, -1, -1, 1]


def _quat2expcoord(q):
    """test13_camera_spherical_joint.py:243-256 (the reference's own conversion of
    a goal orientation into the spherical joint's DOF targets), restated."""
    q = np.asarray(q, np.float64)
    if q[-1] < 0:
        q = -q
    theta = 2.0 * np.arctan2(np.linalg.norm(q[:-1]), q[-1])
    return q[:-1] / (np.sin(theta / 2.0) + 1e-7) * theta


def test_dof_positions_are_exponential_coordinates(gym, tmp_path):
    """test13 drives its spherical joint with dof_positions[3:] =
    quat2expcoord(goal_quat) (:298): a ball joint set to those positions holds
    the bob at goal_quat relative to the joint frame — at the host's initial
    forward kinematics and after a step of the engine (no gravity, no drive) —
    including rotations by more than 90 degrees about tilted axes."""
    d = str(tmp_path)
    rng = np.random.RandomState(4)
    quats = []
    for _ in range(6):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        ang = rng.uniform(0.3, 3.0)
        quats.append(np.array([*(ax * np.sin(0.5 * ang)), np.cos(0.5 * ang)]))
    sim, _ = _scene(gym, d, len(quats), _urdf(d, "b.urdf"), gravity=0.0,
                    init=lambda i: (np.r_[0.0, 0.0, 0.0, _quat2expcoord(quats[i])], np.zeros(6)))
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st, dof = A["body_state0"].copy(), A["dof_state0"].copy()
    oracle.step(p, m, st, dof)
    for i, q in enumerate(quats):
        for s in (A["body_state0"], st):
            got = s[5 * i + 4, 3:7].astype(np.float64)          # the bob (fixed frame is identity)
            assert min(np.abs(got - q).max(), np.abs(got + q).max()) < 2e-6
        assert np.abs(dof[6 * i + 3:6 * i + 6, 0] - _quat2expcoord(q)).max() < 2e-5


def test_rest_without_gravity_is_static(gym, tmp_path):
    """test13's setting (gravity 0, no drives): nothing moves, bit for bit."""
    sim, _ = _scene(gym, str(tmp_path), 2, _urdf(str(tmp_path), "b.urdf", bob_com=(0, 0, 0)), gravity=0.0)
    A = sim.build_model()
    st, dof, _ = _run(sim, 30)
    assert np.array_equal(dof, A["dof_state0"])
    assert np.array_equal(st[:, 0:7], A["body_state0"][:, 0:7])
    assert not st[:, 7:].any()


def test_planar_swing_matches_revolute(gym, tmp_path):
    """Started rotated about the joint frame's x only, the ball-joint pendulum
    swings in the y-z plane like a revolute-x pendulum (the two virtual links'
    rotations stay 0 up to rounding)."""
    d = str(tmp_path)
    th0 = 0.7
    sb, _ = _scene(gym, d, 1, _urdf(d, "b.urdf", prismatic=False), init=lambda i: ([th0, 0, 0], [0, 0, 0]))
    sr, _ = _scene(gym, d, 1, _urdf(d, "r.urdf", prismatic=False, revolute_axis="1 0 0"),
                   init=lambda i: ([th0], [0]))
    stb, dofb, tb = _run(sb, 120)
    str_, dofr, tr = _run(sr, 120)
    for a, b in zip(tb, tr):
        assert np.abs(a[1, 0:7] - b[1, 0:7]).max() < 2e-5
    assert abs(dofb[0, 0] - dofr[0, 0]) < 2e-5 and np.abs(dofb[1:, :]).max() < 1e-5
    assert abs(dofr[0, 0] - th0) > 0.1                                  # it swung


def _conical(gym, d, substeps, frames=240, tilt=0.6, rate=2.0):
    """Tilt about x, angular velocity `rate` about the child frame's y (the joint
    frame's y turned by the tilt: perpendicular to the pivot-COM line, so the
    bob moves azimuthally). Returns (max |r - r0|, Lz(end) / Lz(start), energy
    drift)."""
    sim = _sim(gym, substeps=substeps)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    asset = gym.load_asset(sim, d, _urdf(d, "b.urdf", prismatic=False), opts)
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 2), 8)
    h = gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 1.5)), "ball", 0, 1)
    props = gym.get_actor_dof_properties(env, h)
    props["driveMode"][:] = gymapi.DOF_MODE_NONE
    gym.set_actor_dof_properties(env, h, props)
    s0 = np.zeros(3, dtype=gymapi.DofState.dtype)
    s0["pos"], s0["vel"] = [tilt, 0, 0], [0, rate, 0]
    gym.set_actor_dof_states(env, h, s0, gymapi.STATE_ALL)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st, dof = A["body_state0"].copy(), A["dof_state0"].copy()
    pivot = st[0, 0:3].copy()

    def com(s):
        return s[1, 0:3] + _qrot(s[1, 3:7], np.array([0, 0, -0.5]))

    def lz(s):          # angular momentum about the vertical through the pivot
        return 5.0 * np.cross(com(s) - pivot, s[1, 7:10])[2] + 0.05 * s[1, 12]

    def energy(s):
        return 2.5 * s[1, 7:10] @ s[1, 7:10] + 0.025 * s[1, 10:13] @ s[1, 10:13] + 5.0 * G * com(s)[2]

    oracle.step(p, m, st, dof)
    l0, e0, r0 = lz(st), energy(st), np.linalg.norm(com(st) - pivot)
    dr = 0.0
    for _ in range(frames):
        oracle.step(p, m, st, dof)
        dr = max(dr, abs(np.linalg.norm(com(st) - pivot) - r0))
    assert np.all(np.isfinite(st)) and np.all(np.isfinite(dof)) and abs(l0) > 1.0
    return dr, lz(st) / l0, energy(st) - e0


def test_spherical_pendulum_invariants(gym, tmp_path):
    """A conical swing: the bob stays on its sphere (the joint holds exactly),
    and the vertical angular momentum and the energy — conserved by the
    continuous dynamics — are kept: the joint is integrated on SO(3) in
    exponential coordinates (th <- log(exp(th) exp(h w))), and the three axes'
    velocity product is the ball's v_parent x vJ."""
    d = str(tmp_path)
    for ss in (8, 32):
        dr, lz, de = _conical(gym, d, ss)
        assert dr < 1e-5
        assert abs(lz - 1.0) < 1e-3 and abs(de) < 0.01      # 25 J of potential energy at the pivot depth


@pytest.mark.parametrize("tilt", [1.4, 1.6, 2.2])
def test_conical_swing_through_ninety_degrees(gym, tmp_path, tilt):
    """Swings whose orientation passes and stays beyond 90 degrees from the rest
    direction (1.6 and 2.2 rad of tilt: the bob above the pivot's horizontal),
    where a triple-revolute (x-y-z) packing meets gimbal lock: the same
    invariants hold."""
    d = str(tmp_path)
    dr, lz, de = _conical(gym, d, 16, frames=180, tilt=tilt, rate=4.0)
    assert dr < 5e-5
    assert abs(lz - 1.0) < 2e-3 and abs(de) < 0.05


def _coupled_scene(gym, d, n, gpu=False, seed=0):
    """A ball-joint pendulum (tilted, swinging) over a free box resting on a
    static slab in the same collision group: the env steps in the coupled per-env
    kernel, whose links now include the ball joint's two virtual links."""
    sim = _sim(gym, gpu=gpu)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    asset = gym.load_asset(sim, d, _urdf(d, "b.urdf", prismatic=False), opts)
    box = gym.create_box(sim, 0.3, 0.3, 0.2, gymapi.AssetOptions())
    fixed = gymapi.AssetOptions()
    fixed.fix_base_link = True
    slab = gym.create_box(sim, 1.0, 1.0, 0.1, fixed)
    rng = np.random.RandomState(seed)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 2), 8)
        h = gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 1.4)), "ball", i, 0)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_NONE
        gym.set_actor_dof_properties(env, h, props)
        st = np.zeros(3, dtype=gymapi.DofState.dtype)
        st["pos"] = [0.9 + rng.uniform(-0.05, 0.05), rng.uniform(-0.1, 0.1), 0.0]
        gym.set_actor_dof_states(env, h, st, gymapi.STATE_ALL)
        gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0, 0.05 * rng.uniform(-1, 1), 0.75)), "box", i, 0)
        gym.create_actor(env, slab, gymapi.Transform(gymapi.Vec3(0, 0, 0.6)), "slab", i, 0)
    return sim


def test_coupled_step_ball_joint(gym, tmp_path):
    """The bob (5 kg, 0.5 m below the pivot) swings down onto the box (18 kg)
    on the slab: the coupled step, with the ball joint's virtual links, stops it
    on the box (without the box it swings through to the other side) while the
    slab holds the box up and the bob stays on its sphere."""
    sim = _coupled_scene(gym, str(tmp_path), 1)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st, dof = A["body_state0"].copy(), A["dof_state0"].copy()
    box0 = st[2, 0:3].copy()
    pivot = st[0, 0:3].copy()
    for _ in range(90):
        oracle.step(p, m, st, dof)
        com = st[1, 0:3] + _qrot(st[1, 3:7], np.array([0.0, 0.0, -0.5]))
        assert abs(np.linalg.norm(com - pivot) - 0.5) < 1e-4
    assert np.all(np.isfinite(st)) and np.all(np.isfinite(dof))
    assert dof[0, 0] > 0.3                                          # caught by the box, not swung through
    assert abs(st[2, 2] - box0[2]) < 0.02                           # the slab holds the box
    assert np.linalg.norm(st[2, 0:2] - box0[0:2]) < 0.05


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_ball_joint_parity_gpu(gym, tmp_path):
    """test13's chain (3 prismatic + spherical) under gravity with stiff POS
    drives on random targets: k_artic_lanes bit for bit the oracle, DOF state
    viewed as (num_envs, 6, 1)."""
    d = str(tmp_path)
    n, steps = 64, 40
    rng0 = np.random.RandomState(3)
    init = rng0.uniform(-0.5, 0.5, size=(n, 6)).astype(np.float32)
    sim, _ = _scene(gym, d, n, _urdf(d, "b.urdf"), gpu=True, drive=(400.0, 20.0),
                    init=lambda i: (init[i], np.zeros(6)))
    gym.prepare_sim(sim)
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    assert tuple(dof[:, 0].view(n, 6, 1).shape) == (n, 6, 1) and tuple(rb.shape) == (5 * n, 13)
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    rng = np.random.RandomState(5)
    for _ in range(steps):
        tgt[:, 0] = rng.uniform(-1.0, 1.0, size=ds.shape[0]).astype(np.float32)
        assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(tgt[:, 0].copy()).to("cuda:0")))
        gym.simulate(sim)
        oracle.step(p, m, st, ds, tgt=tgt)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    assert np.all(np.isfinite(got_d)) and np.abs(got_d[:, 1]).max() > 0.1
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


@pytest.mark.gpu
def test_ball_joint_jacobian_mass_matrix_gpu(gym, tmp_path):
    """Jacobian (N, 4, 6, 6): rows for the 4 moving bodies only (the virtual
    links have none); mass matrix (N, 6, 6); against float64 kinematics."""
    d = str(tmp_path)
    n = 16
    rng = np.random.RandomState(9)
    init = rng.uniform(-1.0, 1.0, size=(n, 6)).astype(np.float32)
    sim, asset = _scene(gym, d, n, _urdf(d, "b.urdf"), gpu=True, init=lambda i: (init[i], np.zeros(6)))
    gym.prepare_sim(sim)
    jac = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, "ball"))
    mm = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, "ball"))
    gym.refresh_jacobian_tensors(sim)
    gym.refresh_mass_matrix_tensors(sim)
    assert tuple(jac.shape) == (n, 4, 6, 6) and tuple(mm.shape) == (n, 6, 6)
    A = sim.model_arrays
    art = Articulation(A, 0)
    J, M = jac.cpu().numpy(), mm.cpu().numpy()
    for i in range(n):
        b0 = i * 5
        base = A["body_state0"][b0].astype(np.float64)
        q = A["dof_state0"][i * 6:(i + 1) * 6, 0].astype(np.float64)
        assert np.abs(J[i] - art.jacobian(base, q)).max() < 1e-4
        assert np.abs(M[i] - art.mass_matrix(base, q, b0)).max() < 1e-3 * max(1.0, np.abs(M[i]).max())


@pytest.mark.gpu
def test_coupled_ball_joint_parity_gpu(gym, tmp_path):
    """The coupled scene above, 64 envs: k_env_step bit for bit the oracle."""
    n, steps = 64, 60
    sim = _coupled_scene(gym, str(tmp_path), n, gpu=True, seed=2)
    gym.prepare_sim(sim)
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
    assert np.all(np.isfinite(got))
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
