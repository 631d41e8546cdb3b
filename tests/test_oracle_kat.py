"""Analytic known-answer tests for the C restatement (oracle/) — what pins the
step algorithm to physics, since parity with PhysX itself is unpinned
(SURVEY.md §8c). The GPU kernels are pinned to this oracle bit for bit by
tests/test_parity_gpu.py, so these KATs transfer to the device.

Tolerances are stated per test; positions in metres, velocities in m/s."""
import os
import tempfile

import math

import numpy as np
import pytest

from isaacgym import gymapi
import oracle


def _sim(gym, gravity=(0, 0, -9.8), npos=6, nvel=1, substeps=2, dt=1 / 60, ground=True, mu=1.0, e=0.0,
         contact_offset=0.01, rest_offset=0.0):
    sp = gymapi.SimParams()
    sp.dt = dt
    sp.substeps = substeps
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(*gravity)
    sp.physx.num_position_iterations = npos
    sp.physx.num_velocity_iterations = nvel
    sp.physx.contact_offset = contact_offset
    sp.physx.rest_offset = rest_offset
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    if ground:
        pp = gymapi.PlaneParams()
        pp.normal = gymapi.Vec3(0, 0, 1)
        pp.static_friction = mu
        pp.dynamic_friction = mu
        pp.restitution = e
        gym.add_ground(sim, pp)
    return sim


def _one(gym, sim, asset, pose):
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    gym.create_actor(env, asset, pose, "a", 0, 0)
    sim.build_model()
    return sim.mg_params(), sim.mg_model(), sim.model_arrays["body_state0"].copy()


def _run(p, m, st, steps, dof=None, tgt=None):
    dof = np.zeros((0, 2), np.float32) if dof is None else dof
    cf = None
    for _ in range(steps):
        cf = oracle.step(p, m, st, dof, tgt=tgt)
    return cf


def test_free_fall_semi_implicit_euler(gym):
    """No contacts: n = frames x substeps semi-implicit Euler steps of h,
    v = n g h, z = z0 + g h^2 n (n + 1) / 2 (float64 closed form), rtol 1e-5."""
    sim = _sim(gym, ground=False)
    opts = gymapi.AssetOptions()
    opts.angular_damping = 0.0
    p, m, st = _one(gym, sim, gym.create_box(sim, 1, 1, 1, opts), gymapi.Transform(gymapi.Vec3(0, 0, 100)))
    _run(p, m, st, 60)
    n, h = 120, (1 / 60) / 2
    np.testing.assert_allclose(st[0, 9], -9.8 * n * h, rtol=1e-5)
    np.testing.assert_allclose(st[0, 2], 100 - 9.8 * h * h * n * (n + 1) / 2, rtol=1e-5)
    assert np.all(st[0, [0, 1, 7, 8, 10, 11, 12]] == 0)


def test_resting_box_contact_force(gym):
    """A 1 m box (1000 kg) dropped flat from 0.1 m settles on its face:
    z = 0.5 +- 1e-3, the pose static (< 1 um over the last 100 frames), net
    contact force = m g within 0.1 %. The state's velocity is the last
    velocity sweep's Gauss-Seidel residual: |v|, |w| < 2e-3
    (1.07e-3 with round 6's sweep order, 2e-4 with round 5's, whose position
    sweeps let a pushed body creep: tests/test_ground_patch_kat.py)."""
    sim = _sim(gym)
    p, m, st = _one(gym, sim, gym.create_box(sim, 1, 1, 1, gymapi.AssetOptions()),
                    gymapi.Transform(gymapi.Vec3(0, 0, 0.6)))
    _run(p, m, st, 140)
    pose = st[0, :7].copy()
    cf = _run(p, m, st, 100)
    assert abs(st[0, 2] - 0.5) < 1e-3
    assert np.all(np.abs(st[0, :7] - pose) < 1e-6), st[0, :7] - pose
    assert np.all(np.abs(st[0, 7:13]) < 2e-3)
    np.testing.assert_allclose(cf[0], [0, 0, 1000 * 9.8], rtol=1e-3, atol=1.0)


def test_sliding_box_friction(gym):
    """Box resting on the ground, launched at v0 = 3 m/s along x: Coulomb
    friction (mu = 0.5 * (0.5 + 0.5) = 0.5; a 1 m cube at mu = 1 sits on its
    tipping threshold and pitches onto its leading edge while sliding)
    decelerates it at mu g through the ground patch's two anchors (DESIGN.md
    §3.2.1); it stops after v0 / (mu g) s having slid v0^2 / (2 mu g) m (within
    5 %), drifting < 5 mm sideways and turning < 0.5 degrees (the anchors lie on
    a diagonal of the bottom face and share the patch's budget evenly when both
    slide, so the friction exerts no yaw torque)."""
    mu = 0.5
    sim = _sim(gym, mu=mu)
    box = gym.create_box(sim, 1, 1, 1, gymapi.AssetOptions())
    for sp in box.shape_props:
        sp.friction = mu
    p, m, st = _one(gym, sim, box, gymapi.Transform(gymapi.Vec3(0, 0, 0.5)))
    _run(p, m, st, 30)
    x0 = st[0, 0]
    st[0, 7] = 3.0
    t_stop = None
    for k in range(120):
        _run(p, m, st, 1)
        if t_stop is None and st[0, 7] < 1e-3:
            t_stop = (k + 1) / 60
    assert t_stop is not None
    assert abs(t_stop - 3.0 / (mu * 9.8)) < 0.05 * 3.0 / (mu * 9.8) + 1 / 60
    np.testing.assert_allclose(st[0, 0] - x0, 9.0 / (2 * mu * 9.8), rtol=0.05)
    assert abs(st[0, 1]) < 5e-3
    yaw = 2.0 * math.degrees(math.asin(min(1.0, abs(float(st[0, 5])))))
    assert yaw < 0.5, yaw


def test_restitution_bounce(gym):
    """Sphere (restitution 0.5 with a 0.5 plane: combined 0.5) hits the ground
    at ~6.3 m/s and leaves at about half that speed (within 15 %)."""
    sim = _sim(gym, e=0.5)
    a = gym.create_sphere(sim, 0.2, gymapi.AssetOptions())
    a.shape_props[0].restitution = 0.5
    p, m, st = _one(gym, sim, a, gymapi.Transform(gymapi.Vec3(0, 0, 2.2)))
    vmin, vmax_after = 0.0, 0.0
    for _ in range(90):
        _run(p, m, st, 1)
        vz = st[0, 9]
        if vmax_after == 0.0:
            vmin = min(vmin, vz)
        if vz > 0:
            vmax_after = max(vmax_after, vz)
    assert vmin < -5.5
    assert abs(vmax_after - 0.5 * abs(vmin)) < 0.15 * 0.5 * abs(vmin)


URDF_1DOF = """<?xml version="1.0"?>
<robot name="hinge">
  <link name="base"><collision><geometry><box size="0.1 0.1 0.1"/></geometry></collision></link>
  <link name="arm">
    <inertial><mass value="1.0"/><inertia ixx="0.02" ixy="0" ixz="0" iyy="0.02" iyz="0" izz="0.05"/></inertial>
  </link>
  <joint name="hinge" type="revolute">
    <origin xyz="0 0 0.2"/><parent link="base"/><child link="arm"/><axis xyz="0 0 1"/>
    <limit lower="-3" upper="3" effort="0" velocity="0"/>
  </joint>
</robot>
"""


def _hinge(gym, kp, kd, target, armature=0.0, limits=None):
    sim = _sim(gym, gravity=(0, 0, 0), ground=False, npos=4)
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "hinge.urdf"), "w") as f:
        f.write(URDF_1DOF)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    opts.armature = armature
    a = gym.load_asset(sim, d, "hinge.urdf", opts)
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 1)
    h = gym.create_actor(env, a, gymapi.Transform(gymapi.Vec3(0, 0, 1)), "hinge", 0, 0)
    props = gym.get_actor_dof_properties(env, h)
    props["driveMode"][0] = gymapi.DOF_MODE_POS
    props["stiffness"][0] = kp
    props["damping"][0] = kd
    if limits is not None:
        props["lower"][0], props["upper"][0] = limits
    gym.set_actor_dof_properties(env, h, props)
    sim.build_model()
    tgt = np.zeros((1, 3), np.float32)
    tgt[0, 0] = target
    return sim.mg_params(), sim.mg_model(), sim.model_arrays["body_state0"].copy(), \
        sim.model_arrays["dof_state0"].copy(), tgt


def test_pd_drive_implicit_recurrence(gym):
    """One revolute DOF (I_zz = 0.05 kg m^2, armature 0.01) under a stiff PD
    drive (kp 400, kd 5): the ABA + implicit drive must follow the implicit-Euler
    recurrence (I + a + h kd + h^2 kp) qdd = kp (q* - q - h qd) - kd qd exactly
    (float64 reference, atol 1e-5 rad over 2 s) and settle at the target."""
    kp, kd, arm, q_t = 400.0, 5.0, 0.01, 0.8
    p, m, st, ds, tgt = _hinge(gym, kp, kd, q_t, armature=arm)
    h = (1 / 60) / 2
    q, qd = 0.0, 0.0
    I = 0.05 + arm
    for k in range(120):
        oracle.step(p, m, st, ds, tgt=tgt)
        for _ in range(2):
            qdd = (kp * (q_t - q - h * qd) - kd * qd) / (I + h * kd + h * h * kp)
            qd += h * qdd
            q += h * qd
        assert abs(ds[0, 0] - q) < 1e-5 and abs(ds[0, 1] - qd) < 1e-4, (k, ds[0], q, qd)
    assert abs(ds[0, 0] - q_t) < 1e-3
    # the link pose follows the joint: rotation about z by q
    np.testing.assert_allclose(st[1, 3:7], [0, 0, np.sin(q / 2), np.cos(q / 2)], atol=1e-5)
    np.testing.assert_allclose(st[1, 0:3], [0, 0, 1.2], atol=1e-6)


def test_joint_limit_clamp(gym):
    """A target beyond the upper limit: the joint stops at the limit."""
    p, m, st, ds, tgt = _hinge(gym, 200.0, 5.0, 2.5, armature=0.01, limits=(-0.5, 0.5))
    for _ in range(120):
        oracle.step(p, m, st, ds, tgt=tgt)
    assert ds[0, 0] == pytest.approx(0.5, abs=1e-6)
    assert ds[0, 1] == 0.0


def test_step_threads_equals_step():
    """oracle.step_threads (OpenMP, bench.py's CPU baseline) gives oracle.step's
    result bit for bit on the S1, S2 and S3 scenes."""
    import bench
    import oracle as O
    for leg, n in (("s1", 64), ("s2", 32), ("s3", 8)):
        sim, hook, tgt = bench._cpu_scene(leg, n)
        p, m = sim.mg_params(), sim.mg_model()
        st0 = sim.model_arrays["body_state0"].copy()
        d0 = sim.model_arrays["dof_state0"].copy()
        if tgt is None:
            tgt = np.zeros((max(d0.shape[0], 1), 3), np.float32)
        outs = []
        for nt in (0, 4):
            st, dof = st0.copy(), d0.copy()
            for k in range(5):
                hook(st, tgt, k)
                if nt:
                    O.step_threads(p, m, st, dof, nt, tgt=tgt)
                else:
                    O.step(p, m, st, dof, tgt=tgt)
            outs.append((st, dof))
        assert np.array_equal(outs[0][0], outs[1][0]), leg
        assert np.array_equal(outs[0][1], outs[1][1]), leg
        assert not np.array_equal(outs[0][0], st0), leg
