"""Known-answer tests of the ground friction patch of a free body (DESIGN.md
§3.2.1; oracle/migym_oracle.c gpatch_update_ and rigid_body_step, the bit-exact
restatement of test_isaacgym_amd/csrc/mg_rigid.hip k_rigid_step1), under
test10_servo_vecenv.py's own parameters (:117-144, the friction offset
threshold and correlation distance left at Isaac Gym's defaults 0.04 / 0.025,
ground mu 1) on the servo scene's ground vehicle (mass 100, the 7.5 x 3 x 2.5 m
box proxy of its missing mesh):

  - pushed along the ground's tangent basis it is held up to 0.95 mu m g (after a
    sub-millimetre give the same two anchors hold it, bit for bit) and slides
    above it — from 1.05 mu m g on — at (F - mu m g) / m;
  - pushed along a diagonal of the basis it holds up to sqrt(2) mu m g (the
    budget is per tangent direction, as PhysX's two-direction rows) and slides
    beyond;
  - a support that tilts slowly drops the patch once the tilt since the patch
    was made passes acos(0.999) = 2.56 degrees (the stored normal is
    the one the patch was created with, not the last substep's).
"""
import math

import numpy as np
import pytest

from isaacgym import gymapi
from test_isaacgym_amd import scenes
import oracle

G = 9.8


def _vehicle(gym, yaw=0.0, gravity=-G):
    sp = scenes.servo_sim_params(use_gpu_pipeline=False)
    sp.gravity = gymapi.Vec3(0.0, 0.0, gravity)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    plane.static_friction = 1.0
    plane.dynamic_friction = 1.0
    gym.add_ground(sim, plane)
    opts = gymapi.AssetOptions()
    opts.armature = 0.01
    asset = gym.load_asset(sim, scenes.ASSET_ROOT, "servo/ground_vehicle.urdf", opts)
    env = gym.create_env(sim, gymapi.Vec3(-20, -20, -20), gymapi.Vec3(20, 20, 20), 1)
    pose = gymapi.Transform(gymapi.Vec3(0.0, 0.0, 1.25), gymapi.Quat.from_euler_zyx(0.0, 0.0, yaw))
    gym.create_actor(env, asset, pose, "vehicle", 0, -1)
    A = sim.build_model()
    mu = 0.5 * (float(A["shapes"][0][11]) + 1.0)
    return sim, A, sim.mg_params(), sim.mg_model(), mu


def _settle(A, p, m, cc, frames=60):
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    for _ in range(frames):
        oracle.step(p, m, st, dof, contact_cache=cc)
    return st, dof


@pytest.mark.parametrize("push", [0.5, 0.9, 0.95, 1.05, 1.2])
def test_vehicle_push_along_basis(gym, push):
    sim, A, p, m, mu = _vehicle(gym)
    cc = oracle.contact_cache(m)
    st, dof = _settle(A, p, m, cc)
    rec = cc.body[0]
    assert rec[0] == 2.0                       # two anchors hold the resting vehicle
    mass = 100.0
    F = push * mu * mass * G
    ext = np.zeros((1, 6), np.float32)
    ext[0, 0] = F                              # world x = -t2 of the +z ground basis
    x0 = float(st[0, 0])
    frames = 90
    xs, recs = [], []
    for _ in range(frames):
        oracle.step(p, m, st, dof, ext=ext, contact_cache=cc)
        xs.append(float(st[0, 0]))
        recs.append(cc.body[0].copy())
    if push < 1.0:
        assert abs(xs[-1] - x0) < 1e-3, xs[-1] - x0      # the give of the anchors' drift closing
        assert abs(xs[-1] - xs[30]) < 1e-6
        assert all(r[0] == 2.0 for r in recs[30:])
        assert np.array_equal(recs[-1], recs[30])         # the same anchors, bit for bit
    else:
        t = frames / 60.0
        d_expect = 0.5 * (F - mu * mass * G) / mass * t * t
        assert abs((xs[-1] - x0) - d_expect) < 0.1 * d_expect + 2e-3, (xs[-1] - x0, d_expect)
        assert abs(float(st[0, 2]) - 1.25) < 2e-3         # flat on the ground
        assert abs(float(st[0, 1])) < 5e-3                # no sideways walk


@pytest.mark.parametrize("push,holds", [(0.9, True), (1.3, True), (1.6, False)])
def test_vehicle_push_along_diagonal(gym, push, holds):
    """The tangent budget is mu N per direction of the basis (PhysX's
    two-direction patch rows): along a diagonal the patch holds up to sqrt(2)
    mu m g, and slides beyond. Parity unpinned: this is this build's restatement
    of PhysX's pyramid patch friction; no reference output
    pins the sqrt(2) diagonal budget (Isaac Gym is absent here),
    so the KAT fixes the build's own behaviour, not Isaac Gym's."""
    sim, A, p, m, mu = _vehicle(gym)
    cc = oracle.contact_cache(m)
    st, dof = _settle(A, p, m, cc)
    mass = 100.0
    F = push * mu * mass * G
    ext = np.zeros((1, 6), np.float32)
    ext[0, 0] = F / math.sqrt(2.0)
    ext[0, 1] = F / math.sqrt(2.0)
    p0 = st[0, 0:2].copy()
    for _ in range(90):
        oracle.step(p, m, st, dof, ext=ext, contact_cache=cc)
    moved = float(np.linalg.norm(st[0, 0:2] - p0))
    if holds:
        assert moved < 1e-3, moved
    else:
        assert moved > 0.1, moved


def test_slowly_tilting_support_drops_patch(gym):
    """A 0.2 m cube resting on the ground, turned 0.5 degrees further about one
    bottom edge every step (set as a teleport, zero velocity; gravity keeps the
    normal force, without which every friction row would slip):
    the anchors stay within the correlation distance, so only the normal test
    can drop the patch — and it does at the step where the tilt since the patch
    was made first exceeds 2.56 degrees (6 x 0.5), not before, and the new patch
    is made with the current normal."""
    sp = scenes.servo_sim_params(use_gpu_pipeline=False)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    box = gym.create_box(sim, 0.2, 0.2, 0.2, gymapi.AssetOptions())
    env = gym.create_env(sim, gymapi.Vec3(-1, -1, -1), gymapi.Vec3(1, 1, 1), 1)
    gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0.0, 0.0, 0.1)), "box", 0, 0)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    oracle.step(p, m, st, dof, contact_cache=cc)
    made = cc.body[0].copy()
    assert made[0] == 2.0
    drop_at = None
    for k in range(1, 9):
        th = math.radians(0.5 * k)
        # rotate about the x-axis through the bottom edge (y = -0.1, z = 0)
        st[0, 0:3] = [0.0, -0.1 + 0.1 * math.cos(th) - 0.1 * math.sin(th), 0.1 * math.sin(th) + 0.1 * math.cos(th)]
        st[0, 3:7] = [math.sin(th / 2), 0.0, 0.0, math.cos(th / 2)]
        st[0, 7:13] = 0.0
        oracle.step(p, m, st, dof, contact_cache=cc)
        rec = cc.body[0]
        if drop_at is None and not np.array_equal(rec[1:4], made[1:4]):
            drop_at = k
    assert drop_at == 6, drop_at
    th = math.radians(3.0)
    assert np.allclose(cc.body[0][1:4], [0.0, math.sin(th), math.cos(th)], atol=1e-6)   # made at the 3 degree tilt
