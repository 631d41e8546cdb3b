"""Capsule segment contacts (mg_collide.h
capsule_segment_convex / seg_closest / seg_seg_closest, restated by
oracle/migym_oracle_env.c). Round 3 replaced a capsule by its two end-cap
spheres, so a capsule lying across a box or hull between its caps — the ant's
legs (assets/mjcf/nv_ant.xml:42-44, examples/apply_forces.py:67) and every
humanoid limb — had no contact there and fell through.

CPU (the oracle, known answers):
  - a capsule dropped across a narrow beam (box primitive or hull), both caps
    beyond the beam's sides: it comes to rest on the beam's top face at
    z = top + r, in the middle of its segment;
  - a capsule dropped across a ridge (a box turned 45 degrees): caught at the
    ridge edge by the edge-edge contact, not through;
  - a sphere dropped on the middle of a fixed horizontal capsule: rests on it
    (closest point of the axis segment), where the caps alone let it fall.
GPU: k_env_step bit for bit the oracle on the same scenes (64 envs, small
random offsets), and the ant dropped onto a fixed box.
"""
import math
import os

import numpy as np
import pytest

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import scenes
import oracle

R = 0.04          # capsule radius
L = 0.6           # capsule length between the cap centres
TOP = 0.5         # beam top


def _params(gpu):
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0, 0, -9.8)
    sp.dt, sp.substeps = 1.0 / 60.0, 2
    sp.use_gpu_pipeline = gpu
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 8
    sp.physx.num_velocity_iterations = 1
    sp.physx.contact_offset = 0.005
    sp.physx.rest_offset = 0.0
    return sp


def _beam_hull(d):
    """A 0.2 x 1.0 x 0.1 m beam as a hull (OBJ of its 8 corners)."""
    with open(os.path.join(d, "beam.obj"), "w") as f:
        for sx in (-1, 1):
            for sy in (-1, 1):
                for sz in (-1, 1):
                    f.write("v %g %g %g\n" % (sx * 0.1, sy * 0.5, sz * 0.05))
    with open(os.path.join(d, "beam.urdf"), "w") as f:
        f.write('<robot name="b"><link name="body"><collision><geometry><mesh filename="beam.obj"/></geometry>'
                '</collision></link></robot>')
    return "beam.urdf"


def _scene(gym, d, kind, n=1, gpu=False, seed=0):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, _params(gpu))
    fixed = gymapi.AssetOptions()
    fixed.fix_base_link = True
    rng = np.random.RandomState(seed)
    if kind == "box":
        support = gym.create_box(sim, 0.2, 1.0, 0.1, fixed)
    elif kind == "hull":
        support = gym.load_asset(sim, d, _beam_hull(d), fixed)
        assert support.bodies[0].shapes[0].type == 3           # a hull, not a box
    elif kind == "ridge":
        support = gym.create_box(sim, 0.2, 1.0, 0.2, fixed)
    else:                                                       # "rod": a fixed horizontal capsule
        support = gym.create_capsule(sim, R, L, fixed)
    if kind == "rod":
        mover = gym.create_sphere(sim, 0.05, gymapi.AssetOptions())
    else:
        mover = gym.create_capsule(sim, R, L, gymapi.AssetOptions())
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 8)
        dx, dy = (rng.uniform(-0.005, 0.005, size=2) if i else (0.0, 0.0))
        if kind == "ridge":
            q = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 1, 0), math.pi / 4)
            gym.create_actor(env, support, gymapi.Transform(gymapi.Vec3(0, 0, TOP - 0.1 * math.sqrt(2)), q),
                             "support", i, 0)
        elif kind == "rod":
            gym.create_actor(env, support, gymapi.Transform(gymapi.Vec3(0, 0, TOP)), "support", i, 0)
        else:
            gym.create_actor(env, support, gymapi.Transform(gymapi.Vec3(0, 0, TOP - 0.05)), "support", i, 0)
        z = TOP + (0.05 + R if kind == "rod" else R) + 0.02
        gym.create_actor(env, mover, gymapi.Transform(gymapi.Vec3(dx, dy, z)), "mover", i, 0)
    return sim


@pytest.mark.parametrize("kind", ["box", "hull"])
def test_capsule_rests_across_beam(gym, tmp_path, kind):
    """Both caps beyond the beam's sides (x = +-0.3 vs half width 0.1): only the
    segment contact holds it; it rests at top + r, level."""
    sim = _scene(gym, str(tmp_path), kind)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    for _ in range(60):
        oracle.step(p, m, st, np.zeros((0, 2), np.float32))
    assert abs(float(st[1, 2]) - (TOP + R)) < 2e-3, float(st[1, 2])
    assert np.abs(st[1, 7:13]).max() < 0.05
    assert abs(float(st[1, 0])) < 1e-3                      # balanced over the beam


def test_capsule_caught_by_ridge_edge(gym, tmp_path):
    """A capsule across a ridge (a box edge, turned 45 degrees): the segment
    crosses the box edge between its caps — the edge-edge contact catches it."""
    sim = _scene(gym, str(tmp_path), "ridge")
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    zs = []
    for _ in range(30):
        oracle.step(p, m, st, np.zeros((0, 2), np.float32))
        zs.append(float(st[1, 2]))
    assert min(zs[8:]) > TOP + R - 3e-3, min(zs[8:])         # caught at the edge, not through
    assert abs(zs[-1] - (TOP + R)) < 3e-3


def test_sphere_rests_on_capsule_middle(gym, tmp_path):
    """A sphere dropped on the middle of a fixed horizontal capsule rests on
    it: the closest point of the axis segment, not a cap (the caps are 0.3 m
    away)."""
    sim = _scene(gym, str(tmp_path), "rod")
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    for _ in range(30):
        oracle.step(p, m, st, np.zeros((0, 2), np.float32))
    assert abs(float(st[1, 2]) - (TOP + R + 0.05)) < 2e-3, float(st[1, 2])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["box", "hull", "ridge", "rod"])
def test_capsule_contacts_parity_gpu(gym, tmp_path, kind):
    n, steps = 64, 45
    sim = _scene(gym, str(tmp_path), kind, n, True, seed=3)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    cf = None
    for _ in range(steps):
        gym.simulate(sim)
        cf = oracle.step(p, m, st, np.zeros((0, 2), np.float32))
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_net_contact_force_tensor(sim)
    got = rb.cpu().numpy()
    assert np.all(np.isfinite(got))
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
    assert np.array_equal(ncf.cpu().numpy(), cf)


def _ant_on_box(gym, n, gpu):
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, scenes.ant_sim_params(gpu))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    ant = gym.load_asset(sim, scenes.ASSET_ROOT, "mjcf/ant.xml", gymapi.AssetOptions())
    fixed = gymapi.AssetOptions()
    fixed.fix_base_link = True
    box = gym.create_box(sim, 0.3, 0.3, 0.3, fixed)
    rng = np.random.RandomState(7)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 8)
        q = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 0, 1), float(rng.uniform(-3, 3)))
        gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0, 0, 0.15)), "box", i, 0)
        gym.create_actor(env, ant, gymapi.Transform(gymapi.Vec3(float(rng.uniform(-0.1, 0.1)), 0, 0.9), q),
                         "ant", i, 0)
    return sim


def test_ant_lands_on_box(gym):
    """The ant dropped onto a 0.3 m box: its capsule legs (nv_ant.xml:42-44)
    land on the box's top face and edges, nothing passes through the box."""
    sim = _ant_on_box(gym, 1, False)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st, ds = A["body_state0"].copy(), A["dof_state0"].copy()
    for _ in range(90):
        oracle.step(p, m, st, ds, props=A["dof_props"])
    assert np.all(np.isfinite(st))
    assert float(st[1, 2]) > 0.3                              # the torso stays above the box top


@pytest.mark.gpu
def test_ant_on_box_parity_gpu(gym):
    """64 ants dropped onto fixed boxes, 90 frames: k_env_step bit for bit the
    oracle (capsule-box segment contacts, cap contacts, the ground)."""
    n = 64
    sim = _ant_on_box(gym, n, True)
    gym.prepare_sim(sim)
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    props = sim.model_arrays["dof_props"]
    for _ in range(90):
        gym.simulate(sim)
        oracle.step(p, m, st, ds, props=props)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    assert np.all(np.isfinite(got))
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
