"""Edge crossings between two convex hulls in the coupled per-env step
(mg_collide.h cvx_edges_vs; oracle/migym_oracle_env.c cvx_edges_vs_).

Scene: a fixed cube hull turned 45 degrees about y (a ridge along y) and a free
cube hull turned 45 degrees about x (a bottom edge along x) dropped 2 cm onto
it: the first contact is an edge crossing with no vertex of either cube within
the contact offset of the other, the case the vertex tests alone miss (the cube
fell through the ridge before). It lands on the ridge and balances there until
rounding tips it off (an unstable equilibrium), as a physical cube would.
The same with one of the two cubes a box primitive (gym.create_box): a hull
edge crossing a box edge, where the edge pass gives the edge-edge normal (the
cross product of the two edges) instead of a box face's.
CPU: the oracle's behaviour; GPU: k_env_step bit for bit the oracle, 64 envs
with small random offsets.
"""
import math
import os

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
import oracle

H = 0.05
R2 = H * math.sqrt(2)


def _cube_urdf(d):
    with open(os.path.join(d, "cube.obj"), "w") as f:
        for sx in (-1, 1):
            for sy in (-1, 1):
                for sz in (-1, 1):
                    f.write("v %g %g %g\n" % (sx * H, sy * H, sz * H))
    with open(os.path.join(d, "cube.urdf"), "w") as f:
        f.write('<robot name="c"><link name="body"><collision><geometry><mesh filename="cube.obj"/></geometry>'
                '</collision></link></robot>')
    return "cube.urdf"


KINDS = ("hull_hull", "box_wedge", "box_cube")


def _scene(gym, d, n, gpu, seed=0, kind="hull_hull"):
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
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    f = _cube_urdf(d)
    fixed = gymapi.AssetOptions()
    fixed.fix_base_link = True
    if kind == "box_wedge":
        wedge = gym.create_box(sim, 2 * H, 2 * H, 2 * H, fixed)
    else:
        wedge = gym.load_asset(sim, d, f, fixed)
    if kind == "box_cube":
        cube = gym.create_box(sim, 2 * H, 2 * H, 2 * H, gymapi.AssetOptions())
    else:
        cube = gym.load_asset(sim, d, f, gymapi.AssetOptions())
        assert cube.bodies[0].shapes[0].type == 3              # a hull, not a box
    qy = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 1, 0), math.pi / 4)
    qx = gymapi.Quat.from_axis_angle(gymapi.Vec3(1, 0, 0), math.pi / 4)
    rng = np.random.RandomState(seed)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-0.5, -0.5, 0), gymapi.Vec3(0.5, 0.5, 1), 8)
        dx, dy = (rng.uniform(-0.01, 0.01, size=2) if i else (0.0, 0.0))
        gym.create_actor(env, wedge, gymapi.Transform(gymapi.Vec3(0, 0, 0.5), qy), "wedge", i, 0)
        gym.create_actor(env, cube, gymapi.Transform(gymapi.Vec3(dx, dy, 0.5 + 2 * R2 + 0.02), qx), "cube", i, 0)
    return sim


@pytest.mark.parametrize("kind", KINDS)
def test_cube_lands_on_ridge_edge_crossing(gym, tmp_path, kind):
    sim = _scene(gym, str(tmp_path), 1, False, kind=kind)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    zs = []
    for _ in range(30):
        oracle.step(p, m, st, np.zeros((0, 2), np.float32))
        zs.append(float(st[1, 2]))
    top = 0.5 + 2 * R2                                # centre height resting edge on ridge
    assert min(zs[6:20]) > top - 0.002               # caught by the edge contact, not through
    assert abs(zs[12] - top) < 0.002 and abs(float(st[1, 9])) < 0.2


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_edge_crossing_parity_gpu(gym, tmp_path, kind):
    n, steps = 64, 45
    sim = _scene(gym, str(tmp_path), n, True, seed=4, kind=kind)
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
