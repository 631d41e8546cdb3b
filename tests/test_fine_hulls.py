"""Convex hulls past the importer's 32-vertex default, up to PhysX's cooking
limits (255 vertices / 255 polygons, include/migym.h MG_HULL_MAX_VERTS / _FACES)
in the coupled per-env step: mg_env.hip's cooperative vertex / edge loops walk
such a hull in chunks (MG_NP_HULL_CHUNK), in index order, so the candidates and
their merge order are the oracle's (oracle/migym_oracle_env.c convex_convex_).

Scene: a fixed 120-gon prism (240 vertices, 122 faces, 360 edges) lying along y
and a free 100-gon prism (200 vertices, 102 faces, 300 edges) lying along x,
dropped 2 cm onto it crosswise: faceted cylinders whose flat top / bottom
facets (strips 3 mm wide) cross, so the contacts are edge crossings between
edges past the first chunk, and the vertex tests cover both hulls past index
64 (the old order key of B's vertices); it comes to rest crosswise. The importer's caps are raised
for the two meshes (test_isaacgym_amd/_assets.py HULL_CAPS, MIGYM_HULL_CAPS).
CPU: the importer keeps every vertex and the oracle's prism lands on the other
one; GPU: k_env_np / k_env_step bit for bit the oracle, 64 envs. And a pile
(mg_pile.hip, serial hull tests per pair): three free 200-vertex prisms
stacked crosswise on the 240-vertex one, bit for bit.
"""
import math
import os

import numpy as np
import pytest

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import _assets
import oracle

R = 0.05          # prism radius
L = 0.16          # prism length


def _prism_urdf(d, name, k, axis):
    """A k-gon prism of radius R and length L along axis (0 = x, 1 = y)."""
    with open(os.path.join(d, name + ".obj"), "w") as f:
        for j in range(k):
            a = 2 * math.pi * (j + 0.5) / k
            u, w = R * math.cos(a), R * math.sin(a)
            for s in (-0.5, 0.5):
                p = (s * L, u, w) if axis == 0 else (u, s * L, w)
                f.write("v %.7f %.7f %.7f\n" % p)
    with open(os.path.join(d, name + ".urdf"), "w") as f:
        f.write('<robot name="%s"><link name="body"><collision><geometry><mesh filename="%s.obj"/></geometry>'
                '</collision></link></robot>' % (name, name))
    return name + ".urdf"


@pytest.fixture
def fine_caps(monkeypatch):
    monkeypatch.setitem(_assets.HULL_CAPS, "rod_a.obj", (255, 255))
    monkeypatch.setitem(_assets.HULL_CAPS, "rod_b.obj", (255, 255))


def _scene(gym, d, n, gpu, seed=0, stack=1):
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
    pp = gymapi.PlaneParams()
    pp.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, pp)
    fixed = gymapi.AssetOptions()
    fixed.fix_base_link = True
    base = gym.load_asset(sim, d, _prism_urdf(d, "rod_a", 120, 1), fixed)
    rod = gym.load_asset(sim, d, _prism_urdf(d, "rod_b", 100, 0), gymapi.AssetOptions())
    rng = np.random.RandomState(seed)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-0.5, -0.5, 0), gymapi.Vec3(0.5, 0.5, 1), 8)
        dx, dy = (rng.uniform(-0.01, 0.01, size=2) if i else (0.0, 0.0))
        gym.create_actor(env, base, gymapi.Transform(gymapi.Vec3(0, 0, 0.2), gymapi.Quat()), "base", i, 0)
        for k in range(stack):
            # stack > 1: alternately crosswise (a quarter turn about z every other rod)
            q = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 0, 1), 0.5 * math.pi * (k % 2))
            gym.create_actor(env, rod, gymapi.Transform(gymapi.Vec3(dx, dy, 0.2 + 2 * R * (k + 1) + 0.02 * (k + 1)), q),
                             "rod%d" % k, i, 0)
    return sim, base, rod


def test_fine_hulls_import_and_land(gym, tmp_path, fine_caps):
    """Both hulls keep every vertex (240 / 200, over the old 32 and 64), and
    in the oracle the free prism lands crosswise on the fixed one and rests
    there (it never passes through)."""
    sim, base, rod = _scene(gym, str(tmp_path), 1, False)
    A = sim.build_model()
    nv = sorted(int(A["hulls"][int(s[2])]) for s in A["shapes"] if int(s[0]) == 3)
    assert nv == [200, 240]
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    zs = []
    for _ in range(40):
        oracle.step(p, m, st, np.zeros((0, 2), np.float32))
        zs.append(float(st[1, 2]))
    top = 0.2 + 2 * R                                # resting on the other rod's top
    rf = R * math.cos(math.pi / 100)                 # the facets' inner radius
    assert min(zs) > 0.2 + rf + R * math.cos(math.pi / 120) - 0.003
    assert max(abs(z - top) for z in zs[5:]) < 0.003
    assert np.all(np.isfinite(st))


@pytest.mark.gpu
def test_fine_hulls_parity_gpu(gym, tmp_path, fine_caps):
    """64 envs, 90 frames (landing, contact, resting): GPU state and net
    contact forces == the oracle's, bit for bit; every env on the coupled
    per-env step (k_env_np's cooperative hull loops)."""
    from test_isaacgym_amd import _native as N
    n, steps = 64, 90
    sim, *_ = _scene(gym, str(tmp_path), n, True, seed=4)
    gym.prepare_sim(sim)
    assert N.lib.mg_num_coupled_envs(sim.native) == n
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    cf = None
    for f in range(steps):
        gym.simulate(sim)
        cf = oracle.step(p, m, st, np.zeros((0, 2), np.float32))
        if f % 15 == 14 or f == steps - 1:
            gym.refresh_rigid_body_state_tensor(sim)
            got = rb.cpu().numpy()
            assert np.all(np.isfinite(got))
            assert np.array_equal(got, st), "frame %d: max |diff| %g" % (f, np.abs(got - st).max())
    gym.refresh_net_contact_force_tensor(sim)
    assert np.array_equal(ncf.cpu().numpy(), cf)


@pytest.mark.gpu
def test_fine_hulls_pile_parity_gpu(gym, tmp_path, fine_caps):
    """The pile step (k_pile_step: more than two free bodies, no articulation)
    with 200- / 240-vertex hulls: 64 envs of three prisms dropped in a
    crosswise stack on the fixed one, 90 frames, bit for bit the oracle."""
    from test_isaacgym_amd import _native as N
    n, steps = 64, 90
    sim, *_ = _scene(gym, str(tmp_path), n, True, seed=5, stack=3)
    gym.prepare_sim(sim)
    assert N.lib.mg_num_pile_envs(sim.native) == n
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    for f in range(steps):
        gym.simulate(sim)
        oracle.step(p, m, st, np.zeros((0, 2), np.float32))
        if f % 15 == 14 or f == steps - 1:
            gym.refresh_rigid_body_state_tensor(sim)
            got = rb.cpu().numpy()
            assert np.all(np.isfinite(got))
            assert np.array_equal(got, st), "frame %d: max |diff| %g" % (f, np.abs(got - st).max())
    # the stack topples onto the ground (rounding), but no rod passes into it
    rods = np.arange(st.shape[0]) % 4 != 0
    assert np.all(st[rods, 2] > R - 0.003)
