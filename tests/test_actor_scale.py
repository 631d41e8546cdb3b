"""gym.set_actor_scale (examples/actor_scaling.py:126): an actor's collision
geometry and joint frames scale by s, its mass properties with them (mass s^3,
inertia s^5, centre of mass s) — a body of the same density. Applied when the
scene is packed (test_isaacgym_amd/_sim.py build_model), so the oracle and the
device step the same scaled model; refused after prepare_sim.

CPU: the packed records and the oracle's rest heights (a 2x box rests at twice
the height, a 2x ant's legs reach twice as far); GPU: a mixed scaled scene bit
for bit the oracle.
"""
import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import scenes
import oracle

H = 0.1      # box half extent


def _scene(gym, gpu, n=2, scales=(1.0, 2.0)):
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0, 0, -9.8)
    sp.dt, sp.substeps = 1.0 / 60.0, 2
    sp.use_gpu_pipeline = gpu
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 6
    sp.physx.num_velocity_iterations = 1
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    pp = gymapi.PlaneParams()
    pp.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, pp)
    box = gym.create_box(sim, 2 * H, 2 * H, 2 * H, gymapi.AssetOptions())
    ant = gym.load_asset(sim, scenes.ASSET_ROOT, "mjcf/ant.xml", gymapi.AssetOptions())
    handles = []
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 4)
        s = scales[i % len(scales)]
        b = gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(1.0, 0, 0.5)), "box", i, 0)
        a = gym.create_actor(env, ant, gymapi.Transform(gymapi.Vec3(-1.0, 0, 1.0)), "ant", i, 0)
        assert gym.set_actor_scale(env, b, s) and gym.set_actor_scale(env, a, s)
        assert gym.get_actor_scale(env, b) == s
        handles.append((env, b, a))
    return sim, handles


def test_scaled_records_and_rest(gym):
    sim, handles = _scene(gym, False)
    env1, b1, a1 = handles[1]
    p1 = gym.get_actor_rigid_body_properties(env1, b1)[0]
    p0 = gym.get_actor_rigid_body_properties(handles[0][0], handles[0][1])[0]
    assert p1.mass == pytest.approx(8.0 * p0.mass, rel=1e-6)
    A = sim.build_model()
    # body rows: env 0 (box, ant bodies), env 1 (box, ant bodies)
    nb_env = len(A["body_kind"]) // 2
    m0, m1 = A["body_mass"][0], A["body_mass"][nb_env]
    assert m1[11] == pytest.approx(8.0 * m0[11], rel=1e-6)
    assert np.allclose(m1[1:4], m0[1:4] / 32.0, rtol=1e-5)
    sh = A["shapes"]
    boxes = sh[sh[:, 0] == 1]
    assert sorted(np.round(boxes[:, 1], 6)) == [H, 2 * H]
    # the ant's initial link offsets from its torso double
    st = A["body_state0"]
    d0 = st[1:nb_env, 0:3] - st[1, 0:3]
    d1 = st[nb_env + 1:2 * nb_env, 0:3] - st[nb_env + 1, 0:3]
    assert np.allclose(d1, 2.0 * d0, atol=1e-5)
    # resting heights on the oracle: the box at its (scaled) half extent, the
    # ant's torso at twice the height
    p, m = sim.mg_params(), sim.mg_model()
    s, dof = st.copy(), A["dof_state0"].copy()
    for _ in range(180):
        oracle.step(p, m, s, dof)
    assert s[0, 2] == pytest.approx(H, abs=2e-3)
    assert s[nb_env, 2] == pytest.approx(2 * H, abs=4e-3)
    z0, z1 = s[1, 2], s[nb_env + 1, 2]
    assert z1 == pytest.approx(2.0 * z0, rel=0.08)
    assert np.isfinite(s).all()


def test_scale_refused_after_prepare(gym):
    sim, handles = _scene(gym, False)
    sim.build_model()
    sim.finalize()
    env, b, _ = handles[0]
    assert not gym.set_actor_scale(env, b, 3.0) and gym.get_actor_scale(env, b) == 1.0


@pytest.mark.gpu
def test_scaled_scene_parity_gpu(gym):
    """64 envs alternating scale 1 / 2 / 0.5 (boxes and ants in one coupled env
    each), 90 frames: the device state equals the oracle's bit for bit."""
    n, frames = 64, 90
    sim, _ = _scene(gym, True, n=n, scales=(1.0, 2.0, 0.5))
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    st, dof = A["body_state0"].copy(), A["dof_state0"].copy()
    for f in range(frames):
        gym.simulate(sim)
        oracle.step(p, m, st, dof)
        if f % 30 == 29:
            gym.refresh_rigid_body_state_tensor(sim)
            got = rb.cpu().numpy()
            assert np.array_equal(got, st), "frame %d: max |diff| %g" % (f, np.abs(got - st).max())
    torch.cuda.synchronize()
