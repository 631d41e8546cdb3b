"""Friction anchors of the coupled step on the device:
k_env_step's patch records, anchor rows and slip release against the oracle's
restatement (oracle/migym_oracle_env.c patch_update_), bit for bit.

64 envs of a tile on a table, each yawed differently and pushed sideways every
frame by its own force from 0.3 to 2 mu m g (held by its anchors, or
slipping and re-anchoring; the per-direction bound of the tangent rows holds
up to sqrt(2) mu m g along a diagonal of the patch basis), through gym.apply_rigid_body_force_tensors — the
device keeps its patches inside the sim, the oracle in the cache that goes with
its state array.
"""
import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
import oracle

pytestmark = pytest.mark.gpu
G = 9.8


def _scene(gym, n, corr=0.0005, yaw_step=0.1):
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0, 0, -G)
    sp.dt = 1.0 / 60.0
    sp.substeps = 2
    sp.use_gpu_pipeline = True
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 8
    sp.physx.num_velocity_iterations = 1
    sp.physx.contact_offset = 0.001
    sp.physx.rest_offset = 0.0
    sp.physx.friction_offset_threshold = 0.001
    sp.physx.friction_correlation_distance = corr
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    table = gym.create_box(sim, 0.6, 1.0, 0.4, opts)
    tile = gym.create_box(sim, 0.1, 0.1, 0.02, gymapi.AssetOptions())
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 8)
        gym.create_actor(env, table, gymapi.Transform(gymapi.Vec3(0.5, 0, 0.2)), "table", i, 0)
        pose = gymapi.Transform(gymapi.Vec3(0.45, 0.1, 0.4101))
        pose.r = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 0, 1), yaw_step * i)
        gym.create_actor(env, tile, pose, "tile", i, 0)
    gym.prepare_sim(sim)
    return sim


@pytest.mark.parametrize("corr", [0.0005, 0.3])
def test_friction_anchor_push_parity_gpu(gym, corr):
    """corr 0.0005 (franka_cube_ik_osc.py's): two anchors per patch, sharing
    the budget — held below 0.9 mu m g, sliding above 1.5; 0.3 (above the
    tile's diagonal): one anchor carries the patch, and with no torsional
    friction the pushed tile pivots about it (parity only)."""
    from test_isaacgym_amd import _native as N
    n, frames = 64, 90
    sim = _scene(gym, n, corr)
    assert N.lib.mg_num_coupled_envs(sim.native) == n
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    mass = 1000.0 * 0.1 * 0.1 * 0.02
    push = np.linspace(0.3, 2.0, n).astype(np.float32) * np.float32(mass * G)
    yaw = 0.7 * np.arange(n)
    f = torch.zeros((n, 2, 3), device="cuda:0")
    t = torch.zeros((n, 2, 3), device="cuda:0")
    ext = np.zeros((2 * n, 6), np.float32)
    moved = np.zeros(n)
    for k in range(frames):
        on = k >= 20                       # settle, then push
        fx = (push * np.cos(yaw)).astype(np.float32) if on else np.zeros(n, np.float32)
        fy = (push * np.sin(yaw)).astype(np.float32) if on else np.zeros(n, np.float32)
        f[:, 1, 0] = torch.from_numpy(fx).cuda()
        f[:, 1, 1] = torch.from_numpy(fy).cuda()
        assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(f), gymtorch.unwrap_tensor(t),
                                                  gymapi.ENV_SPACE)
        ext[1::2, 0] = fx
        ext[1::2, 1] = fy
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        cf = oracle.step(p, m, st, dof, ext=ext)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        got = rb.cpu().numpy()
        if not np.array_equal(got, st):
            bad = np.argwhere(got != st)
            pytest.fail("frame %d: first differing body/field %s, max |diff| %g"
                        % (k, bad[:3].tolist(), np.abs(got - st).max()))
        assert np.array_equal(ncf.cpu().numpy(), cf), "frame %d: net contact force" % k
        if k == 19:
            x20 = got[1::2, 0:2].copy()
    if corr > 0.1:
        return
    moved = np.linalg.norm(got[1::2, 0:2] - x20, axis=1)
    held = push < 0.9 * mass * G
    slid = push > 1.5 * mass * G
    assert held.any() and slid.any()
    assert np.all(moved[held] < 1e-3)             # held in place by the anchors
    assert np.all(moved[slid] > 0.02)             # slipping patches slide


def test_friction_anchor_basis_push_gpu(gym):
    """Pushes along the patch's tangent basis (t1 = +y, t2 = -x for the +z
    table top), where the per-direction budget is exact: held below 0.95 mu m g
    (both anchors share the push; the patch slips only when both clamp), sliding
    from 1.05 mu m g on at (F - mu m g) / m, bit for bit with the oracle."""
    pushes = np.array([0.5, 0.9, 0.95, 1.05] * 2, np.float32)
    along_y = np.arange(pushes.size) >= 4
    n, settle, frames = pushes.size, 20, 60
    sim = _scene(gym, n, yaw_step=0.0)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    mu = float(0.5 * (A["shapes"][0][11] + A["shapes"][1][11]))
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    mass = 1000.0 * 0.1 * 0.1 * 0.02
    F = pushes * np.float32(mu * mass * G)
    fx = np.where(along_y, 0.0, F).astype(np.float32)           # +x (toward the table's far edge)
    fy = np.where(along_y, -F, 0.0).astype(np.float32)          # -y
    f = torch.zeros((n, 2, 3), device="cuda:0")
    t = torch.zeros((n, 2, 3), device="cuda:0")
    ext = np.zeros((2 * n, 6), np.float32)
    for k in range(settle + frames):
        if k == settle:
            f[:, 1, 0] = torch.from_numpy(fx).cuda()
            f[:, 1, 1] = torch.from_numpy(fy).cuda()
            ext[1::2, 0] = fx
            ext[1::2, 1] = fy
            x0 = st[1::2, 0:2].copy()
        assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(f), gymtorch.unwrap_tensor(t),
                                                  gymapi.ENV_SPACE)
        gym.simulate(sim)
        oracle.step(p, m, st, dof, ext=ext)
    gym.refresh_rigid_body_state_tensor(sim)
    got = rb.cpu().numpy()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
    moved = np.linalg.norm(st[1::2, 0:2] - x0, axis=1)
    held = pushes <= 0.95
    assert np.all(moved[held] < 1e-3), moved[held]
    tt = frames / 60.0
    expect = 0.5 * (pushes[~held] - 1.0) * mu * G * tt * tt
    assert np.all(np.abs(moved[~held] - expect) < 0.15 * expect), (moved[~held], expect)
