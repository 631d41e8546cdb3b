"""The free-body pile step on the device (csrc/mg_pile.hip k_pile_step,
DESIGN.md §3.10) against its restatement (oracle/migym_oracle_pile.c), bit
for bit — rigid-body state and net contact force, every frame:

  - examples/1080_balls_of_solitude.py's scene (30 balls per env, group i,
    filter 0, y-up, 1 substep, TGS 4/1) at the script's 36 envs and at 256 —
    the pyramids fall, the layers meet at ~10 m/s and collapse;
  - ragged heaps of spheres, boxes, capsules and hulls (3 to 64 free bodies per
    env, on a fixed box and the ground), z-up and y-up, with indexed root-state
    teleports and external wrenches through the tensor API mid-run;
  - a 4 x 4 x 4 block of touching boxes, whose contacts overflow the per-env
    tables (128 active pairs / 256 points): the truncation rule is part of the
    parity;
  - 4096 envs of the pyramid (the bench's S6 size) on the multi-threaded
    oracle.
"""
import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import scenes
import oracle
import pile_scenes as PS

pytestmark = pytest.mark.gpu


def _check(k, rb, ncf, st, cf):
    got = rb.cpu().numpy()
    if not np.array_equal(got, st):
        bad = np.argwhere(got != st)
        pytest.fail("frame %d: first differing body/field %s, max |diff| %g"
                    % (k, bad[:3].tolist(), np.abs(got - st).max()))
    gcf = ncf.cpu().numpy()
    if not np.array_equal(gcf, cf):
        bad = np.argwhere(gcf != cf)
        pytest.fail("frame %d: net contact force differs at %s" % (k, bad[:3].tolist()))


@pytest.mark.parametrize("n", [36, 256])
def test_ball_pyramid_parity_gpu(gym, n):
    from test_isaacgym_amd import _native as N
    sim, envs = scenes.ball_pile_scene(gym, n, use_gpu_pipeline=True)
    gym.prepare_sim(sim)
    assert N.lib.mg_num_pile_envs(sim.native) == n
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    for k in range(150):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        cf = oracle.step(p, m, st, dof)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        _check(k, rb, ncf, st, cf)
    y = st[:, 1].reshape(n, 30)
    assert y.max() < 1.5 and y.min() > 0.19                       # collapsed onto the ground


@pytest.mark.parametrize("up", ["z", "y"])
def test_mixed_pile_parity_gpu(gym, tmp_path, up):
    from test_isaacgym_amd import _native as N
    n = 64
    sim, info = PS.mixed_pile_scene(gym, n, True, d=str(tmp_path), up=up)
    gym.prepare_sim(sim)
    assert N.lib.mg_num_pile_envs(sim.native) == n
    nb = sum(info["bodies_per_env"])
    assert max(info["bodies_per_env"]) == 65                      # 64 free bodies + the fixed box
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    first = np.cumsum([0] + info["bodies_per_env"][:-1])
    rng = np.random.RandomState(3)
    f = torch.zeros((nb, 3), device="cuda:0")
    t = torch.zeros((nb, 3), device="cuda:0")
    for k in range(120):
        ext = None
        if k == 40:
            # teleport the first free body of every other env back up, spinning
            gym.refresh_actor_root_state_tensor(sim)
            idx = (first[::2] + 1).astype(np.int32)
            up_i = 2 if up == "z" else 1
            root[idx, up_i] = 0.6
            root[idx, 10:13] = torch.tensor([3.0, -2.0, 1.0], device="cuda:0")
            ids = torch.from_numpy(idx).cuda()
            assert gym.set_actor_root_state_tensor_indexed(sim, gymtorch.unwrap_tensor(root),
                                                           gymtorch.unwrap_tensor(ids), len(idx))
            st[idx, up_i] = np.float32(0.6)
            st[idx, 10:13] = np.array([3.0, -2.0, 1.0], np.float32)
        if 50 <= k < 80:
            fa = rng.uniform(-2, 2, size=(nb, 3)).astype(np.float32)
            ta = rng.uniform(-0.05, 0.05, size=(nb, 3)).astype(np.float32)
            f.copy_(torch.from_numpy(fa))
            t.copy_(torch.from_numpy(ta))
            assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(f), gymtorch.unwrap_tensor(t),
                                                      gymapi.ENV_SPACE)
            ext = np.concatenate([fa, ta], axis=1)
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        cf = oracle.step(p, m, st, dof, ext=ext)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        _check(k, rb, ncf, st, cf)


def test_overflowing_block_parity_gpu(gym):
    """64 touching 0.1 m cubes in a 4 x 4 x 4 block: ~900 candidate contact
    points a substep against the 256-point table; the pairs past the first
    overflow are dropped for the substep, on both sides alike."""
    from test_isaacgym_amd import _native as N
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, PS.sim_params(True, npos=4, contact_offset=0.02))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    box = gym.create_box(sim, 0.1, 0.1, 0.1, gymapi.AssetOptions())
    n = 8
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 4)
        for k in range(64):
            x, y, z = k % 4, (k // 4) % 4, k // 16
            pose = gymapi.Transform(gymapi.Vec3(0.1 * x + 0.001 * i, 0.1 * y, 0.05 + 0.1 * z))
            gym.create_actor(env, box, pose, None, i, 0)
    gym.prepare_sim(sim)
    assert N.lib.mg_num_pile_envs(sim.native) == n
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    for k in range(30):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        cf = oracle.step(p, m, st, dof)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        _check(k, rb, ncf, st, cf)


def test_ball_pyramid_4096_gpu(gym):
    n = 4096
    sim, envs = scenes.ball_pile_scene(gym, n, use_gpu_pipeline=True)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    for k in range(75):
        gym.simulate(sim)
        cf = oracle.step_threads(p, m, st, dof, 16)
        if k % 15 == 14:
            gym.fetch_results(sim, True)
            gym.refresh_rigid_body_state_tensor(sim)
            gym.refresh_net_contact_force_tensor(sim)
            _check(k, rb, ncf, st, cf)


def test_piles_beside_other_env_kinds_gpu(gym):
    """Pile envs in one sim with every other kind of env — coupled envs of
    two free bodies (k_env_step), uncoupled free bodies (k_rigid_step1) and
    fixed-base articulations (the chain kernel) — each stepped by its own
    kernel over the shared SoA state: all bit-exact against the oracle."""
    from test_isaacgym_amd import _native as N, scenes as SC
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, PS.sim_params(True))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    ball = gym.create_sphere(sim, 0.05, gymapi.AssetOptions())
    box = gym.create_box(sim, 0.1, 0.1, 0.1, gymapi.AssetOptions())
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    opts.default_dof_drive_mode = gymapi.DOF_MODE_POS
    gimbal = gym.load_asset(sim, SC.ASSET_ROOT, "servo/gimbal.urdf", opts)
    kinds = []
    for i in range(24):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 6)
        k = i % 4
        kinds.append(k)
        if k == 0:       # a pile: 5 balls in a column
            for j in range(5):
                gym.create_actor(env, ball, gymapi.Transform(gymapi.Vec3(0.01 * j, 0, 0.1 + 0.12 * j)), None, i, 0)
        elif k == 1:     # two boxes, one on the other: a coupled env (k_env_step)
            gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0, 0, 0.05)), None, i, 0)
            gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0.02, 0, 0.2)), None, i, 0)
        elif k == 2:     # free bodies that may not touch each other: uncoupled
            for j in range(3):
                gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0.3 * j, 0, 0.3)), None, i, 1)
        else:            # a fixed-base gimbal driven to a target
            h = gym.create_actor(env, gimbal, gymapi.Transform(gymapi.Vec3(0, 2, 3)), None, i, 1)
            props = gym.get_actor_dof_properties(env, h)
            props["stiffness"][:] = 50.0
            props["damping"][:] = 5.0
            gym.set_actor_dof_properties(env, h, props)
    gym.prepare_sim(sim)
    assert N.lib.mg_num_pile_envs(sim.native) == 6
    assert N.lib.mg_num_coupled_envs(sim.native) == 6             # k_env_step's envs (piles not counted)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    dofs = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    st = A["body_state0"].copy()
    dof = A["dof_state0"].copy()
    nd = dof.shape[0]
    tgt = np.zeros((nd, 3), np.float32)
    tgt[:, 0] = np.tile(np.array([0.5, -0.4, 0.3], np.float32), nd // 3)
    gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(tgt[:, 0].copy()).cuda()))
    for k in range(90):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        cf = oracle.step(p, m, st, dof, tgt=tgt, props=A["dof_props"])
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        gym.refresh_dof_state_tensor(sim)
        _check(k, rb, ncf, st, cf)
        assert np.array_equal(dofs.cpu().numpy(), dof), "frame %d: DOF state" % k
