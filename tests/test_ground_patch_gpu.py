"""GPU parity of the free bodies' ground friction patches (DESIGN.md §3.2.1,
mg_rigid.hip k_rigid_step1 with its persistent [MG_FP_N][nf1] record table)
against the oracle (oracle/migym_oracle.c rigid_body_step, its body cache kept
from step to step the same way), bit for bit:

  - test10's servo scene (UAV + ground vehicle per env, the patch parameters at
    Isaac Gym's defaults) under a random root teleport every frame (vehicles
    thrown at up to 50 m/s: anchors made and dropped), then one gentle teleport
    of every vehicle to 0.15 m above its rest height at rest and 40 frames in
    which they land and come to rest on their anchors;
  - ground vehicles pushed sideways through apply_rigid_body_force_tensors at
    0.5 / 0.9 / 1.1 / 1.5 mu m g (held below, sliding above), with a teleport
    of every other env half-way (the held anchors let go of a moved body).
"""
import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import scenes
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_servo_teleports_then_rest_bitexact(gym):
    n, teleports, rest = 256, 40, 40
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    acts = scenes.servo_actions(n, teleports, DEV, seed=31)
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    st = sim.model_arrays["body_state0"].copy()
    roots = sim.model_arrays["actor_root_body"]
    dof = np.zeros((0, 2), np.float32)
    gym.refresh_actor_root_state_tensor(sim)
    held_seen = 0
    for k in range(teleports + rest):
        if k < teleports:
            root[:, 3:10] = acts[k]
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            st[roots, 3:10] = acts[k].cpu().numpy()
        elif k == teleports:
            # vehicles set down at rest, upright at the last action's yaw (one
            # thrown at 50 m/s may have tumbled in the frame after its teleport;
            # set down tilted, one landed on its side with round 6's sweep
            # order — physics, not the patch under test)
            root[1::2, 2] = 1.4
            root[1::2, 3:7] = acts[k - 1][1::2, 0:4]
            root[1::2, 7:13] = 0.0
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            st[roots[1::2], 2] = 1.4
            st[roots[1::2], 3:7] = acts[k - 1][1::2, 0:4].cpu().numpy()
            st[roots[1::2], 7:13] = 0.0
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        cf = oracle.step(p, m, st, dof, contact_cache=cc)
        got = rb.cpu().numpy()
        assert np.array_equal(got, st), "frame %d: max |diff| %g" % (k, np.abs(got - st).max())
        assert np.array_equal(ncf.cpu().numpy(), cf), "frame %d: contact force" % k
        held_seen = max(held_seen, int((cc.body[:, 0] == 2.0).sum()))
    assert held_seen >= n                      # every vehicle came to rest on two anchors
    veh = roots[1::2]
    assert np.all(np.abs(st[veh, 2] - 1.25) < 2e-3) and np.all(np.abs(st[veh, 7:10]) < 1e-2)


def test_vehicle_pushes_bitexact(gym):
    n, frames = 64, 90
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    A = sim.model_arrays
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    nb = st.shape[0]
    for _ in range(60):                      # the vehicles settle (the UAVs keep falling)
        gym.simulate(sim)
        oracle.step(p, m, st, dof, contact_cache=cc)
    mu = 0.5 * (float(A["shapes"][int(A["tmpl_body_i"][A["body_tmpl"][1]][0])][11]) + 1.0)
    force = np.zeros((nb, 3), np.float32)
    pushes = np.array([0.5, 0.9, 1.1, 1.5], np.float32)[np.arange(n) % 4]
    force[1::2, 0] = pushes * mu * 100.0 * 9.8
    force[1::2, 1] = np.where(np.arange(n) % 8 >= 4, 0.3, 0.0) * mu * 100.0 * 9.8
    ext = np.zeros((nb, 6), np.float32)
    ext[:, 0:3] = force
    ft = torch.from_numpy(force).to(DEV)
    tq = torch.zeros_like(ft)
    x0 = st[1::2, 0].copy()
    for k in range(frames):
        if k == frames // 2:                 # teleport every other vehicle 2 m sideways
            gym.refresh_actor_root_state_tensor(sim)
            sel = torch.arange(1, 2 * n, 4, device=DEV)
            root[sel, 1] += 2.0
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            st[np.arange(1, 2 * n, 4), 1] += 2.0
        assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(ft), gymtorch.unwrap_tensor(tq),
                                                  gymapi.ENV_SPACE)
        gym.simulate(sim)
        oracle.step(p, m, st, dof, ext=ext, contact_cache=cc)
    gym.refresh_rigid_body_state_tensor(sim)
    got = rb.cpu().numpy()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
    moved = np.abs(st[1::2, 0] - x0)
    assert np.all(moved[pushes < 1.0] < 2e-3) and np.all(moved[pushes > 1.0] > 0.05)


def _yup_vehicle_scene(gym, n):
    """Isaac Gym's default y-up sim (UP_AXIS_Y, gravity -y, plane normal +y) with
    one ground vehicle per env: the ground-patch rows take the general-normal
    path (mg_rigid.hip BasisGen anchors), not the packed +Z one."""
    sp = scenes.servo_sim_params(True)
    sp.up_axis = gymapi.UP_AXIS_Y
    sp.gravity = gymapi.Vec3(0.0, -9.8, 0.0)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 1, 0)
    plane.static_friction = 1
    plane.dynamic_friction = 1
    gym.add_ground(sim, plane)
    opts = gymapi.AssetOptions()
    opts.armature = 0.01
    veh = gym.load_asset(sim, scenes.ASSET_ROOT, "servo/ground_vehicle.urdf", opts)
    rng = np.random.RandomState(3)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-20, 0, -20), gymapi.Vec3(20, 20, 20), 8)
        pose = gymapi.Transform()
        pose.p = gymapi.Vec3(0.0, 1.35 + 0.1 * rng.rand(), 0.0)
        # upright (the body's z axis on +y), turned about +y by a random yaw. Round
        # 5 left the body's z horizontal: the vehicle then stood 3 m tall on a
        # 2.5 m base, which tips at 2.5 / (2 * 1.5) = 0.83 mu m g — a push at 0.9
        # across that base tipped it, which the test read as sliding
        pose.r = (gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 1, 0), float(rng.uniform(-np.pi, np.pi))) *
                  gymapi.Quat.from_axis_angle(gymapi.Vec3(1, 0, 0), -0.5 * np.pi))
        gym.create_actor(env, veh, pose, "veh%d" % i, i, -1)
    return sim


def test_yup_ground_patch_pushes_bitexact(gym):
    """y-up ground: randomly yawed upright vehicles land on the plane and are
    pushed along x / z (the basis directions t2 / t1 of the +y ground) at 0.5 /
    0.9 / 1.1 / 1.5 mu m g; GPU == oracle bit for bit including the net contact
    force, every frame. Held (< 2 mm) at 0.5 and 0.9 whatever the yaw, sliding
    at 1.1 and 1.5. Round 5's sweep order let yawed vehicles creep at 0.9 (the
    normal rows solved before the anchors' rows left a rotation about the line
    through the two anchors in the integrated velocity; VERDICT r05 item 1,
    tests/test_ground_patch_kat.py). Parity with PhysX unpinned."""
    n, settle, frames = 64, 45, 45
    sim = _yup_vehicle_scene(gym, n)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    A = sim.model_arrays
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    for k in range(settle):
        gym.simulate(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        cf = oracle.step(p, m, st, dof, contact_cache=cc)
        assert np.array_equal(rb.cpu().numpy(), st), "settle frame %d" % k
        assert np.array_equal(ncf.cpu().numpy(), cf), "settle frame %d: contact force" % k
    assert int((cc.body[:, 0] == 2.0).sum()) == n          # every vehicle rests on two anchors
    mu = 0.5 * (float(A["shapes"][int(A["tmpl_body_i"][A["body_tmpl"][0]][0])][11]) + 1.0)
    pushes = np.array([0.5, 0.9, 1.1, 1.5], np.float32)[np.arange(n) % 4]
    force = np.zeros((n, 3), np.float32)
    along_z = np.arange(n) % 8 >= 4
    force[~along_z, 0] = pushes[~along_z] * mu * 100.0 * 9.8
    force[along_z, 2] = pushes[along_z] * mu * 100.0 * 9.8
    ext = np.zeros((n, 6), np.float32)
    ext[:, 0:3] = force
    ft = torch.from_numpy(force).to(DEV)
    tq = torch.zeros_like(ft)
    x0 = st[:, [0, 2]].copy()
    for k in range(frames):
        assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(ft), gymtorch.unwrap_tensor(tq),
                                                  gymapi.ENV_SPACE)
        gym.simulate(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        cf = oracle.step(p, m, st, dof, ext=ext, contact_cache=cc)
        assert np.array_equal(rb.cpu().numpy(), st), "push frame %d: max |diff| %g" % (
            k, np.abs(rb.cpu().numpy() - st).max())
        assert np.array_equal(ncf.cpu().numpy(), cf), "push frame %d: contact force" % k
    moved = np.linalg.norm(st[:, [0, 2]] - x0, axis=1)
    assert np.all(moved[pushes < 1.0] < 2e-3), moved[pushes < 1.0]
    assert np.all(moved[pushes > 1.0] > 0.05)


def test_yawed_vehicle_pushes_bitexact(gym):
    """z-up (the packed +Z solver, tgs_zp): the servo scene's vehicles teleported
    upright to random yaws, settled, then pushed along world x or y at 0.9 /
    0.95 / 1.05 / 1.5 mu m g. GPU == oracle bit for bit (state, contact force)
    every frame; held (< 2 mm, < 0.1 mm over the last 40 frames) below mu m g at
    every yaw, sliding above. S1's actions teleport every vehicle to a random
    yaw every step, so the headline workload's friction depends
    on this; round 5's sweep order let 0.9 mu m g pushes across the anchors'
    line creep."""
    n, settle, frames = 128, 60, 90
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    A = sim.model_arrays
    st = A["body_state0"].copy()
    roots = A["actor_root_body"]
    veh = roots[1::2]
    dof = np.zeros((0, 2), np.float32)
    yaw = np.random.RandomState(11).uniform(-np.pi, np.pi, n).astype(np.float32)
    quat = np.zeros((n, 4), np.float32)
    quat[:, 2] = np.sin(0.5 * yaw)
    quat[:, 3] = np.cos(0.5 * yaw)
    gym.refresh_actor_root_state_tensor(sim)
    root[1::2, 2] = 1.3
    root[1::2, 3:7] = torch.from_numpy(quat).to(DEV)
    root[1::2, 7:13] = 0.0
    assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
    st[veh, 2] = 1.3
    st[veh, 3:7] = quat
    st[veh, 7:13] = 0.0
    for k in range(settle):
        gym.simulate(sim)
        oracle.step(p, m, st, dof, contact_cache=cc)
    gym.refresh_rigid_body_state_tensor(sim)
    assert np.array_equal(rb.cpu().numpy(), st)
    assert np.all(cc.body[veh, 0] == 2.0)
    mu = 0.5 * (float(A["shapes"][int(A["tmpl_body_i"][A["body_tmpl"][veh[0]]][0])][11]) + 1.0)
    pushes = np.array([0.9, 0.95, 1.05, 1.5], np.float32)[np.arange(n) % 4]
    along_y = np.arange(n) % 8 >= 4
    nb = st.shape[0]
    force = np.zeros((nb, 3), np.float32)
    force[veh[~along_y], 0] = pushes[~along_y] * mu * 100.0 * 9.8
    force[veh[along_y], 1] = pushes[along_y] * mu * 100.0 * 9.8
    ext = np.zeros((nb, 6), np.float32)
    ext[:, 0:3] = force
    ft = torch.from_numpy(force).to(DEV)
    tq = torch.zeros_like(ft)
    x0 = st[veh, 0:2].copy()
    for k in range(frames):
        if k == frames - 40:
            x50 = st[veh, 0:2].copy()
        assert gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(ft), gymtorch.unwrap_tensor(tq),
                                                  gymapi.ENV_SPACE)
        gym.simulate(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        cf = oracle.step(p, m, st, dof, ext=ext, contact_cache=cc)
        got = rb.cpu().numpy()
        assert np.array_equal(got, st), "push frame %d: max |diff| %g" % (k, np.abs(got - st).max())
        assert np.array_equal(ncf.cpu().numpy(), cf), "push frame %d: contact force" % k
    moved = np.linalg.norm(st[veh, 0:2] - x0, axis=1)
    late = np.linalg.norm(st[veh, 0:2] - x50, axis=1)
    assert np.all(moved[pushes < 1.0] < 2e-3), moved[pushes < 1.0]
    assert np.all(late[pushes < 1.0] < 1e-4), late[pushes < 1.0]   # f32 ulps of x ~ 100 m
    assert np.all(moved[pushes > 1.0] > 0.05)


def test_reset_in_place_keeps_patch_bitexact(gym):
    """A root-state set that moves a resting vehicle by less than the friction
    correlation distance (0.2 mm here, the default distance is 25 mm) keeps its
    patch: the anchors are kept across teleports on purpose, as PhysX keeps a
    pair's friction patches across setGlobalPose and drops an anchor only when
    its two copies drift apart. A 5 cm move drops them. GPU
    == oracle bit for bit, anchors included."""
    n = 64
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    st = sim.model_arrays["body_state0"].copy()
    roots = sim.model_arrays["actor_root_body"]
    dof = np.zeros((0, 2), np.float32)
    for _ in range(60):
        gym.simulate(sim)
        oracle.step(p, m, st, dof, contact_cache=cc)
    veh = roots[1::2]
    assert np.all(cc.body[veh, 0] == 2.0)
    before = cc.body[veh].copy()
    gym.refresh_actor_root_state_tensor(sim)
    for shift in (0.0002, 0.05):
        root[1::2, 0] += shift
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        st[veh, 0] += shift
        for _ in range(3):
            gym.simulate(sim)
            oracle.step(p, m, st, dof, contact_cache=cc)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_actor_root_state_tensor(sim)
        assert np.array_equal(rb.cpu().numpy(), st), "shift %g" % shift
        if shift < 0.025:   # the held anchors are the ones made before the set, bit for bit
            assert np.array_equal(cc.body[veh, 4:], before[:, 4:])
