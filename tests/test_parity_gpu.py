"""GPU parity: the HIP step kernels (through the C ABI, driven by the gymapi
tensor API exactly like test10_servo_vecenv.py:376-456) against the C
restatement in oracle/ on the same inputs.

Tolerance: the device and the oracle evaluate the same fp32 expressions in the
same order with FMA contraction off, so the expected difference is zero; the
hard assertion is |gpu - oracle| <= 1e-5 * max(1, |x|) per element (positions
up to ~1e3 m, velocities up to 1e3 m/s), and bit-exactness is asserted
separately so a drift in either build shows up by name.
"""
import os

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import scenes
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
RTOL = 1e-5


def _close(a, b):
    return np.abs(a - b) <= RTOL * np.maximum(1.0, np.abs(b))


def _tensors(gym, sim):
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    return root, rb, dof, ncf


def test_servo_single_step_parity(gym):
    """Every step starts the oracle from the device's own state (after the
    root teleport), so each simulate() is compared on identical inputs."""
    n, steps = 256, 40
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root, rb, _, ncf = _tensors(gym, sim)
    acts = scenes.servo_actions(n, steps, DEV, seed=1)
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)      # the ground patches persist from step to step, as on the device
    gym.refresh_actor_root_state_tensor(sim)
    worst = 0.0
    exact = True
    for k in range(steps):
        root[:, 3:10] = acts[k]
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.refresh_rigid_body_state_tensor(sim)
        inp = rb.cpu().numpy().copy()
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        gym.refresh_actor_root_state_tensor(sim)
        got = rb.cpu().numpy()
        cf = oracle.step(p, m, inp, np.zeros((0, 2), np.float32), contact_cache=cc)
        assert np.all(_close(got, inp)), "step %d: max |diff| %g" % (k, np.abs(got - inp).max())
        assert np.all(_close(ncf.cpu().numpy(), cf))
        worst = max(worst, float(np.abs(got - inp).max()))
        exact = exact and np.array_equal(got, inp) and np.array_equal(ncf.cpu().numpy(), cf)
    assert exact, "within tolerance but not bit-exact (max |diff| %g)" % worst


def test_servo_large_launch_step_parity(gym):
    """131072 envs = 262144 single-shape bodies = 4096 waves, more than one
    resident round of k_rigid_step1, so the launch dispatches back to front
    (mg_launch_rigid_step): still bit for bit the oracle's step."""
    n, steps = 131072, 2
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root, rb, _, ncf = _tensors(gym, sim)
    acts = scenes.servo_actions(n, steps, DEV, seed=3)
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(steps):
        root[:, 3:10] = acts[k]
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.refresh_rigid_body_state_tensor(sim)
        inp = rb.cpu().numpy().copy()
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        got = rb.cpu().numpy()
        cf = oracle.step(p, m, inp, np.zeros((0, 2), np.float32), contact_cache=cc)
        assert np.array_equal(got, inp), "step %d: max |diff| %g" % (k, np.abs(got - inp).max())
        assert np.array_equal(ncf.cpu().numpy(), cf)


def test_servo_large_launch_fused_rows(gym):
    """The wide launch with the refresh fused into the step (STEP_FUSION_ALL):
    each wave writes its 64 rows through an LDS transpose (k_rigid_step1's wide
    branch); the root and rigid-body tensors equal the unfused sequence's bit
    for bit."""
    n, steps = 131072, 3
    acts = scenes.servo_actions(n, steps, DEV, seed=5)
    sims = []
    for fusion in (gymapi.STEP_FUSION_ALL, 0):
        sim, _ = scenes.servo_scene(gym, n)
        gym.prepare_sim(sim)
        gym.set_step_fusion(sim, fusion)
        sims.append((sim, _tensors(gym, sim)))
        gym.refresh_actor_root_state_tensor(sim)
    for k in range(steps):
        for sim, (root, _, _, _) in sims:
            root[:, 3:10] = acts[k]
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            gym.simulate(sim)
            gym.refresh_actor_root_state_tensor(sim)
            gym.refresh_rigid_body_state_tensor(sim)
        torch.cuda.synchronize()
        (ra, rba, _, _), (rb_, rbb, _, _) = sims[0][1], sims[1][1]
        assert torch.equal(ra, rb_), "step %d: root state differs" % k
        assert torch.equal(rba, rbb), "step %d: rigid-body state differs" % k
    for sim, _ in sims:
        gym.destroy_sim(sim)


def test_fused_step_matches_unfused(gym):
    """Step fusion (mg_set_fusion): the root-state set read by the step kernel
    and the paired root + rigid-body refresh give the same tensors, bit for bit,
    as the scatter / two-gather sequence; a reader between set and simulate
    sees the set rows (the deferred set is flushed first)."""
    from test_isaacgym_amd import _native as N
    n, steps = 512, 24
    sims = []
    for fused in (True, False):
        sim, _ = scenes.servo_scene(gym, n)
        gym.prepare_sim(sim)
        if fused:
            gym.set_step_fusion(sim, gymapi.STEP_FUSION_ALL)
        sims.append((sim, _tensors(gym, sim)))
    acts = scenes.servo_actions(n, steps, DEV, seed=4)
    for sim, (root, _, _, _) in sims:
        gym.refresh_actor_root_state_tensor(sim)
    for k in range(steps):
        for sim, (root, rb, _, _) in sims:
            root[:, 3:10] = acts[k]
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            gym.simulate(sim)
            gym.fetch_results(sim, True)
            gym.refresh_actor_root_state_tensor(sim)
            gym.refresh_rigid_body_state_tensor(sim)
        (ra, rba, _, _), (rb_, rbb, _, _) = sims[0][1], sims[1][1]
        assert torch.equal(ra, rb_), "step %d: root state differs" % k
        assert torch.equal(rba, rbb), "step %d: rigid-body state differs" % k
    # set, then read before simulate: the reader sees the set rows
    sim, (root, rb, _, _) = sims[0]
    want = root.clone()
    want[:, 0:3] += 1.0
    root.copy_(want)
    assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
    gym.refresh_rigid_body_state_tensor(sim)
    roots = torch.as_tensor(sim.model_arrays["actor_root_body"], device=DEV, dtype=torch.long)
    assert torch.equal(rb[roots], want)
    root.zero_()
    gym.refresh_actor_root_state_tensor(sim)
    assert torch.equal(root, want)


def test_step_out_fusion(gym):
    """STEP_FUSION_STEP_OUT (the refresh fused into the step, include/migym.h
    MG_FUSE_STEP_OUT): simulate writes the bound root and rigid-body tensors
    itself. Eager and in a captured hipGraph the tensors equal the unfused
    set / simulate / refresh sequence bit for bit; a tensor the user writes
    between simulate and its refresh is re-gathered by the refresh (Isaac Gym's
    refresh overwrites it); the rigid-body refresh serves the step's rows."""
    n, steps, chunk = 256, 12, 4
    acts = scenes.servo_actions(n, steps, DEV, seed=11)
    sims = []
    for fusion in (gymapi.STEP_FUSION_ALL, 0):
        sim, _ = scenes.servo_scene(gym, n)
        gym.prepare_sim(sim)
        gym.set_step_fusion(sim, fusion)
        sims.append((sim, _tensors(gym, sim)))
        gym.refresh_actor_root_state_tensor(sim)

    def step(sim, root, k):
        root[:, 3:10] = acts[k]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, False)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)

    (sa, (ra, rba, _, _)), (sb, (rb_, rbb, _, _)) = sims
    for k in range(chunk):            # eager
        step(sa, ra, k)
        step(sb, rb_, k)
        torch.cuda.synchronize()
        assert torch.equal(ra, rb_) and torch.equal(rba, rbb), "eager step %d" % k
    # captured: `chunk` steps per graph, replayed; the unfused sim steps eagerly
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for j in range(chunk):
                step(sa, ra, chunk + j)
    torch.cuda.current_stream().wait_stream(side)
    g.replay()
    for j in range(chunk):
        step(sb, rb_, chunk + j)
    torch.cuda.synchronize()
    assert torch.equal(ra, rb_) and torch.equal(rba, rbb), "captured steps"
    # a write between simulate and refresh: the refresh restores the state
    for sim, (root, rb, _, _) in sims:
        root[:, 3:10] = acts[2 * chunk]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        root.fill_(-3.0)
        rb[:, 5] = 9.0
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
    torch.cuda.synchronize()
    assert torch.equal(ra, rb_) and torch.equal(rba, rbb), "refresh after a user write"
    assert not torch.any(ra == -3.0)
    # the refreshes after the step read the same rows the step wrote
    roots = torch.as_tensor(sa.model_arrays["actor_root_body"], device=DEV, dtype=torch.long)
    assert torch.equal(rba[roots], ra)
    for sim, _ in sims:
        gym.destroy_sim(sim)


def test_step_fusion_copy_at_set_contract(gym):
    """Isaac Gym reads a set_*_tensor source during the set call (SURVEY.md §8b
    Ownership). With step fusion off (the default) a source written after its
    set and before simulate does not reach the step: the result equals a sim
    given an untouched copy, bit for bit. With fusion on (opt-in) that write
    raises MigymError instead of being read. Same for DOF position targets. A
    rigid-body tensor edited by the user survives a root refresh (fusion off),
    and with fusion on a later rigid-body refresh re-gathers the edited tensor."""
    from test_isaacgym_amd import _native as N
    n = 64
    acts = scenes.servo_actions(n, 2, DEV, seed=9)
    outs = []
    for mode in ("copy", "write_after_set"):
        sim, _ = scenes.servo_scene(gym, n)
        gym.prepare_sim(sim)
        root, rb, _, _ = _tensors(gym, sim)
        gym.refresh_actor_root_state_tensor(sim)
        root[:, 3:10] = acts[0]
        src = root.clone()
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(src))
        if mode == "write_after_set":
            src[:, 3:10] = acts[1]          # too late: the set already took its copy
        gym.simulate(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        outs.append(rb.clone())
        # user edits to the rigid-body tensor survive a root refresh (no fusion)
        rb[:, 0] = -7.0
        gym.refresh_actor_root_state_tensor(sim)
        assert torch.all(rb[:, 0] == -7.0)
        gym.destroy_sim(sim)
    assert torch.equal(outs[0], outs[1])
    # fusion on: the same write raises at simulate; an edited rb tensor is re-gathered
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    gym.set_step_fusion(sim, gymapi.STEP_FUSION_ALL)
    root, rb, _, _ = _tensors(gym, sim)
    gym.refresh_actor_root_state_tensor(sim)
    src = root.clone()
    src[:, 3:10] = acts[0]
    assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(src))
    src[:, 3:10] = acts[1]
    with pytest.raises(N.MigymError):
        gym.simulate(sim)
    assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(src))
    gym.simulate(sim)
    gym.refresh_actor_root_state_tensor(sim)       # fused: fills rb as well
    want = rb.clone()
    rb[:, 0] = -7.0
    gym.refresh_rigid_body_state_tensor(sim)
    assert torch.equal(rb, want)
    gym.destroy_sim(sim)
    # DOF position targets
    tg = scenes.gimbal_targets(16, 2, DEV, seed=3)
    douts = []
    for fusion in (0, gymapi.STEP_FUSION_ALL):
        for write_after in (False, True):
            sim, _ = scenes.gimbal_scene(gym, 16)
            gym.prepare_sim(sim)
            gym.set_step_fusion(sim, fusion)
            dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
            t = tg[0].clone()
            assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(t))
            if write_after:
                t.copy_(tg[1])
            if fusion and write_after:
                with pytest.raises(N.MigymError):
                    gym.simulate(sim)
            else:
                gym.simulate(sim)
                gym.refresh_dof_state_tensor(sim)
                douts.append(dof.clone())
            gym.destroy_sim(sim)
    assert len(douts) == 3
    assert torch.equal(douts[0], douts[1]) and torch.equal(douts[0], douts[2])


def test_servo_trajectory_bitexact(gym):
    """A 120-frame rollout with a random root teleport every frame, device vs
    oracle from the same initial state: no re-synchronisation."""
    n, steps = 128, 120
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root, rb, _, _ = _tensors(gym, sim)
    acts = scenes.servo_actions(n, steps, DEV, seed=2)
    acts_h = acts.cpu().numpy()
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    roots = sim.model_arrays["actor_root_body"]
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(steps):
        root[:, 3:10] = acts[k]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_actor_root_state_tensor(sim)
        # oracle: the same teleport of every root row, then the step
        st[roots, 3:10] = acts_h[k]
        oracle.step(p, m, st, np.zeros((0, 2), np.float32))
    gym.refresh_rigid_body_state_tensor(sim)
    got = rb.cpu().numpy()
    assert np.all(np.isfinite(got))
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


def test_primitive_drops_parity(gym):
    """Boxes, spheres and capsules dropped at random orientations onto the
    ground: every contact branch of the kernel, 240 frames, bit for bit."""
    sp = scenes.servo_sim_params(True)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    plane.restitution = 0.5
    gym.add_ground(sim, plane)
    assets = [gym.create_box(sim, 1.0, 0.5, 0.3, gymapi.AssetOptions()),
              gym.create_sphere(sim, 0.3, gymapi.AssetOptions()),
              gym.create_capsule(sim, 0.2, 0.8, gymapi.AssetOptions())]
    rng = np.random.RandomState(42)
    for i in range(96):
        env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 10)
        q = gymapi.Quat(*rng.randn(4)).normalize()
        pose = gymapi.Transform(gymapi.Vec3(0, 0, 0.5 + 2 * rng.rand()), q)
        gym.create_actor(env, assets[i % 3], pose, "obj", i, 0)
    gym.prepare_sim(sim)
    _, rb, _, ncf = _tensors(gym, sim)
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    for _ in range(240):
        gym.simulate(sim)
        cf = oracle.step(p, m, st, np.zeros((0, 2), np.float32))
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_net_contact_force_tensor(sim)
    got = rb.cpu().numpy()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
    assert np.array_equal(ncf.cpu().numpy(), cf)
    # physics sanity: everything came to rest on the ground
    assert np.all(got[:, 2] > 0.05) and np.all(got[:, 2] < 0.6)


def _mesh_urdf(tmp, name, verts, extra_box=False):
    """A single-link URDF whose collision is a mesh (vertex-only OBJ) and
    optionally a box as a second shape."""
    with open(os.path.join(tmp, name + ".obj"), "w") as f:
        for v in verts:
            f.write("v %.9g %.9g %.9g\n" % tuple(v))
    box = ('<collision><origin xyz="0 0 0.15"/><geometry><box size="0.2 0.1 0.1"/></geometry></collision>'
           if extra_box else "")
    with open(os.path.join(tmp, name + ".urdf"), "w") as f:
        f.write('<robot name="%s"><link name="body"><collision><origin xyz="0.02 0 0" rpy="0.3 0 0"/>'
                '<geometry><mesh filename="%s.obj"/></geometry></collision>%s</link></robot>' % (name, name, box))
    return name + ".urdf"


def test_hull_drops_parity(gym, tmp_path):
    """Convex-hull free bodies (random point clouds -> hulls of <= 32 vertices;
    one single-shape, one hull + box) dropped onto the ground: the hull branch
    of the free-body kernel (static and shift-register slots), 180 frames, bit
    for bit."""
    rng = np.random.RandomState(5)
    files = []
    for k in range(3):
        pts = rng.normal(size=(60, 3)) * np.array([0.15, 0.1, 0.08])
        files.append(_mesh_urdf(str(tmp_path), "cloud%d" % k, pts, extra_box=(k == 2)))
    sp = scenes.servo_sim_params(True)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    assets = [gym.load_asset(sim, str(tmp_path), f, gymapi.AssetOptions()) for f in files]
    assert all(a.bodies[0].shapes[0].type == 3 for a in assets)
    for i in range(48):
        env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 8)
        q = gymapi.Quat(*rng.randn(4)).normalize()
        pose = gymapi.Transform(gymapi.Vec3(0, 0, 0.3 + rng.rand()), q)
        gym.create_actor(env, assets[i % 3], pose, "obj", i, 0)
    gym.prepare_sim(sim)
    _, rb, _, ncf = _tensors(gym, sim)
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    for _ in range(180):
        gym.simulate(sim)
        cf = oracle.step(p, m, st, np.zeros((0, 2), np.float32))
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_net_contact_force_tensor(sim)
    got = rb.cpu().numpy()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
    assert np.array_equal(ncf.cpu().numpy(), cf)
    assert np.all(got[:, 2] > 0.0) and np.all(got[:, 2] < 0.5)          # at rest on the ground
    assert np.all(np.abs(got[:, 7:10]) < 0.05)


def test_decomposed_mesh_drops_parity(gym, tmp_path):
    """A concave mesh split into convex hulls (AssetOptions.vhacd_enabled: a U
    of 3 pieces, a multi-shape body) dropped onto the ground at random poses:
    the free-body kernel's shift-register slots over several hulls, bit for bit
    the oracle, and at rest."""
    import test_importer
    f = test_importer._u_urdf(str(tmp_path), scale=0.1)
    sp = scenes.servo_sim_params(True)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    opts = gymapi.AssetOptions()
    opts.vhacd_enabled = True
    opts.vhacd_params.max_convex_hulls = 4
    asset = gym.load_asset(sim, str(tmp_path), f, opts)
    assert len(asset.bodies[0].shapes) >= 2
    rng = np.random.RandomState(7)
    for i in range(32):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 8)
        q = gymapi.Quat(*rng.randn(4)).normalize()
        gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 0.4 + 0.3 * rng.rand()), q), "u", i, 0)
    gym.prepare_sim(sim)
    _, rb, _, ncf = _tensors(gym, sim)
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    for _ in range(150):
        gym.simulate(sim)
        cf = oracle.step(p, m, st, np.zeros((0, 2), np.float32))
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_net_contact_force_tensor(sim)
    got = rb.cpu().numpy()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()
    assert np.array_equal(ncf.cpu().numpy(), cf)
    assert np.all(got[:, 2] > 0.0) and np.all(got[:, 2] < 0.4)


def test_gimbal_parity(gym):
    """S2: the 3-DOF camera gimbal under random PD position targets."""
    n, steps = 256, 60
    sim, _ = scenes.gimbal_scene(gym, n)
    gym.prepare_sim(sim)
    _, rb, dof, _ = _tensors(gym, sim)
    tg = scenes.gimbal_targets(n, steps, DEV, seed=3)
    tg_h = tg.cpu().numpy()
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    for k in range(steps):
        t = tg[k].contiguous()
        assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(t))
        gym.simulate(sim)
        tgt[:, 0] = tg_h[k]
        oracle.step(p, m, st, ds, tgt=tgt)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d = dof.cpu().numpy()
    got = rb.cpu().numpy()
    assert np.all(np.isfinite(got_d))
    assert np.all(_close(got_d, ds)) and np.all(_close(got, st))
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


def test_gimbal_effort_limit_parity(gym):
    """Stiff, lightly damped PD drives (kp 2000, kd 0.5) on 10 kg links against the URDF's 10 N m effort limit:
    the implicit drive force exceeds the limit, so the articulated-body pass is
    re-solved with those drives at constant +-effort — bit for
    bit the oracle's re-solve."""
    n, steps = 128, 40
    sim, _ = scenes.gimbal_scene(gym, n, stiffness=2000.0, damping=0.5, link_mass_scale=1000.0)
    gym.prepare_sim(sim)
    _, rb, dof, _ = _tensors(gym, sim)
    tg = scenes.gimbal_targets(n, steps, DEV, seed=5)
    tg_h = tg.cpu().numpy()
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    for k in range(steps):
        assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k].contiguous()))
        gym.simulate(sim)
        tgt[:, 0] = tg_h[k]
        oracle.step(p, m, st, ds, tgt=tgt)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    assert np.all(np.isfinite(got_d))
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


def _tree_urdf(d):
    """A fixed base with two revolute branches of two links each (not a serial
    chain: the lane-parallel articulation kernel), 5 kg links, 20 N m limits."""
    link = ('<link name="%s"><inertial><origin xyz="0.2 0 0"/><mass value="5"/>'
            '<inertia ixx="0.02" iyy="0.08" izz="0.08" ixy="0" ixz="0" iyz="0"/></inertial>'
            '<collision><origin xyz="0.2 0 0"/><geometry><box size="0.4 0.05 0.05"/></geometry></collision></link>')
    joint = ('<joint name="%s" type="revolute"><parent link="%s"/><child link="%s"/>'
             '<origin xyz="%s" rpy="0 0 0"/><axis xyz="%s"/><limit lower="-2" upper="2" effort="20" velocity="50"/></joint>')
    body = ['<link name="base"><inertial><mass value="1"/><inertia ixx="0.01" iyy="0.01" izz="0.01" ixy="0" ixz="0" iyz="0"/>'
            '</inertial></link>']
    body += [link % n for n in ("a1", "a2", "b1", "b2")]
    body += [joint % ("ja1", "base", "a1", "0 0 0", "0 0 1"), joint % ("ja2", "a1", "a2", "0.4 0 0", "0 1 0"),
             joint % ("jb1", "base", "b1", "0 0 0.1", "0 0 1"), joint % ("jb2", "b1", "b2", "0.4 0 0", "1 0 0")]
    with open(os.path.join(d, "tree.urdf"), "w") as f:
        f.write('<robot name="tree">' + "".join(body) + "</robot>")
    return "tree.urdf"


def test_tree_effort_limit_parity(gym, tmp_path):
    """A branched articulation (k_artic_lanes, not the chain kernel) with stiff
    drives on heavy links: the effort-limit re-solve of the lane-parallel
    articulated-body pass, bit for bit the oracle."""
    sp = gymapi.SimParams()
    sp.dt, sp.substeps = 1.0 / 60.0, 2
    sp.gravity = gymapi.Vec3(0.0, 0.0, -9.8)
    sp.physx.solver_type = 1
    sp.use_gpu_pipeline = True
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    asset = gym.load_asset(sim, str(tmp_path), _tree_urdf(str(tmp_path)), opts)
    n, steps = 64, 40
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 8)
        h = gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 1)), "tree", i, 1)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_POS
        props["stiffness"][:] = 3000.0
        props["damping"][:] = 1.0
        gym.set_actor_dof_properties(env, h, props)
    gym.prepare_sim(sim)
    _, rb, dof, _ = _tensors(gym, sim)
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    rng = np.random.RandomState(11)
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    for k in range(steps):
        tgt[:, 0] = rng.uniform(-1.5, 1.5, size=ds.shape[0]).astype(np.float32)
        assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(tgt[:, 0].copy()).to(DEV)))
        gym.simulate(sim)
        oracle.step(p, m, st, ds, tgt=tgt)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
    assert np.all(np.isfinite(got_d))
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


def test_gimbal_velocity_drive_parity(gym):
    """DOF_MODE_VEL (examples/dof_controls.py:89-150: velocity targets, the
    stiffness is ignored, damping drives the joint speed): random velocity
    targets through set_dof_velocity_target_tensor, every other frame only the
    odd envs' targets through the _indexed setter; 60 frames bit for bit."""
    n, steps = 128, 60
    sim, _ = scenes.gimbal_scene(gym, n, drive_mode=gymapi.DOF_MODE_VEL, stiffness=50.0, damping=2.0)
    gym.prepare_sim(sim)
    _, rb, dof, _ = _tensors(gym, sim)
    tg = scenes.gimbal_targets(n, steps, DEV, seed=7) * 2.0
    tg_h = tg.cpu().numpy()
    odd = torch.arange(1, n, 2, dtype=torch.int32, device=DEV)
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    for k in range(steps):
        t = tg[k].contiguous()
        if k % 2 == 0:
            assert gym.set_dof_velocity_target_tensor(sim, gymtorch.unwrap_tensor(t))
            tgt[:, 1] = tg_h[k]
        else:
            assert gym.set_dof_velocity_target_tensor_indexed(sim, gymtorch.unwrap_tensor(t),
                                                               gymtorch.unwrap_tensor(odd), odd.numel())
            rows = (np.arange(1, n, 2)[:, None] * 3 + np.arange(3)[None, :]).ravel()
            tgt[rows, 1] = tg_h[k][rows]
        gym.simulate(sim)
        oracle.step(p, m, st, ds, tgt=tgt)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    got_d = dof.cpu().numpy()
    got = rb.cpu().numpy()
    assert np.all(np.isfinite(got_d)) and np.abs(got_d[:, 1]).max() > 0.1       # the drives moved the joints
    assert np.array_equal(got_d, ds), "max |diff| %g" % np.abs(got_d - ds).max()
    assert np.array_equal(got, st), "max |diff| %g" % np.abs(got - st).max()


def test_tensor_api_semantics(gym):
    """acquire returns one persistent storage (test10 :372 vs :400); refresh
    publishes the step; the _indexed setter touches only the listed actors; the
    CPU pipeline (host tensors, test10's mode) gives the same numbers."""
    n = 64
    sims = {}
    for gpu_pipe in (True, False):
        sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=gpu_pipe)
        gym.prepare_sim(sim)
        t1 = gym.acquire_actor_root_state_tensor(sim)
        t2 = gym.acquire_actor_root_state_tensor(sim)
        assert t1.data_address == t2.data_address
        root = gymtorch.wrap_tensor(t1)
        assert root.data_ptr() == t1.data_address
        assert root.device.type == ("cuda" if gpu_pipe else "cpu")
        before = root.clone()
        gym.simulate(sim)
        assert torch.equal(root, before)        # not refreshed yet
        gym.refresh_actor_root_state_tensor(sim)
        assert not torch.equal(root, before)    # the vehicles fell
        sims[gpu_pipe] = (sim, root)
    assert np.array_equal(sims[True][1].cpu().numpy(), sims[False][1].numpy())

    sim, root = sims[True]
    gym.refresh_actor_root_state_tensor(sim)
    new = root.clone()
    new[:, 2] += 5.0
    idx = torch.tensor([3, 10, 11], dtype=torch.int32, device=DEV)
    assert gym.set_actor_root_state_tensor_indexed(sim, gymtorch.unwrap_tensor(new), gymtorch.unwrap_tensor(idx), 3)
    expect = root.clone()
    expect[idx.long()] = new[idx.long()]
    gym.refresh_actor_root_state_tensor(sim)
    assert torch.equal(root, expect)
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    assert dof.shape == (0, 2)
    assert gym.refresh_dof_state_tensor(sim)


def test_servo_4096_properties(gym):
    """The bench workload (4096 envs): 30 frames of random teleports, then every
    root is stopped (v = w = 0) with the vehicles levelled; 15 s later the
    vehicles rest flat on the ground (box proxy half-height 1.25 m). Two sims
    must agree bit for bit; state stays finite with unit quaternions."""
    n = 4096
    outs = []
    for _ in range(2):
        sim, _ = scenes.servo_scene(gym, n)
        gym.prepare_sim(sim)
        root, rb, _, _ = _tensors(gym, sim)
        acts = scenes.servo_actions(n, 30, DEV, seed=4)
        gym.refresh_actor_root_state_tensor(sim)
        for k in range(30):
            root[:, 3:10] = acts[k]
            gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            gym.simulate(sim)
            gym.refresh_actor_root_state_tensor(sim)
        root[:, 7:13] = 0.0
        root[1::2, 3:7] = acts[29, 1::2, 0:4]          # vehicle: yaw-only attitude
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        for _ in range(900):
            gym.simulate(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        outs.append(rb.cpu().numpy().copy())
        gym.destroy_sim(sim)
    a, b = outs
    assert np.array_equal(a, b)
    assert np.all(np.isfinite(a))
    qn = np.linalg.norm(a[:, 3:7], axis=1)
    assert np.all(np.abs(qn - 1) < 1e-5)
    car = a[1::2]
    assert np.all(np.abs(car[:, 2] - 1.25) < 0.01), (car[:, 2].min(), car[:, 2].max())
    assert np.all(np.abs(car[:, 7:10]) < 0.01), np.abs(car[:, 7:10]).max()


def _np_quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def _np_rot(q, v):
    x, y, z, w = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    return R @ v


def test_gimbal_jacobian_matches_float64_kinematics(gym):
    """refresh_jacobian_tensors (examples/franka_cube_ik_osc.py:305-311) at random
    joint angles vs a float64 forward-kinematics Jacobian of the link origins:
    atol 1e-5 (unit-scale lever arms)."""
    n = 32
    sim, envs = scenes.gimbal_scene(gym, n)
    gym.prepare_sim(sim)
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    jac = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, "gimbal"))
    assert tuple(jac.shape) == (n, 3, 6, 3)
    rng = np.random.RandomState(0)
    q = rng.uniform(-1.5, 1.5, (n, 3)).astype(np.float32)
    st = torch.zeros((3 * n, 2), dtype=torch.float32, device=DEV)
    st[:, 0] = torch.from_numpy(q.reshape(-1)).to(DEV)
    assert gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(st))
    gym.refresh_jacobian_tensors(sim)
    J = jac.cpu().numpy()
    asset = sim.assets[0]
    base = sim.model_arrays["body_state0"][0::4]
    for e in range(n):
        ps, qs, zs = [base[e, 0:3].astype(np.float64)], [base[e, 3:7].astype(np.float64)], [None]
        for k, j in enumerate(asset.joints):
            th = float(q[e, k])
            qrel = _np_quat_mul(j.q, np.r_[j.axis * np.sin(th / 2), np.cos(th / 2)])
            ps.append(ps[j.parent] + _np_rot(qs[j.parent], j.p))
            qs.append(_np_quat_mul(qs[j.parent], qrel))
            zs.append(_np_rot(qs[-1], j.axis))
        for l in range(1, 4):
            ref = np.zeros((6, 3))
            for jl in range(1, l + 1):                 # the gimbal is a chain: ancestors 1..l
                ref[:3, jl - 1] = np.cross(zs[jl], ps[l] - ps[jl])
                ref[3:, jl - 1] = zs[jl]
            np.testing.assert_allclose(J[e, l - 1], ref, atol=1e-5)


def test_mass_matrix_consistent_with_aba(gym):
    """CRBA mass matrix (refresh_mass_matrix_tensors) against the ABA step: from
    rest, gravity off, one substep of h with unit EFFORT on DOF k gives
    qd = h (M + diag(armature))^-1 e_k, so M_ab qd / h must be the identity
    (two independent algorithms; rtol 1e-3 in float32)."""
    sp = gymapi.SimParams()
    sp.dt = 1.0 / 600.0
    sp.substeps = 1
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0, 0, 0)
    sp.use_gpu_pipeline = True
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    opts.armature = 0.002
    asset = gym.load_asset(sim, scenes.ASSET_ROOT, "servo/gimbal.urdf", opts)
    n = 3
    rng = np.random.RandomState(1)
    q0 = rng.uniform(-1.2, 1.2, (n, 3)).astype(np.float32)
    for e in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 2)
        h = gym.create_actor(env, asset, gymapi.Transform(gymapi.Vec3(0, 0, 1)), "gimbal", e, 1)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_EFFORT
        props["stiffness"][:] = 0
        props["damping"][:] = 0
        props["effort"][:] = 0          # no clamp
        props["velocity"][:] = 0
        gym.set_actor_dof_properties(env, h, props)
        ds = np.zeros(3, gymapi.DofState.dtype)
        ds["pos"] = q0[e]
        gym.set_actor_dof_states(env, h, ds, gymapi.STATE_ALL)
    gym.prepare_sim(sim)
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    mm = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, "gimbal"))
    gym.refresh_mass_matrix_tensors(sim)
    M = mm.cpu().numpy().astype(np.float64)
    assert np.allclose(M, np.transpose(M, (0, 2, 1)))
    Minv = np.zeros((n, 3, 3))
    init = torch.zeros((3 * n, 2), dtype=torch.float32, device=DEV)
    init[:, 0] = torch.from_numpy(q0.reshape(-1)).to(DEV)
    for k in range(3):
        gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(init))
        tau = torch.zeros(3 * n, dtype=torch.float32, device=DEV)
        tau[k::3] = 1.0
        gym.set_dof_actuation_force_tensor(sim, gymtorch.unwrap_tensor(tau))
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        Minv[:, :, k] = dof.cpu().numpy()[:, 1].reshape(n, 3) / sp.dt
    for e in range(n):
        eye = (M[e] + 0.002 * np.eye(3)) @ Minv[e]
        np.testing.assert_allclose(eye, np.eye(3), atol=2e-3)


def test_hipgraph_replay_matches_eager(gym):
    """The tensor-API step captured into a hipGraph (torch.cuda.graph; the library
    records its kernels into the capture and leaves out its timing events) and
    replayed 50 times gives the same states, bit for bit, as 50 eager steps; so
    does a graph of 5 consecutive steps replayed 10 times (bench.py's chunks)."""
    from test_isaacgym_amd import _native as N
    n, steps = 256, 50
    outs = []
    for mode in ("eager", "graph", "graph5", "graph5_fused"):
        sim, _ = scenes.servo_scene(gym, n)
        gym.prepare_sim(sim)
        if mode == "graph5_fused":   # MG_FUSE_IN_CAPTURE: the fused set / refresh inside the graph
            gym.set_step_fusion(sim, gymapi.STEP_FUSION_ALL)
        root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
        rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
        acts = scenes.servo_actions(n, 8, DEV, seed=5)
        kdev = torch.zeros(1, dtype=torch.long, device=DEV)

        def step():
            root[:, 3:10] = acts.index_select(0, kdev).squeeze(0)
            kdev.add_(1)
            kdev.remainder_(acts.shape[0])
            gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
            gym.simulate(sim)
            gym.fetch_results(sim, True)
            gym.refresh_actor_root_state_tensor(sim)
            gym.refresh_rigid_body_state_tensor(sim)

        gym.refresh_actor_root_state_tensor(sim)
        if mode == "eager":
            for _ in range(steps):
                step()
        else:
            per = 5 if mode.startswith("graph5") else 1
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(per):
                    step()
            # capture records without executing: replay all the steps
            for _ in range(steps // per):
                g.replay()
        torch.cuda.synchronize()
        outs.append(rb.cpu().numpy().copy())
        gym.destroy_sim(sim)
    assert np.all(np.isfinite(outs[0]))
    assert np.array_equal(outs[0], outs[1]), "max |diff| %g" % np.abs(outs[0] - outs[1]).max()
    assert np.array_equal(outs[0], outs[2]), "max |diff| %g" % np.abs(outs[0] - outs[2]).max()
    assert np.array_equal(outs[0], outs[3]), "max |diff| %g" % np.abs(outs[0] - outs[3]).max()


def test_gimbal_shared_and_mixed_props_parity(gym):
    """k_artic_chain reads a template's DOF properties, link mass constants and
    gravity flag as wave-uniform scalars while every instance agrees
    (migym_capi.cpp chain_uni_*), per lane otherwise: 20 steps shared, 20 with
    one gimbal's stiffness and effort changed through set_actor_dof_properties
    (the per-lane path), 20 with it restored (shared again) — bit for bit the
    oracle throughout."""
    n, steps = 192, 60
    sim, envs = scenes.gimbal_scene(gym, n)
    gym.prepare_sim(sim)
    _, rb, dof, _ = _tensors(gym, sim)
    tg = scenes.gimbal_targets(n, steps, DEV, seed=9)
    tg_h = tg.cpu().numpy()
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    st = A["body_state0"].copy()
    ds = A["dof_state0"].copy()
    props = A["dof_props"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    env, h = envs[5], 0
    base = gym.get_actor_dof_properties(env, h)
    for k in range(steps):
        if k in (20, 40):
            pr = base.copy()
            if k == 20:
                pr["stiffness"][:] = 80.0
                pr["effort"][:] = 4.0
            assert gym.set_actor_dof_properties(env, h, pr)
            d0 = 5 * 3
            props[d0:d0 + 3, 1] = pr["stiffness"]
            props[d0:d0 + 3, 3] = pr["effort"]
        assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k].contiguous()))
        gym.simulate(sim)
        tgt[:, 0] = tg_h[k]
        oracle.step(p, m, st, ds, tgt=tgt, props=props)
        if k in (19, 39, 59):
            gym.refresh_dof_state_tensor(sim)
            gym.refresh_rigid_body_state_tensor(sim)
            got_d, got = dof.cpu().numpy(), rb.cpu().numpy()
            assert np.array_equal(got_d, ds), "step %d: max |diff| %g" % (k, np.abs(got_d - ds).max())
            assert np.array_equal(got, st), "step %d: max |diff| %g" % (k, np.abs(got - st).max())
