"""GPU: the refresh fused into the articulation step (STEP_FUSION_STEP_OUT on
serial chains, mg_chain.hip k_artic_chain) and the copy-at-set guard of step
fusion (gymapi._check_held).

S2's loop is set_dof_position_target_tensor -> simulate -> refresh_dof_state_tensor
-> refresh_rigid_body_state_tensor (test12_add_joint.py.py:129,155;
test13_camera_spherical_joint.py:266-269). With STEP_OUT the chain kernel writes
the bound DOF-state, rigid-body and actor-root rows itself and the refreshes
launch nothing. Every check is bit for bit against the unfused sequence (the
gathers of the SoA state) and the oracle's chain step.
"""
import math

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import _native as N, scenes
import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _tensors(gym, sim):
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    return root, rb, dof


def test_gimbal_step_out_fusion(gym):
    """Eager, captured and write-after-simulate: a fused gimbal sim's DOF,
    rigid-body and root tensors equal the unfused sim's bit for bit, and both
    equal the oracle. 1000 gimbals: the last 64-lane block is partly empty."""
    n, chunk = 1000, 4
    tg = scenes.gimbal_targets(n, 3 * chunk + 1, DEV, seed=21)
    sims = []
    for fusion in (gymapi.STEP_FUSION_ALL, 0):
        sim, _ = scenes.gimbal_scene(gym, n)
        gym.prepare_sim(sim)
        gym.set_step_fusion(sim, fusion)
        sims.append((sim, _tensors(gym, sim)))
    assert N.lib.mg_step_out_supported(sims[0][0].native) == 1

    def step(sim, k, root_too=True):
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k]))
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        if root_too:
            gym.refresh_actor_root_state_tensor(sim)

    (sa, (ra, rba, da)), (sb, (rb_, rbb, db)) = sims
    p, m = sa.mg_params(), sa.mg_model()
    st = sa.model_arrays["body_state0"].copy()
    ds = sa.model_arrays["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    tg_h = tg.cpu().numpy()

    def same(what):
        torch.cuda.synchronize()
        assert torch.equal(da, db), "%s: DOF state differs" % what
        assert torch.equal(rba, rbb), "%s: rigid-body state differs" % what
        assert torch.equal(ra, rb_), "%s: root state differs" % what

    for k in range(chunk):                      # eager
        step(sa, k)
        step(sb, k)
        tgt[:, 0] = tg_h[k]
        oracle.step(p, m, st, ds, tgt=tgt)
        same("eager step %d" % k)
    assert np.array_equal(da.cpu().numpy(), ds), "fused DOF state vs oracle"
    assert np.array_equal(rba.cpu().numpy(), st), "fused rigid-body state vs oracle"
    # captured: `chunk` fused steps per graph; the unfused sim steps eagerly
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for j in range(chunk):
                step(sa, chunk + j)
    torch.cuda.current_stream().wait_stream(side)
    g.replay()
    for j in range(chunk):
        step(sb, chunk + j)
    same("captured steps")
    # a write between simulate and refresh: the refresh restores the state
    for sim, (root, rb, dof) in sims:
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[2 * chunk]))
        gym.simulate(sim)
        dof.fill_(-3.0)
        rb[:, 5] = 9.0
        root.fill_(-4.0)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_actor_root_state_tensor(sim)
    same("refresh after a user write")
    assert not torch.any(da == -3.0) and not torch.any(ra == -4.0)
    # write -> refresh -> write -> refresh with no simulate between:
    # the second refresh overwrites the user's values again, as Isaac Gym's does
    for sim, (root, rb, dof) in sims:
        dof.fill_(-5.0)
        rb[:, 5] = 7.0
        root.fill_(-6.0)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_actor_root_state_tensor(sim)
    same("second refresh after a user write")
    assert not torch.any(da == -5.0) and not torch.any(ra == -6.0) and not torch.any(rba[:, 5] == 7.0)
    # a DOF-state set after the step: the next refresh shows the set, not the step's rows
    for sim, (root, rb, dof) in sims:
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[2 * chunk + 1]))
        gym.simulate(sim)
        new = torch.zeros_like(dof)
        new[:, 0] = 0.25
        assert gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(new))
        gym.refresh_dof_state_tensor(sim)
        assert torch.equal(dof, new)
    # roots are the fixed bases: the root rows are the bases' rigid-body rows
    roots = torch.as_tensor(sa.model_arrays["actor_root_body"], device=DEV, dtype=torch.long)
    assert torch.equal(rba[roots], ra)
    for sim, _ in sims:
        gym.destroy_sim(sim)


def _mixed_scene(gym, n):
    """Per env the servo scene's two free bodies and one gimbal (filter 1 against
    the free bodies' -1: no contacts, so every body is stepped by a STEP_OUT
    kernel: k_rigid_step1 and k_artic_chain in one simulate)."""
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, scenes.servo_sim_params(True))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    assets = []
    for f in ("servo/uav.urdf", "servo/ground_vehicle.urdf"):
        opts = gymapi.AssetOptions()
        opts.armature = 0.01
        assets.append(gym.load_asset(sim, scenes.ASSET_ROOT, f, opts))
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    opts.default_dof_drive_mode = gymapi.DOF_MODE_POS
    gimbal = gym.load_asset(sim, scenes.ASSET_ROOT, "servo/gimbal.urdf", opts)
    per_row = int(math.sqrt(n))
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-20, -20, -20), gymapi.Vec3(20, 20, 20), per_row)
        gym.create_actor(env, assets[0], gymapi.Transform(gymapi.Vec3(-10.0, 0.0, 102.0)), "uav", i, -1)
        h = gym.create_actor(env, gimbal, gymapi.Transform(gymapi.Vec3(0.0, 2.0, 3.0)), "gimbal", i, 1)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_POS
        props["stiffness"][:] = 50.0
        props["damping"][:] = 5.0
        gym.set_actor_dof_properties(env, h, props)
        gym.create_actor(env, assets[1], gymapi.Transform(gymapi.Vec3(0.0, 0.0, 2.0)), "car", i, -1)
    return sim


def test_mixed_free_bodies_and_chains_step_out(gym):
    """Free bodies and gimbals in one sim: with STEP_OUT both kernels write
    their rows (the actor rows interleave UAV, gimbal base, vehicle), equal to
    the unfused sim's tensors and to the oracle, bit for bit."""
    n, steps = 200, 6
    sims = []
    for fusion in (gymapi.STEP_FUSION_STEP_OUT, 0):
        sim = _mixed_scene(gym, n)
        gym.prepare_sim(sim)
        gym.set_step_fusion(sim, fusion)
        sims.append((sim, _tensors(gym, sim)))
    assert N.lib.mg_step_out_supported(sims[0][0].native) == 1
    (sa, (ra, rba, da)), (sb, (rb_, rbb, db)) = sims
    p, m = sa.mg_params(), sa.mg_model()
    st = sa.model_arrays["body_state0"].copy()
    ds = sa.model_arrays["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    rng = np.random.RandomState(5)
    for k in range(steps):
        tgt[:, 0] = rng.uniform(-1.5, 1.5, ds.shape[0]).astype(np.float32)
        t = torch.from_numpy(tgt[:, 0].copy()).to(DEV)
        for sim, (root, rb, dof) in sims:
            gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(t))
            gym.simulate(sim)
            gym.refresh_actor_root_state_tensor(sim)
            gym.refresh_rigid_body_state_tensor(sim)
            gym.refresh_dof_state_tensor(sim)
        oracle.step(p, m, st, ds, tgt=tgt)
        torch.cuda.synchronize()
        assert torch.equal(ra, rb_) and torch.equal(rba, rbb) and torch.equal(da, db), "step %d" % k
    assert np.array_equal(rba.cpu().numpy(), st)
    assert np.array_equal(da.cpu().numpy(), ds)
    for sim, _ in sims:
        gym.destroy_sim(sim)


def test_step_out_only_keeps_copy_at_set(gym):
    """STEP_FUSION_STEP_OUT alone defers no set, so a source written
    after its set (host or device, root state or DOF targets) is Isaac Gym's
    copy-at-set case: no error, and the step sees the value at the set call."""
    n = 32
    acts = scenes.servo_actions(n, 2, DEV, seed=2)
    outs = []
    for fusion in (0, gymapi.STEP_FUSION_STEP_OUT):
        for host in (False, True):
            sim, _ = scenes.servo_scene(gym, n)
            gym.prepare_sim(sim)
            gym.set_step_fusion(sim, fusion)
            root, rb, _ = _tensors(gym, sim)
            gym.refresh_actor_root_state_tensor(sim)
            src = root.clone()
            src[:, 3:10] = acts[0]
            if host:
                src = src.cpu()
            assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(src))
            src[:, 3:10] = acts[1].to(src.device)
            gym.simulate(sim)                           # must not raise
            gym.refresh_rigid_body_state_tensor(sim)
            outs.append(rb.clone())
            gym.destroy_sim(sim)
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    tg = scenes.gimbal_targets(16, 2, DEV, seed=4)
    douts = []
    for fusion in (0, gymapi.STEP_FUSION_STEP_OUT):
        sim, _ = scenes.gimbal_scene(gym, 16)
        gym.prepare_sim(sim)
        gym.set_step_fusion(sim, fusion)
        dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
        t = tg[0].clone()
        assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(t))
        t.copy_(tg[1])
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        douts.append(dof.clone())
        gym.destroy_sim(sim)
    assert torch.equal(douts[0], douts[1])


def test_raised_fused_set_is_discarded(gym):
    """when simulate raises because a deferred set's source was
    written after the set, the pending set is dropped on the C side too: a
    retried simulate does not read the modified source, it steps as if the
    set had not been made."""
    n = 16
    tg = scenes.gimbal_targets(n, 2, DEV, seed=8)
    outs = []
    for mode in ("raised", "never_set"):
        sim, _ = scenes.gimbal_scene(gym, n)
        gym.prepare_sim(sim)
        gym.set_step_fusion(sim, gymapi.STEP_FUSION_ALL)
        dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
        if mode == "raised":
            t = tg[0].clone()
            assert gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(t))
            t.copy_(tg[1])
            with pytest.raises(N.MigymError):
                gym.simulate(sim)
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        outs.append(dof.clone())
        gym.destroy_sim(sim)
    assert torch.equal(outs[0], outs[1])


def test_gimbal_uniform_props_graph_replay(gym):
    """a hipGraph captured while every gimbal shared its DOF
    properties (k_artic_chain's wave-uniform constants) keeps stepping with the
    right properties after set_actor_dof_properties makes one env differ, and
    again after it is restored: the kernel reads the uniformity flag at run
    time. Replays are bit for bit the oracle stepped with the same props."""
    n, chunk = 128, 3
    sim, envs = scenes.gimbal_scene(gym, n)
    gym.prepare_sim(sim)
    gym.set_step_fusion(sim, gymapi.STEP_FUSION_ALL)
    _, rb, dof = _tensors(gym, sim)
    tg = scenes.gimbal_targets(n, chunk, DEV, seed=13)
    tg_h = tg.cpu().numpy()
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    st = A["body_state0"].copy()
    ds = A["dof_state0"].copy()
    props = A["dof_props"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)

    def step(k):
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k]))
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for k in range(chunk):
                step(k)
    torch.cuda.current_stream().wait_stream(side)
    env, h = envs[7], 0
    base = gym.get_actor_dof_properties(env, h)
    for phase in ("captured uniform", "one env differs", "restored"):
        if phase != "captured uniform":
            pr = base.copy()
            if phase == "one env differs":
                pr["stiffness"][:] = 400.0
                pr["damping"][:] = 1.0
                pr["effort"][:] = 3.0
            assert gym.set_actor_dof_properties(env, h, pr)
            props[7 * 3:7 * 3 + 3, 1] = pr["stiffness"]
            props[7 * 3:7 * 3 + 3, 2] = pr["damping"]
            props[7 * 3:7 * 3 + 3, 3] = pr["effort"]
        g.replay()
        for k in range(chunk):
            tgt[:, 0] = tg_h[k]
            oracle.step(p, m, st, ds, tgt=tgt, props=props)
        torch.cuda.synchronize()
        assert np.array_equal(dof.cpu().numpy(), ds), "%s: DOF state max |diff| %g" % (
            phase, np.abs(dof.cpu().numpy() - ds).max())
        assert np.array_equal(rb.cpu().numpy(), st), "%s: rigid-body state" % phase
    gym.destroy_sim(sim)


def test_gimbal_wide_launch_rows_through_lds(gym):
    """more than 65,536 gimbals (a launch wider than one resident
    round) takes k_artic_chain's full-wave LDS row path; 65,536 + 64*3 + 17 leaves
    the last wave partly filled. Fused (STEP_FUSION_ALL) and unfused sims give
    the same DOF, rigid-body and root tensors bit for bit, and both equal the
    oracle."""
    n, steps = 65536 + 64 * 3 + 17, 2
    tg = scenes.gimbal_targets(n, steps, DEV, seed=23)
    sims = []
    for fusion in (gymapi.STEP_FUSION_ALL, 0):
        sim, _ = scenes.gimbal_scene(gym, n)
        gym.prepare_sim(sim)
        gym.set_step_fusion(sim, fusion)
        sims.append((sim, _tensors(gym, sim)))
    (sa, (ra, rba, da)), (sb, (rb_, rbb, db)) = sims
    p, m = sa.mg_params(), sa.mg_model()
    st = sa.model_arrays["body_state0"].copy()
    ds = sa.model_arrays["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    tg_h = tg.cpu().numpy()
    for k in range(steps):
        for sim, _ in sims:
            gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k]))
            gym.simulate(sim)
            gym.refresh_dof_state_tensor(sim)
            gym.refresh_rigid_body_state_tensor(sim)
            gym.refresh_actor_root_state_tensor(sim)
        tgt[:, 0] = tg_h[k]
        oracle.step(p, m, st, ds, tgt=tgt)
        torch.cuda.synchronize()
        assert torch.equal(da, db) and torch.equal(rba, rbb) and torch.equal(ra, rb_), "step %d: fused != unfused" % k
    assert np.array_equal(da.cpu().numpy(), ds)
    assert np.array_equal(rba.cpu().numpy(), st)
    roots = torch.as_tensor(sa.model_arrays["actor_root_body"], device=DEV, dtype=torch.long)
    assert torch.equal(rba[roots], ra)
    for sim, _ in sims:
        gym.destroy_sim(sim)


def _gimbal_box_scene(gym, n, box_every, heavy_every=0):
    """gimbal_scene's gimbals (fixed base at (0, 2, 3), POS drives kp 50, kd 5)
    with a free 0.2 m box created after the gimbal in every `box_every`-th env
    (filter 1 against the gimbal's 1: no contacts, so the box steps alone on the
    ground in k_rigid_step1). The boxes' rows interleave the gimbals' rows in
    the rigid-body and root tensors, so the fused refresh's rows are not affine
    in the instance (out_aff 0); every `heavy_every`-th env's gimbal links get
    1.5x their mass (the link mass rows then differ: UNI 0)."""
    sp = gymapi.SimParams()
    sp.substeps = 2
    sp.dt = 1.0 / 60.0
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0.0, 0.0, -9.8)
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 4
    sp.physx.num_velocity_iterations = 1
    sp.use_gpu_pipeline = True
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    opts.default_dof_drive_mode = gymapi.DOF_MODE_POS
    gimbal = gym.load_asset(sim, scenes.ASSET_ROOT, "servo/gimbal.urdf", opts)
    box = gym.create_box(sim, 0.2, 0.2, 0.2, gymapi.AssetOptions())
    per_row = int(math.sqrt(n))
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, -1), gymapi.Vec3(1, 1, 1), per_row)
        h = gym.create_actor(env, gimbal, gymapi.Transform(gymapi.Vec3(0.0, 2.0, 3.0)), "gimbal", i, 1)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_POS
        props["stiffness"][:] = 50.0
        props["damping"][:] = 5.0
        gym.set_actor_dof_properties(env, h, props)
        if heavy_every and i % heavy_every == 0:
            bp = gym.get_actor_rigid_body_properties(env, h)
            for b in bp:
                b.mass = b.mass * 1.5
            gym.set_actor_rigid_body_properties(env, h, bp, True)
        if i % box_every == 0:
            gym.create_actor(env, box, gymapi.Transform(gymapi.Vec3(0.5, 0.0, 0.3)), "box", i, 1)
    return sim


def _artic_groups(sim):
    import ctypes
    buf = (ctypes.c_int32 * (8 * N.MG_DEBUG_GROUP_N))()
    ng = N.lib.mg_debug_artic_groups(sim.native, buf, len(buf))
    assert ng >= 0, N.last_error()
    a = np.frombuffer(buf, np.int32).reshape(-1, N.MG_DEBUG_GROUP_N)[:ng]
    keys = ("nl", "step_count", "chain", "uni_mass", "uni_dof", "aff", "out_aff", "step_out_ok")
    return [dict(zip(keys, map(int, r))) for r in a]


@pytest.mark.parametrize("heavy_every", [0, 7], ids=["uni", "nonuni"])
def test_gimbal_nonaffine_one_lane_forms(gym, heavy_every):
    """the one-lane chain kernel's forms without computed
    rows (k_artic_chain<4, 0, UNI, AFF = 0>) on the GPU. 65,536 + 64 x 5 + 23
    gimbals (a launch wider than one resident round, so full contiguous waves
    take the LDS row path; the last wave partly filled) interleaved with free
    boxes in every 997th env (waves that straddle a box store their rows lane
    by lane). `uni`: fused (STEP_FUSION_ALL) -> <4,0,1,0> (out_aff 0), unfused
    -> <4,0,1,1>; `nonuni` (every 7th gimbal 1.5x heavier): <4,0,0,0> both
    ways. Fused and unfused DOF, rigid-body and root tensors agree bit for bit,
    and both equal oracle.step (gimbals and boxes)."""
    n, steps = 65536 + 64 * 5 + 23, 2
    tg = scenes.gimbal_targets(n, steps, DEV, seed=29)
    sims = []
    for fusion in (gymapi.STEP_FUSION_ALL, 0):
        sim = _gimbal_box_scene(gym, n, 997, heavy_every)
        gym.prepare_sim(sim)
        gym.set_step_fusion(sim, fusion)
        sims.append((sim, _tensors(gym, sim)))
    (sa, (ra, rba, da)), (sb, (rb_, rbb, db)) = sims
    grp = [g for g in _artic_groups(sa) if g["step_count"] > 0]
    assert len(grp) == 1, grp
    g = grp[0]
    assert (g["nl"], g["step_count"], g["chain"]) == (4, n, 1), g
    assert g["uni_mass"] == (0 if heavy_every else 1), g
    assert g["aff"] == 1 and g["out_aff"] == 0 and g["step_out_ok"] == 1, g
    assert N.lib.mg_step_out_supported(sa.native) == 1
    p, m = sa.mg_params(), sa.mg_model()
    st = sa.model_arrays["body_state0"].copy()
    ds = sa.model_arrays["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    tg_h = tg.cpu().numpy()
    for k in range(steps):
        for sim, _ in sims:
            gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k]))
            gym.simulate(sim)
            gym.refresh_dof_state_tensor(sim)
            gym.refresh_rigid_body_state_tensor(sim)
            gym.refresh_actor_root_state_tensor(sim)
        tgt[:, 0] = tg_h[k]
        oracle.step(p, m, st, ds, tgt=tgt)
        torch.cuda.synchronize()
        assert torch.equal(da, db) and torch.equal(rba, rbb) and torch.equal(ra, rb_), "step %d: fused != unfused" % k
    assert np.abs(ds[:, 1]).max() > 0.05
    assert np.array_equal(da.cpu().numpy(), ds), "max |diff| %g" % np.abs(da.cpu().numpy() - ds).max()
    assert np.array_equal(rba.cpu().numpy(), st), "max |diff| %g" % np.abs(rba.cpu().numpy() - st).max()
    roots = torch.as_tensor(sa.model_arrays["actor_root_body"], device=DEV, dtype=torch.long)
    assert torch.equal(rba[roots], ra)
    for sim, _ in sims:
        gym.destroy_sim(sim)
