"""S3 on the GPU: the Franka cube-pick scene of examples/franka_cube_ik_osc.py
through the coupled per-env step (mg_env.hip), driven by the script's own OSC
controller (test_isaacgym_amd.franka_control, restating :348-410) on the
device Jacobian / mass-matrix tensors.

Parity: every frame's GPU state must equal the C restatement
(oracle/migym_oracle_env.c) fed the same actions, bit for bit (the same fp32
expressions in the same order, no FMA contraction on either side).
Physics: the pick loop lifts cubes (the script's whole point), and the
Jacobian / mass matrix match float64 textbook kinematics (tests/kinematics64.py).
"""
import os

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import franka_control, scenes
import kinematics64 as K
import oracle
import franka_geom as FG

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


# MIGYM_FRANKA_ASSET (measurements only): another proxy,
# e.g. franka_hand64/franka_proxy.urdf with MIGYM_HULL_CAPS and a library built
# with larger MG_HULL_MAX_*; unset, the in-tree asset
FRANKA_ASSET = os.environ.get("MIGYM_FRANKA_ASSET", "franka/franka_proxy.urdf")


def _setup(gym, n, seed=42):
    sim, info = scenes.franka_scene(gym, n, use_gpu_pipeline=True, seed=seed, asset_file=FRANKA_ASSET)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    jac = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, "franka"))
    mm = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, "franka"))
    ctl = franka_control.CubePick(n, info["init_pos"], info["init_rot"], info["default_dof_pos"], DEV)
    return sim, info, rb, dof, jac, mm, ctl


def _control(gym, sim, info, rb, dof, jac, mm, ctl, n):
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_dof_state_tensor(sim)
    gym.refresh_jacobian_tensors(sim)
    gym.refresh_mass_matrix_tensors(sim)
    h = info["hand_index"]
    bi = torch.tensor(info["box_idxs"], device=DEV)
    hi = torch.tensor(info["hand_idxs"], device=DEV)
    dp = dof[:, 0].view(n, 9, 1)
    dv = dof[:, 1].view(n, 9, 1)
    pa, ea = ctl.step(rb, dp, dv, jac[:, h - 1, :, :7], mm[:, :7, :7], bi, hi)
    gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(pa.contiguous()))
    gym.set_dof_actuation_force_tensor(sim, gymtorch.unwrap_tensor(ea.contiguous()))
    return pa, ea


def test_franka_env_classification(gym):
    """Every env is one coupled-step lane (cube + table in group i, filter 0;
    Franka filter 2): no body goes through the uncoupled kernels."""
    from test_isaacgym_amd import _native as N
    sim, info, *_ = _setup(gym, 8)
    assert N.lib.mg_num_coupled_envs(sim.native) == 8


def test_franka_pick_parity_bitexact(gym):
    """64 envs, 240 frames of the OSC pick loop (approach, grasp contacts,
    lift): GPU state == oracle state after every frame."""
    # MIGYM_PARITY_ENVS / _FRAMES: a longer run for measurements
    n = int(os.environ.get("MIGYM_PARITY_ENVS", "64"))
    frames = int(os.environ.get("MIGYM_PARITY_FRAMES", "240"))
    sim, info, rb, dof, jac, mm, ctl = _setup(gym, n)
    p, m = sim.mg_params(), sim.mg_model()
    A = sim.model_arrays
    st = A["body_state0"].copy()
    ds = A["dof_state0"].copy()
    tgt = np.zeros((ds.shape[0], 3), np.float32)
    tgt[:, 0] = ds[:, 0]
    gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(torch.from_numpy(tgt[:, 0].copy()).to(DEV)))
    lifted = np.zeros(n, bool)
    for f in range(frames):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        oracle.step(p, m, st, ds, tgt=tgt, props=A["dof_props"])
        pa, ea = _control(gym, sim, info, rb, dof, jac, mm, ctl, n)
        got, got_d = rb.cpu().numpy(), dof.cpu().numpy()
        assert np.all(np.isfinite(got))
        if not (np.array_equal(got, st) and np.array_equal(got_d, ds)):
            bad = np.argwhere(got != st)
            pytest.fail("frame %d: first differing body/field %s, max |diff| %g (dof %g)"
                        % (f, bad[:3].tolist(), np.abs(got - st).max(), np.abs(got_d - ds).max()))
        tgt[:, 0] = pa.reshape(-1).cpu().numpy()
        tgt[:, 2] = ea.reshape(-1).cpu().numpy()
        lifted |= st[info["box_idxs"], 2] > 0.45
    assert lifted.sum() >= 1      # the window reaches grasp-and-lift contacts


@pytest.mark.parametrize("n", [256, 4096])
def test_franka_pick_lifts_cubes(gym, n):
    """Config 3 (examples/franka_cube_ik_osc.py --num_envs 4096) at 256 and at
    the full 4096 envs, 600 frames (10 s) of the script's loop: at least 88 % of
    the cubes are grasped and lifted above 0.55 m (the script drops them at
    0.6 m, :405; measured round 6: 93.8 % at 256 envs, 91.6 % at 4096,
    profiles/r06_franka_stats.log), state stays finite, no cube sinks into the
    table or the ground, and hand / finger hulls do not stay inside the table.
    Parity unpinned: no reference output shows a grasp or a hull's depth in the
    table; these bounds pin this build's behaviour."""
    frames = 600
    sim, info, rb, dof, jac, mm, ctl = _setup(gym, n)
    maxz = torch.zeros(n, device=DEV)
    bi = torch.tensor(info["box_idxs"], device=DEV)
    hi = torch.tensor(info["hand_idxs"], device=DEV)
    hulls = torch.stack([hi, hi + 1, hi + 2], 1)
    A = sim.model_arrays
    off = float(sim.params.physx.contact_offset)
    # hand / finger hulls inside the table box (tests/franka_geom.py), every frame
    deep_run = torch.zeros((2, n), dtype=torch.int64, device=DEV)   # consecutive frames deeper than 1 / 5 mm
    worst_run = torch.zeros_like(deep_run)
    worst = torch.zeros(n, dtype=torch.float64, device=DEV)
    lim = torch.tensor([off, 0.005], dtype=torch.float64, device=DEV)[:, None]
    for f in range(frames):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        _control(gym, sim, info, rb, dof, jac, mm, ctl, n)
        maxz = torch.maximum(maxz, rb[bi, 2])
        d = FG.penetration_depth(A, rb, hulls, bi - 1)
        worst = torch.maximum(worst, d)
        deep_run = torch.where(d[None, :] > lim, deep_run + 1, torch.zeros_like(deep_run))
        worst_run = torch.maximum(worst_run, deep_run)
    assert torch.isfinite(rb).all()
    # No hand or finger stays inside the table. With Isaac Gym's 1 mm contact
    # offset (franka_cube_ik_osc.py:123) a hull moving at up to ~2 m/s enters
    # the table by up to a substep's travel before its first contact exists (no
    # speculative contacts; tools/diag_franka_env.py: 160 of 4096 envs pass 1 mm
    # in some frame, the deepest 17.6 mm, a hand driven down at a cube on the
    # floor; 31 pass 5 mm, each for at most 2 frames). With the torch controller's
    # trajectories one arm in 4096 (env 2581, profiles/r06_diag_franka.jsonl;
    # the one-kernel controller's, the default since round 6, differ in float32
    # rounding and have no such arm: longest run 18 frames) wedged below the
    # table top at a corner —
    # the hand against the -y face, finger A the -x face, finger B pressed down
    # on the top at ~480 N by the OSC torques — and that finger rests 1.32 mm in
    # for the remaining 390 frames. Measured cause (round 6 A/B, DESIGN.md
    # §3.6.1): the sweep order, normal rows then the anchors' rows, with only the
    # last position sweep closing on the normal rows: the velocity integrated in
    # the earlier sweeps is the one the friction rows left, under a steady load
    # a fixed overlap. Closing every sweep on the normal rows ends every run past
    # 1 mm within 2 frames, but the fingers' normal rows then undo the grip's
    # friction (15 % of the cubes lifted), so the order stays and the bound is
    # on how many envs hold such an overlap.
    stats = {"n": n, "worst_mm": round(1e3 * float(worst.max()), 2), "worst_env": int(worst.argmax()),
             "envs_past_1mm": int((worst > off).sum()), "envs_past_5mm": int((worst > 0.005).sum()),
             "longest_run_past_1mm": int(worst_run[0].max()), "longest_run_past_5mm": int(worst_run[1].max()),
             "last_frame_worst_mm": round(1e3 * float(d.max()), 2),
             "lifted_frac": round(float((maxz > 0.55).float().mean()), 4)}
    print("hull-in-table:", stats)
    stats["envs_run_past_1mm_over_40"] = int((worst_run[0] > 40).sum())
    assert stats["worst_mm"] < 20.0, stats                          # measured 17.63 (4096), 6.97 (256)
    assert stats["longest_run_past_5mm"] <= 3, stats                # measured 2 / 1
    assert stats["last_frame_worst_mm"] <= 5.0, stats               # measured 3.56 / 0.69
    assert stats["envs_run_past_1mm_over_40"] <= max(n // 1000, 1), stats   # the wedged arm above
    frac = float((maxz > 0.55).float().mean())
    assert frac >= 0.88, "only %.4f of the cubes were lifted" % frac
    # nothing sinks through the table or the ground. A cube whose footprint
    # overlaps the table's (top at 0.4 m, half extents 0.3 / 0.5 m, cube half
    # size 0.0225 m) must not rest below the top. A cube at rest below the top
    # beside the table must be carried by the robot: the contacts the narrow
    # phase handed to the step (mg_debug_copy_env_ctab) include one between the
    # cube and a link of the arm. The one such cube at 4096 envs (env 3043,
    # tools/diag_franka_env.py, profiles/r05_diag_franka.jsonl) was knocked off
    # the table's edge and rests on the forearm (links 4 and 5), pressed
    # against the table's -x face; the arm reached around the table's corner
    # after it and is wedged between joint 2's upper limit (a constraint row)
    # and the table — finger A closed and pressing the corner (~980 N: the
    # OSC torques of up to 87 N m at short levers against the limit row's
    # reaction), finger B open — with no hull inside the table. Carried by the
    # arm, not by the fingers, so the fingers are not required.
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    gym.refresh_net_contact_force_tensor(sim)
    z = rb[bi, 2]
    assert float(z.min()) > 0.0
    still = rb[bi, 7:10].norm(dim=1) < 0.05
    rel = rb[bi, 0:2] - rb[bi - 1, 0:2]            # from the table centre (the body before the cube)
    overlap = (rel[:, 0].abs() < 0.3 + 0.0225) & (rel[:, 1].abs() < 0.5 + 0.0225)
    below = (z > 0.3) & (z < 0.4225 - 0.005) & still
    sunk = below & overlap
    assert int(sunk.sum()) == 0, "cubes at rest inside the table: %s" % z[sunk][:8].tolist()
    beside = (below & ~overlap).nonzero().flatten().tolist()
    for e in beside:
        rows = _env_contacts(sim, e)
        on_arm = [(a, b) for a, b, _ in rows if (a == 64 and 0 <= b < 16) or (b == 64 and 0 <= a < 16)]
        assert on_arm, "env %d: cube at rest below the table top beside it with no contact on the arm: %s" % (
            e, rows)
    assert len(beside) <= max(n // 1000, 1)    # a rare case, not a pattern


def _env_contacts(sim, e):
    """Env e's contacts of the last substep as k_env_np handed them to the step
    (participants a, b: link l, free body 64 + k, static 80 + s, ground -1;
    separation): mg_debug_copy_env_ctab (every env of the scene is coupled, so
    env e is coupled env e; the library sizes the record)."""
    import ctypes
    from test_isaacgym_amd import _native as N
    cap = N.lib.mg_env_ctab_floats()
    buf = (ctypes.c_float * cap)()
    n = N.lib.mg_debug_copy_env_ctab(sim.native, e, buf, cap)
    N.check(n if n < 0 else 0, "mg_debug_copy_env_ctab")
    maxct = (n - 8) // 24
    a = np.frombuffer(buf, np.float32)[:n]
    ib = a.view(np.int32)
    return [(int(ib[8 + 10 * c]), int(ib[9 + 10 * c]), float(a[16 + 10 * c])) for c in range(min(int(ib[0]), maxct))]


def test_franka_jacobian_mass_matrix_float64(gym):
    """Device Jacobian (link origins) and CRBA mass matrix of the Franka at
    random joint configurations vs float64 kinematics64 (rtol 1e-4)."""
    n = 16
    sim, info, rb, dof, jac, mm, ctl = _setup(gym, n)
    A = sim.model_arrays
    rng = np.random.RandomState(5)
    props = A["dof_props"][:9]
    lo, hi = props[:, 5], props[:, 6]
    q = (lo + (hi - lo) * rng.uniform(0.1, 0.9, (n, 9))).astype(np.float32)
    init = torch.zeros((9 * n, 2), dtype=torch.float32, device=DEV)
    init[:, 0] = torch.from_numpy(q.reshape(-1)).to(DEV)
    gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(init))
    gym.refresh_jacobian_tensors(sim)
    gym.refresh_mass_matrix_tensors(sim)
    art = K.Articulation(A, 0)
    J = jac.cpu().numpy()
    M = mm.cpu().numpy()
    for e in range(n):
        fb = int(A["artic_i"][e, 0])
        base = A["body_state0"][fb]
        Jr = art.jacobian(base, q[e].astype(np.float64))
        Mr = art.mass_matrix(base, q[e].astype(np.float64), fb)
        assert np.allclose(J[e], Jr, rtol=1e-4, atol=1e-5), np.abs(J[e] - Jr).max()
        assert np.allclose(M[e], Mr, rtol=1e-4, atol=1e-5), np.abs(M[e] - Mr).max()


def test_box_stacks_parity_bitexact(gym):
    """Coupled envs without an articulation (the no-articulation launch group):
    per env a fixed table, a cube on it and a second cube dropped onto the
    first with a random spin (free-static and free-free rows, ground rows);
    150 frames, GPU == oracle bit for bit after every frame."""
    n, frames = 96, 150
    sp = scenes.franka_sim_params(True)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    table = gym.create_box(sim, 0.6, 1.0, 0.4, opts)
    cube = gym.create_box(sim, 0.06, 0.06, 0.06, gymapi.AssetOptions())
    rng = np.random.RandomState(11)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 10)
        gym.create_actor(env, table, gymapi.Transform(gymapi.Vec3(0.5, 0, 0.2)), "table", i, 0)
        p1 = gymapi.Transform(gymapi.Vec3(0.5 + rng.uniform(-0.1, 0.1), rng.uniform(-0.2, 0.2), 0.43))
        p1.r = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 0, 1), rng.uniform(-3, 3))
        gym.create_actor(env, cube, p1, "c1", i, 0)
        p2 = gymapi.Transform(gymapi.Vec3(p1.p.x + rng.uniform(-0.02, 0.02), p1.p.y, 0.6))
        p2.r = gymapi.Quat.from_axis_angle(gymapi.Vec3(rng.normal(), rng.normal(), 1.0), rng.uniform(-1, 1))
        gym.create_actor(env, cube, p2, "c2", i, 0)
    gym.prepare_sim(sim)
    from test_isaacgym_amd import _native as N
    assert N.lib.mg_num_coupled_envs(sim.native) == n
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    ds = sim.model_arrays["dof_state0"].copy()
    for f in range(frames):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_rigid_body_state_tensor(sim)
        oracle.step(p, m, st, ds)
        got = rb.cpu().numpy()
        if not np.array_equal(got, st):
            bad = np.argwhere(got != st)
            pytest.fail("frame %d: first differing body/field %s, max |diff| %g" % (f, bad[:3].tolist(),
                                                                                 np.abs(got - st).max()))
    # the dropped cubes end on the first ones or on the table, none below the table top
    assert np.all(st[2::3, 2] > 0.39)


def test_franka_loop_hipgraph_matches_eager(gym):
    """The whole S3 frame (simulate, refreshes incl. Jacobian / mass matrix, the
    torch OSC controller, DOF target / effort setters) captured into a hipGraph
    and replayed gives the same states as the eager loop, bit for bit."""
    n, steps = 64, 40
    outs = []
    for mode in ("eager", "graph"):
        sim, info, rb, dof, jac, mm, ctl = _setup(gym, n)
        h = info["hand_index"]
        bi = torch.tensor(info["box_idxs"], device=DEV)
        hi = torch.tensor(info["hand_idxs"], device=DEV)
        j_eef, mm7 = jac[:, h - 1, :, :7], mm[:, :7, :7]
        dp, dv = dof[:, 0].view(n, 9, 1), dof[:, 1].view(n, 9, 1)

        def frame():
            gym.simulate(sim)
            gym.fetch_results(sim, True)
            gym.refresh_rigid_body_state_tensor(sim)
            gym.refresh_dof_state_tensor(sim)
            gym.refresh_jacobian_tensors(sim)
            gym.refresh_mass_matrix_tensors(sim)
            pa, ea = ctl.step(rb, dp, dv, j_eef, mm7, bi, hi)
            gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(pa))
            gym.set_dof_actuation_force_tensor(sim, gymtorch.unwrap_tensor(ea))

        if mode == "eager":
            for _ in range(steps):
                frame()
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                frame()
            for _ in range(steps):
                g.replay()
        torch.cuda.synchronize()
        outs.append((rb.cpu().numpy().copy(), dof.cpu().numpy().copy()))
        gym.destroy_sim(sim)
    assert np.array_equal(outs[0][0], outs[1][0]), np.abs(outs[0][0] - outs[1][0]).max()
    assert np.array_equal(outs[0][1], outs[1][1])
