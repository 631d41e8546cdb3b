"""Headline benchmark: env-steps/sec of the servo vecenv.

One step = the tensor-API loop of test10_servo_vecenv.py:376-456 with the host
controller replaced by a bank of pre-generated random actions already resident
in HBM:
    root[:, 3:10] = actions[k]                     (quat + linear velocity, all 2N actors)
    gym.set_actor_root_state_tensor(sim, root)      (teleport)
    gym.simulate(sim); gym.fetch_results(sim, False)
    gym.refresh_actor_root_state_tensor(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    gym.refresh_dof_state_tensor(sim)               (0 DOFs in S1)

Multi-GPU (BASELINE config 4): one process and one sim per GPU,
4096 envs per rank (weak scaling). `--gpus N` either runs under
torch.distributed.run (WORLD_SIZE set) or, without it, starts the N rank
processes itself (test_isaacgym_amd/launch.py) before anything touches the GPU.
Envs never interact, so the timed loop has no collective; at N > 1 a second leg
times the optional RCCL all-gather of the root-state observation over xGMI
(`allgather`), and `--allgather` puts it inside the timed loop instead.

Timing: W warm-up steps, a kernel-timing segment (>= 100 eager launches with
dispatch-timestamp events), an eager segment with timing off, then the timed
region — EXACTLY `--steps` steps replayed as hipGraphs, bracketed by barrier +
synchronize, repeated `--repeats` times; `value` uses the median repeat of the
per-repeat maximum over ranks.

Prints ONE JSON line (rank 0). `roofline` prices the dominant kernel
(k_rigid_step1, one launch per simulate) at SURVEY.md §8d's algorithmic bytes:
376 B per env per simulate (2 bodies x (state in 52 + state out 52 + mass
properties 44 + shape 40)), plus 208 B when the refresh is fused into the step
(the rigid-body and root rows it then writes), over its average duration from the kernel's own
dispatch timestamps (hipExtLaunchKernelGGL start / stop events on the simulate
stream, the interval rocprofv3 reports). `large_n` repeats that at 262,144 envs,
where the kernel leaves the latency regime. `cpu_baseline` times the C
restatement (oracle/, "port") on the host cores on a bounded sample of the same
workload.
"""
import argparse
import importlib.util
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node), 4096 servo envs; 1/2/4/8-GPU scaling"
ENVS_PER_GPU = 4096
LARGE_N = 262144
SIM_BYTES_PER_ENV = 376          # simulate share of the 688 B/env-step
# with the refresh fused into the step (STEP_FUSION_STEP_OUT) the kernel also
# writes each body's rigid-body row and its actor's root row: + 2 x (52 + 52) B
SIM_OUT_BYTES_PER_ENV = SIM_BYTES_PER_ENV + 2 * (52 + 52)
STEP_BYTES_PER_ENV = 688         # whole tensor-API step
S2_BYTES_PER_ENV = 532           # SURVEY.md §8d S2 (servo-arm gimbal)
S2_LARGE_N = 262144
S3_BYTES_PER_ENV = 5844          # SURVEY.md §8d S3 (Franka cube pick, the whole tensor-API step)
# S6 ball piles (examples/1080_balls_of_solitude.py): per ball
# and simulate, state in 52 + out 52 + mass properties 44 + net contact force
# 12 (SURVEY §8d's per-body pricing; the shape and the pair list are template
# data shared by every env, read through L2), x 30 balls
S6_BALLS = 30
S6_BYTES_PER_ENV = S6_BALLS * (52 + 52 + 44 + 12)
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
KERNEL_TIMED_LAUNCHES = 128      # eager launches with dispatch timestamps (ring holds 256)
GRAPH_CHUNK_MAX = 64             # tensor-API steps captured per hipGraph at most (amortizes the graph launch)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--repeats", type=int, default=5, help="timed regions of --steps steps; value = median")
    ap.add_argument("--envs", type=int, default=ENVS_PER_GPU, help="envs per GPU")
    ap.add_argument("--allgather", action="store_true",
                    help="RCCL all-gather of the root state inside the timed loop (N > 1)")
    ap.add_argument("--backend", choices=("auto", "nccl", "gloo"), default="auto",
                    help="process-group backend for N > 1 (auto: RCCL when every rank has its own GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: ranks build their shards and check the gathered layout over gloo")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-gimbal", action="store_true", help="skip the secondary S2 servo-arm measurement")
    ap.add_argument("--no-franka", action="store_true", help="skip the secondary S3 Franka cube-pick measurement")
    ap.add_argument("--no-cameras", action="store_true", help="skip the secondary S5 camera-render measurement")
    ap.add_argument("--no-piles", action="store_true", help="skip the secondary S6 ball-pile measurement")
    ap.add_argument("--pile-envs", type=int, default=ENVS_PER_GPU, help="envs of the S6 ball-pile leg")
    ap.add_argument("--no-large-n", action="store_true", help="skip the 262,144-env S1 kernel leg")
    ap.add_argument("--no-default-legs", action="store_true",
                    help="skip the S1 library-default (fusion off) and CPU-pipeline legs")
    ap.add_argument("--pmc-calibrate", action="store_true",
                    help="before the warm-up, 4 indexed root-state sets of every actor (k_scatter_rows: the "
                         "known-volume kernel profiles/collect_pmc.py calibrates FETCH_SIZE on)")
    ap.add_argument("--large-n", type=int, default=LARGE_N)
    ap.add_argument("--camera-envs", type=int, default=1024)
    ap.add_argument("--eager", action="store_true",
                    help="time the Python loop itself instead of a hipGraph replay of the step")
    return ap.parse_args(argv)


def _launcher():
    """test_isaacgym_amd/launch.py loaded by path: the parent must not import the
    package (it loads libmigym.so) before the ranks exist."""
    spec = importlib.util.spec_from_file_location("_mg_launch", os.path.join(ROOT, "test_isaacgym_amd", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# --------------------------------------------------------------------------- helpers
def graph_chunk(steps, cap=GRAPH_CHUNK_MAX):
    """Steps per captured graph: the largest divisor of the timed step count
    that is <= cap, so a timed region of `steps` replays steps / chunk graphs
    (one graph for --steps <= 64: the driver's 20-step region is one launch)."""
    return max(d for d in range(1, min(steps, cap) + 1) if steps % d == 0)


def bank_slots(chunk, at_least=64):
    """Action-bank size: a multiple of the graph chunk (each captured graph
    covers `chunk` consecutive slots), at least `at_least` slots."""
    return chunk * -(-at_least // chunk)


def capture_chunks(step, slots, chunk):
    """hipGraphs of `chunk` consecutive steps each, covering the action slots
    0..slots-1 in order (graph c runs step(c * chunk) .. step(c * chunk + chunk - 1)),
    sharing one memory pool. Replaying graph (k / chunk) % len runs exactly the
    steps the eager loop would run for k .. k + chunk - 1."""
    import torch
    graphs, pool = [], None
    for c in range(slots // chunk):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            for j in range(c * chunk, (c + 1) * chunk):
                step(j)
        pool = g.pool()
        graphs.append(g)
    return graphs


def kernel_stats(sim, n_launches, run):
    """Run `run()` (n_launches eager simulate calls) with dispatch-timestamp
    events on, then return (avg_ms, min_ms, launches) of the step kernels."""
    import ctypes
    import torch
    from test_isaacgym_amd import _native as N
    N.lib.mg_set_kernel_timing(sim.native, 1)
    try:
        run()
        torch.cuda.synchronize()
    finally:
        N.lib.mg_set_kernel_timing(sim.native, 0)
    avg, lo = ctypes.c_float(), ctypes.c_float()
    used = N.lib.mg_step_time_stats(sim.native, min(n_launches, 256), ctypes.byref(avg), ctypes.byref(lo), None)
    if used <= 0:
        return None, None, 0
    # a simulate with more launches than the library's timer slots would sum
    # only the first kKern kernels: refuse the number, loudly
    missed = N.lib.mg_step_untimed_launches(sim.native, int(used))
    if missed != 0:
        raise RuntimeError("kernel timing: %d launch(es) per simulate ran untimed (mg_step_untimed_launches); "
                           "the summed kernel time would undercount" % missed)
    return avg.value, lo.value, int(used)


STEP_FUSION_NOTE = ("opt-in step fusion (gym.set_step_fusion(sim, STEP_FUSION_ALL)): every step writes the "
                    "action into the source before its set and never touches it again before simulate, so "
                    "the deferred read equals Isaac Gym's copy-at-set (checked by version counters); the step "
                    "kernel writes the bound root / rigid-body tensors itself and the refreshes after it "
                    "launch nothing (STEP_OUT); every API call of the loop is still made; off by default "
                    "in the library")


def fuse_in_capture(sim):
    """Opt in to step fusion, inside captures too (STEP_FUSION_ALL): every
    (captured) step of this leg is set -> simulate -> refresh, so each set is
    consumed by the simulate after it and its source is not written in between
    (include/migym.h; the S3 leg's frames end with the DOF setters and keep the
    default, no fusion)."""
    from isaacgym import gymapi
    gymapi.acquire_gym().set_step_fusion(sim, gymapi.STEP_FUSION_ALL)


def load_pmc(name):
    """Committed rocprofv3 PMC summary (profiles/<round>_pmc_<name>.json, newest
    round first, written by profiles/collect_pmc.py): (dict, file) or (None, None)."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(ROOT, "profiles", "%s_pmc_%s.json" % (rnd, name))
        if os.path.exists(path):
            with open(path) as f:
                return json.load(f), os.path.relpath(path, ROOT)
    return None, None


def rigid_roofline(n, kern_ms, kmin, launches, segment, step_out=True):
    """step_out: the timed launches ran with STEP_FUSION_STEP_OUT (the kernel
    writes the bound rigid-body and root tensors: SIM_OUT_BYTES_PER_ENV)."""
    bpe = SIM_OUT_BYTES_PER_ENV if step_out else SIM_BYTES_PER_ENV
    bytes_launch = bpe * n
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9 if kern_ms else None
    pmc, pmc_file = load_pmc("rigid_%d" % n)
    return {"bound": "hbm", "kernel": "k_rigid_step1",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
            "traffic_source": pmc_file,
            "traffic_read_write": ([pmc["fetch_kib_raw"] * 1024 * pmc["read_factor_calibrated"],
                                    pmc["write_kib_raw"] * 1024 * pmc.get("write_calibration", {}).get("write_factor", 1.0)]
                                   if pmc and "fetch_kib_raw" in pmc and "read_factor_calibrated" in pmc else None),
            "algorithmic_bytes_per_launch": bytes_launch,
            "algorithmic_bytes_per_env": bpe,
            "algorithmic_bytes_note": ("376 B simulate share (SURVEY.md §8d) + the rigid-body and root rows the "
                                       "kernel writes with the refresh fused into it (2 x (52 + 52) B)"
                                       if step_out else "376 B simulate share (SURVEY.md §8d)"),
            "kernel_ms_avg": kern_ms, "kernel_ms_min": kmin, "kernel_launches_timed": launches,
            "kernel_timing": "dispatch timestamps of every k_rigid_step launch (hipExtLaunchKernelGGL start/stop "
                             "events, the interval rocprofv3 reports) over %s" % segment,
            "kernel_bytes_needed_per_env": kernel_bytes_needed(step_out)}


def kernel_bytes_needed(step_out):
    """What k_rigid_step1 itself must move per servo env (the
    traffic accounting), beside SURVEY's 376 / 584 B pricing: the servo
    templates' mass and shape rows are wave-uniform (0 B per body), while the
    contact force and the ground-patch record (MG_FP_N = 16 floats per body:
    the anchor count, read and written every step, and the normal plus two
    anchor pairs, 60 B, read and written while the vehicle's patch is held)
    are not in SURVEY's share."""
    rd = {"state_in": 2 * 52, "patch_count": 2 * 4, "patch_anchors": 60}
    wr = {"state_out": 2 * 52, "contact_force": 2 * 12, "patch_count": 2 * 4, "patch_anchors": 60}
    if step_out:
        wr["rigid_body_and_root_rows"] = 2 * (52 + 52)
    return {"read": sum(rd.values()), "write": sum(wr.values()), "total": sum(rd.values()) + sum(wr.values()),
            "read_parts": rd, "write_parts": wr}


# --------------------------------------------------------------------------- CPU baseline
def cpu_threads():
    """(all host cores as os.cpu_count() reports them, the CPUs this process may
    run on, the cgroup CPU quota in CPUs or None)."""
    ncpu = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = ncpu
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return ncpu, aff, quota


def _cpu_scene(leg, n):
    """The bench legs' scenes on the host (no GPU pipeline): (sim, per-step
    hook(state, k), tgt). S1 teleports every root each step like the GPU leg;
    S2 draws new PD targets each step; S3 holds the Franka at its default DOF
    targets (the OSC controller is not part of the oracle)."""
    import numpy as np
    from isaacgym import gymapi
    from test_isaacgym_amd import scenes
    gym = gymapi.acquire_gym()
    if leg == "s1":
        sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=False)
        sim.build_model()
        roots = sim.model_arrays["actor_root_body"]
        acts = scenes.servo_actions(n, 16, "cpu", seed=0).numpy()

        def hook(st, tgt, k):
            st[roots, 3:10] = acts[k % len(acts)]
        return sim, hook, None
    if leg == "s2":
        sim, _ = scenes.gimbal_scene(gym, n, use_gpu_pipeline=False)
        sim.build_model()
        tg = scenes.gimbal_targets(n, 16, "cpu", seed=0).numpy()
        tgt = np.zeros((3 * n, 3), np.float32)

        def hook(st, tgt, k):
            tgt[:, 0] = tg[k % len(tg)]
        return sim, hook, tgt
    if leg == "s6":
        sim, _ = scenes.ball_pile_scene(gym, n, use_gpu_pipeline=False)
        sim.build_model()
        p, m = sim.mg_params(), sim.mg_model()
        import oracle
        st0 = sim.model_arrays["body_state0"]
        dof0 = sim.model_arrays["dof_state0"].copy()
        for _ in range(90):   # the GPU leg times the collapsed piles: drop them first
            oracle.step_threads(p, m, st0, dof0, max(1, cpu_threads()[1]))
        return sim, (lambda st, tgt, k: None), None
    sim, info = scenes.franka_scene(gym, n, use_gpu_pipeline=False)
    sim.build_model()
    nd = sim.model_arrays["dof_state0"].shape[0]
    tgt = np.zeros((nd, 3), np.float32)
    tgt[:, 0] = np.tile(np.asarray(info["default_dof_pos"], np.float32), nd // 9)
    return sim, (lambda st, tgt, k: None), tgt


def cpu_leg(leg, n, seconds, thread_counts):
    """env-steps/s of oracle.step_threads (the C restatement on OpenMP host
    threads) on the leg's n-env scene, per thread count, each for ~seconds."""
    import numpy as np
    import oracle
    sim, hook, tgt = _cpu_scene(leg, n)
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    dof = sim.model_arrays["dof_state0"].copy()
    if tgt is None:
        tgt = np.zeros((max(dof.shape[0], 1), 3), np.float32)
    cforce = np.zeros((st.shape[0], 3), np.float32)
    out = {}
    for nt, secs in thread_counts:
        steps, t0 = 0, time.perf_counter()
        while True:
            hook(st, tgt, steps)
            oracle.step_threads(p, m, st, dof, nt, tgt=tgt, cforce=cforce)
            steps += 1
            el = time.perf_counter() - t0
            if (el >= secs and steps >= 3) or steps >= 100000:
                break
        out[nt] = (n * steps / el, steps, el)
    return out


def cpu_baseline(seconds=10.0):
    """SURVEY.md §8d "CPU beside it" / BASELINE.md §3: the oracle (C restatement,
    "port") on the host's cores (OpenMP, num_threads set explicitly), on the
    three bench scenes at 4096 envs: S1 (the headline), S2, S3.

    `cores` is the CPUs this process can actually use: os.cpu_count() bounded by
    the affinity mask and the cgroup CPU quota (the GPU box reports 256 CPUs but
    grants a quota of 16; 256 OpenMP threads under that quota are throttled to a
    few steps per second, so that figure is reported beside it, not as the
    baseline). Also 1 thread for S1."""
    ncpu, aff, quota = cpu_threads()
    usable = max(1, min(ncpu, aff, int(quota) if quota else ncpu))
    n = ENVS_PER_GPU
    extra = [(ncpu, seconds * 0.1)] if ncpu != usable else []
    s1 = cpu_leg("s1", n, seconds, [(usable, seconds * 0.4), (1, seconds * 0.2)] + extra)
    s2 = cpu_leg("s2", n, seconds, [(usable, seconds * 0.3)] + extra)
    s3 = cpu_leg("s3", n, seconds, [(usable, seconds * 0.5)] + extra)
    s6 = cpu_leg("s6", n, seconds, [(usable, seconds * 0.3)])

    def leg(r, what):
        v, steps, el = r[usable]
        d = {"value": v, "unit": "env-steps/s", "cores": usable, "steps": steps, "seconds": el, "sample": what}
        if ncpu in r and ncpu != usable:
            d["value_all_host_threads"] = r[ncpu][0]
        return d
    out = leg(s1, "%d simulate() steps of the 4096-env servo scene with random root teleports (S1)" % s1[usable][1])
    out.update({"kind": "port", "host_cpu_count": ncpu, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                "single_thread_value": s1[1][0],
                "note": "oracle/migym_oracle.c (CPU restatement, not Isaac Gym: the reference engine is a closed "
                        "binary absent here) via oracle_step_mt, OpenMP with num_threads = cores = os.cpu_count() "
                        "bounded by the affinity mask and the cgroup CPU quota; value_all_host_threads = the same "
                        "with os.cpu_count() threads, throttled by that quota",
                "s2": leg(s2, "%d simulate() steps of 4096 3-DOF gimbals under random PD targets (S2)" % s2[usable][1]),
                "s3": leg(s3, "%d simulate() steps of 4096 Franka cube-pick envs holding their default DOF "
                              "targets (S3 physics only; the OSC controller is not in the oracle)" % s3[usable][1]),
                "s6": leg(s6, "%d simulate() steps of 4096 envs of 1080_balls_of_solitude.py's 30-ball pyramid, "
                              "after 90 frames of collapse (S6)" % s6[usable][1])})
    out["sample"] = out["sample"] + "; S2, S3 and S6 under s2 / s3 / s6"
    return out


# --------------------------------------------------------------------------- secondary legs (N = 1)
def gimbal_rate(n, steps, warmup, dev, use_graph=True):
    """S2 servo-arm: n fixed-base 3-DOF gimbals under random PD
    position targets; one step = set_dof_position_target_tensor -> simulate ->
    refresh DOF + rigid-body state. Returns env-steps/s and the step kernel time."""
    import torch
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes
    gym = gymapi.acquire_gym()
    sim, _ = scenes.gimbal_scene(gym, n, use_gpu_pipeline=True, device=dev.index or 0)
    gym.prepare_sim(sim)
    fuse_in_capture(sim)
    gym.acquire_dof_state_tensor(sim)
    gym.acquire_rigid_body_state_tensor(sim)
    chunk = graph_chunk(steps)
    tg = scenes.gimbal_targets(n, bank_slots(chunk), dev, seed=0)

    def step(k):
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k % tg.shape[0]]))
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)

    for k in range(warmup):
        step(k)
    kms, kmin, used = kernel_stats(sim, KERNEL_TIMED_LAUNCHES,
                                   lambda: [step(warmup + k) for k in range(KERNEL_TIMED_LAUNCHES)])
    graphs = None
    base = -(-(warmup + KERNEL_TIMED_LAUNCHES + chunk) // chunk) * chunk
    if use_graph:
        try:
            graphs = capture_chunks(step, tg.shape[0], chunk)
            graphs[(base // chunk - 1) % len(graphs)].replay()
        except Exception as ex:
            print("*** bench: S2 hipGraph capture failed (%s); timing the eager loop" % ex, file=sys.stderr)
            graphs = None
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if graphs is not None:
        for i in range(steps // chunk):
            graphs[(base // chunk + i) % len(graphs)].replay()
    else:
        for k in range(steps):
            step(base + k)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    gym.destroy_sim(sim)
    ach = S2_BYTES_PER_ENV * n / (kms * 1e-3) / 1e9 if kms else None
    pmc, pmc_file = load_pmc("gimbal_%d" % n)
    # four lanes per gimbal when the launch fits one resident round (mg_chain.hip MG_CHAIN_QUAD_MAX)
    kname = "k_artic_chain_q<4>" if n * 4 <= 64 * 1024 else "k_artic_chain<4>"
    return {"envs": n, "env_steps_per_s": n * steps / el, "ms_per_step": 1e3 * el / steps,
            "timed_loop": ("hipGraph replay, %d steps per graph" % chunk) if graphs is not None else "eager Python loop",
            "kernel": "S2 articulation step (%s)" % kname, "kernel_ms_avg": kms, "kernel_ms_min": kmin,
            "kernel_launches_timed": used, "algorithmic_bytes_per_env": S2_BYTES_PER_ENV,
            "kernel_achieved_GBs": ach,
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": ach, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": (ach / HBM_PEAK_GBS) if ach else None,
                         "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None, "traffic_source": pmc_file,
                         "algorithmic_bytes_per_launch": S2_BYTES_PER_ENV * n,
                         "note": "SURVEY.md §8d S2: 532 B per env-step (DOF state in/out, targets, drive params, "
                                 "link mass properties, target set, DOF + rigid-body refresh) priced on the "
                                 "simulate kernel's own dispatch-timestamp duration"}}


def franka_rate(n, steps, warmup, dev, use_graph=True):
    """S3 Franka cube pick: examples/franka_cube_ik_osc.py's
    loop at n envs, OSC controller: simulate -> fetch_results -> refresh rigid-body /
    DOF / Jacobian / mass-matrix tensors -> the script's controller on the device
    (test_isaacgym_amd.franka_control) -> set DOF position targets and efforts.
    Returns env-steps/s and the coupled-step kernel time."""
    import torch
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import _native as N, franka_control, scenes
    gym = gymapi.acquire_gym()
    sim, info = scenes.franka_scene(gym, n, use_gpu_pipeline=True, device=dev.index or 0)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    jac = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, "franka"))
    mm = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, "franka"))
    ctl = franka_control.CubePick(n, info["init_pos"], info["init_rot"], info["default_dof_pos"], dev)
    h = info["hand_index"]
    bi = torch.tensor(info["box_idxs"], device=dev)
    hi = torch.tensor(info["hand_idxs"], device=dev)
    j_eef = jac[:, h - 1, :, :7]
    mm7 = mm[:, :7, :7]
    dp = dof[:, 0].view(n, 9, 1)
    dv = dof[:, 1].view(n, 9, 1)
    lifted = torch.zeros(n, dtype=torch.bool, device=dev)

    def step():
        gym.simulate(sim)
        gym.fetch_results(sim, False)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_jacobian_tensors(sim)
        gym.refresh_mass_matrix_tensors(sim)
        pa, ea = ctl.step(rb, dp, dv, j_eef, mm7, bi, hi)
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(pa))
        gym.set_dof_actuation_force_tensor(sim, gymtorch.unwrap_tensor(ea))
        lifted.logical_or_(rb[bi, 2] > 0.55)

    for _ in range(warmup):
        step()
    kms, kmin, used = kernel_stats(sim, 100, lambda: [step() for _ in range(100)])
    torch.cuda.synchronize(dev)
    t_e = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize(dev)
    eager_ms = 1e3 * (time.perf_counter() - t_e) / 10
    graph = None
    chunk = graph_chunk(steps, 8)
    if use_graph:
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(3):
                    step()
            torch.cuda.current_stream(dev).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(chunk):
                    step()
            graph.replay()
        except Exception as ex:
            print("*** bench: S3 hipGraph capture failed (%s); timing the eager loop" % ex, file=sys.stderr)
            graph = None
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if graph is not None:
        for _ in range(steps // chunk):
            graph.replay()
    else:
        for _ in range(steps):
            step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ach = S3_BYTES_PER_ENV * n / (kms * 1e-3) / 1e9 if kms else None
    pmc, pmc_file = load_pmc("env_step_%d" % n)
    out = {"envs": n, "env_steps_per_s": n * steps / el, "ms_per_step": 1e3 * el / steps,
           "kernel": "S3 coupled step: per substep k_env_np<16,16,16> (narrow phase) + k_env_step<16,16>, "
                     "2 substeps (the frame's kernels summed)", "kernel_ms_avg": kms, "kernel_ms_min": kmin,
           "kernel_launches_timed": used,
           "roofline": {"bound": "hbm", "kernel": "k_env_np + k_env_step (one frame)", "achieved": ach,
                        "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": (ach / HBM_PEAK_GBS) if ach else None,
                        # per frame (the summed launches the roofline prices); older summaries kept
                        # the per-frame value under hbm_bytes_per_launch
                        "traffic": (pmc.get("hbm_bytes_per_frame", pmc.get("hbm_bytes_per_launch"))
                                    if pmc else None), "traffic_unit": "bytes per frame", "traffic_source": pmc_file,
                        "traffic_read_factor_borrowed": pmc.get("read_factor_borrowed", True) if pmc else None,
                        "algorithmic_bytes_per_frame": S3_BYTES_PER_ENV * n,
                        "algorithmic_bytes_per_env": S3_BYTES_PER_ENV,
                        "note": "SURVEY.md §8d S3: 5,844 B per env-step (rigid-body refresh, DOF state, targets and "
                                "efforts, Jacobian, mass matrix, DOF / body constants, contact warm-start state) "
                                "priced on the frame's coupled-step kernels' summed dispatch-timestamp durations "
                                "(two substeps, each a narrow-phase and a step launch); latency bound (16 lanes per "
                                "env, 1024 waves per launch on 1024 SIMDs): DESIGN.md §3.6.2, §5"},
           "coupled_envs": int(N.lib.mg_num_coupled_envs(sim.native)),
           "cubes_lifted_frac": float(lifted.float().mean()),
           "controller": "OSC (franka_cube_ik_osc.py:59-79,348-410) on the device",
           "timed_loop": ("hipGraph replay, %d steps per graph" % chunk) if graph is not None else "eager Python loop",
           "eager_ms_per_step": eager_ms}
    gym.destroy_sim(sim)
    return out


def camera_rate(n, steps, warmup, dev, use_graph=True, width=1600, height=900):
    """S5 (config 5, test11_servo_vecenv_camerazoom.py): the S1 servo step plus
    one 1600x900 camera per env on the UAV (local (5, 0, 0), FOLLOW_TRANSFORM,
    horizontal FOV 30 degrees) rendered into a GPU color tensor every step by
    render_all_camera_sensors. Returns env-steps/s and the render kernel's
    time and write bandwidth (roofline: the kernel streams W*H*4 bytes per
    camera to HBM; reads are the env's few shapes)."""
    import numpy as np
    import torch
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import _native as N, scenes
    gym = gymapi.acquire_gym()
    sim, envs = scenes.servo_scene(gym, n, use_gpu_pipeline=True, device=dev.index or 0)
    imgs = scenes.attach_servo_cameras(gym, sim, envs, width, height, 30.0)
    gym.prepare_sim(sim)
    fuse_in_capture(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gym.acquire_rigid_body_state_tensor(sim)
    acts = scenes.servo_actions(n, 16, dev, seed=5)

    def step(k):
        root[:, 3:10] = acts[k % acts.shape[0]]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, False)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.render_all_camera_sensors(sim)

    gym.refresh_actor_root_state_tensor(sim)
    for k in range(warmup):
        step(k)
    rms = []
    N.lib.mg_set_kernel_timing(sim.native, 1)
    for k in range(20):
        step(warmup + k)
        rms.append(N.lib.mg_last_render_ms(sim.native))
    N.lib.mg_set_kernel_timing(sim.native, 0)
    torch.cuda.synchronize(dev)
    graphs = None
    if use_graph:
        try:
            graphs, pool = [], None
            for j in range(acts.shape[0]):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    step(j)
                pool = g.pool()
                graphs.append(g)
            for j in range(2):
                graphs[(warmup + 20 + j) % len(graphs)].replay()
        except Exception as ex:
            print("*** bench: S5 hipGraph capture failed (%s); timing the eager loop" % ex, file=sys.stderr)
            graphs = None
    base = warmup + 22
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(steps):
        if graphs is not None:
            graphs[(base + k) % len(graphs)].replay()
        else:
            step(base + k)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    lit = float((imgs[0][0][..., :3].amax(-1) > 0).float().mean())
    lit_all = float(np.mean([float((imgs[i][0][..., :3].amax(-1) > 0).float().mean())
                             for i in range(0, n, max(1, n // 16))]))
    gym.destroy_sim(sim)
    rms = [r for r in rms if r > 0]
    rk = float(np.mean(rms)) if rms else float("nan")
    wbytes = n * width * height * 4
    ach = wbytes / (rk * 1e-3) / 1e9
    pmc, pmc_file = load_pmc("render_%dx%dx%d" % (n, width, height))
    traffic = pmc.get("write_bytes_per_launch_from_WRITE_SIZE_KB") if pmc else None
    return {"envs": n, "cameras": n, "resolution": [width, height], "env_steps_per_s": n * steps / el,
            "ms_per_step": 1e3 * el / steps, "timed_loop": "hipGraph replay" if graphs is not None else "eager",
            "kernel": "k_render", "kernel_ms_avg": rk, "kernel_launches_timed": len(rms),
            "image_bytes_per_launch": wbytes,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": pmc_file},
            "env0_non_sky_fraction": lit, "sampled_cameras_non_sky_fraction": lit_all}


def pile_rate(n, steps, warmup, dev, use_graph=True):
    """S6 ball piles: examples/1080_balls_of_solitude.py's scene at n envs (30
    balls per env in one collision group, y-up, 1 substep, TGS 4/1; the script
    runs 36) — every env a pile stepped by k_pile_step. One
    step = simulate -> fetch_results -> refresh the rigid-body tensor. Timed
    from the pyramids' collapse on (the warm-up drops them: 60 frames to the
    ground), replayed as hipGraphs."""
    import torch
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import _native as N, scenes
    gym = gymapi.acquire_gym()
    sim, envs = scenes.ball_pile_scene(gym, n, use_gpu_pipeline=True, device=dev.index or 0)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))

    def step():
        gym.simulate(sim)
        gym.fetch_results(sim, False)
        gym.refresh_rigid_body_state_tensor(sim)

    for _ in range(warmup):
        step()
    kms, kmin, used = kernel_stats(sim, 100, lambda: [step() for _ in range(100)])
    graph, chunk = None, graph_chunk(steps, 16)
    if use_graph:
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(3):
                    step()
            torch.cuda.current_stream(dev).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(chunk):
                    step()
            graph.replay()
        except Exception as ex:
            print("*** bench: S6 hipGraph capture failed (%s); timing the eager loop" % ex, file=sys.stderr)
            graph = None
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if graph is not None:
        for _ in range(steps // chunk):
            graph.replay()
    else:
        for _ in range(steps):
            step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    y = rb[:, 1].view(n, S6_BALLS)
    ach = S6_BYTES_PER_ENV * n / (kms * 1e-3) / 1e9 if kms else None
    pmc, pmc_file = load_pmc("pile_%d" % n)
    out = {"envs": n, "bodies": n * S6_BALLS, "env_steps_per_s": n * steps / el, "ms_per_step": 1e3 * el / steps,
           "kernel": "k_pile_step (one launch per simulate)", "kernel_ms_avg": kms, "kernel_ms_min": kmin,
           "kernel_launches_timed": used, "pile_envs": int(N.lib.mg_num_pile_envs(sim.native)),
           "roofline": {"bound": "hbm", "kernel": "k_pile_step", "achieved": ach, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": (ach / HBM_PEAK_GBS) if ach else None,
                        "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None, "traffic_source": pmc_file,
                        "algorithmic_bytes_per_env": S6_BYTES_PER_ENV,
                        "note": "30 balls x (state in 52 + out 52 + mass 44 + contact force 12 B); the kernel is "
                                "bound by its per-env serial work (narrow phase of 465 candidate pairs, the "
                                "colouring, the colour-by-colour sweeps), not by HBM: DESIGN.md §3.10"},
           "balls_height_range_m": [float(y.min()), float(y.max())],
           "timed_loop": ("hipGraph replay, %d steps per graph" % chunk) if graph is not None else "eager Python loop"}
    gym.destroy_sim(sim)
    return out


def s1_rate(n, steps, dev, use_graph=True, fused=True, seed=1, unfused_kernel=False):
    """S1 at `n` envs on one GPU: the same tensor-API step as the headline;
    k_rigid_step's own duration over KERNEL_TIMED_LAUNCHES eager launches and the
    graph-replayed step rate. fused=False runs the library default (no step
    fusion: the set is a scatter launch, the refreshes are gathers), which is
    what an unmodified test10 gets. unfused_kernel: also time the kernel with
    fusion off (the large-N leg's A/B)."""
    import torch
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=True, device=dev.index or 0)
    gym.prepare_sim(sim)
    if fused:
        fuse_in_capture(sim)
    else:
        gym.set_step_fusion(sim, 0)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gym.acquire_rigid_body_state_tensor(sim)
    gym.acquire_dof_state_tensor(sim)
    # graphs of `chunk` steps over a bank of `slots` actions (at large N, 16 slots
    # of 2n root rows each and graphs of at most 16 steps)
    chunk = graph_chunk(steps, 16 if n > 65536 else GRAPH_CHUNK_MAX)
    acts = scenes.servo_actions(n, bank_slots(chunk, 16), dev, seed=seed)

    def step(k):
        root[:, 3:10] = acts[k % acts.shape[0]]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, False)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_dof_state_tensor(sim)

    gym.refresh_actor_root_state_tensor(sim)
    warm = 30        # the clocks and caches settle before the kernel-timing segment
    for k in range(warm):
        step(k)
    kms, kmin, used = kernel_stats(sim, KERNEL_TIMED_LAUNCHES,
                                   lambda: [step(warm + k) for k in range(KERNEL_TIMED_LAUNCHES)])
    assert acts.shape[0] % chunk == 0
    graphs = None
    base = -(-(warm + KERNEL_TIMED_LAUNCHES) // chunk) * chunk
    if use_graph:
        try:
            graphs = capture_chunks(step, acts.shape[0], chunk)
            graphs[(base // chunk) % len(graphs)].replay()
            base += chunk
        except Exception as ex:
            print("*** bench: S1 (%d envs) hipGraph capture failed (%s); timing the eager loop" % (n, ex),
                  file=sys.stderr)
            graphs = None
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if graphs is not None:
        for i in range(steps // chunk):
            graphs[(base // chunk + i) % len(graphs)].replay()
    else:
        for k in range(steps):
            step(base + k)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    out = {"envs": n, "env_steps_per_s": n * steps / el, "ms_per_step": 1e3 * el / steps, "steps": steps,
           "step_fusion": "STEP_FUSION_ALL" if fused else "off (library default)",
           "timed_loop": ("hipGraph replay, %d steps per graph" % chunk) if graphs is not None else "eager",
           "roofline": rigid_roofline(n, kms, kmin, used, "%d eager steps after a %d-step warm-up" % (used, warm),
                                      step_out=fused)}
    if unfused_kernel:
        # the same kernel without the fused root-state read (mg_set_fusion 0: the set
        # is a scatter launch and the step reads the SoA state): at this size the
        # fused read costs the kernel the user rows' other-template halves (test10's
        # actor rows alternate UAV / vehicle, whose waves run apart: DESIGN.md §3.2)
        prev = gym.set_step_fusion(sim, 0)
        ukms, ukmin, uused = kernel_stats(sim, KERNEL_TIMED_LAUNCHES,
                                          lambda: [step(k) for k in range(KERNEL_TIMED_LAUNCHES)])
        gym.set_step_fusion(sim, prev)
        out["roofline_unfused"] = rigid_roofline(n, ukms, ukmin, uused,
                                                 "%d eager steps with step fusion off (scatter launch, then the "
                                                 "step kernel on the SoA state)" % uused, step_out=False)
    gym.destroy_sim(sim)
    return out


def large_n_rate(n, steps, dev, use_graph=True):
    """S1 at `n` envs (SURVEY.md §8d's large-N regime point), fused as the headline."""
    return s1_rate(n, steps, dev, use_graph, fused=True, seed=1, unfused_kernel=True)


def s1_cpu_pipeline_rate(n, steps, warmup):
    """test10_servo_vecenv.py's own mode (:130 sets physx.use_gpu only; SURVEY.md
    §0.7): use_gpu_pipeline False, so the state tensors are host tensors. One step
    = the actions written into the host root tensor, set (H2D), simulate,
    fetch_results(sim, True), refresh root / rigid-body / DOF (D2H), the eager
    Python loop (host tensors cannot be captured). The physics is the same GPU
    step; the difference to the GPU pipeline is the PCIe mirror and the sync."""
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gym.acquire_rigid_body_state_tensor(sim)
    gym.acquire_dof_state_tensor(sim)
    assert root.device.type == "cpu"
    acts = scenes.servo_actions(n, 16, "cpu", seed=2)

    def step(k):
        root[:, 3:10] = acts[k % acts.shape[0]]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_dof_state_tensor(sim)

    gym.refresh_actor_root_state_tensor(sim)
    for k in range(warmup):
        step(k)
    t0 = time.perf_counter()
    for k in range(steps):
        step(warmup + k)
    el = time.perf_counter() - t0
    gym.destroy_sim(sim)
    return {"envs": n, "env_steps_per_s": n * steps / el, "ms_per_step": 1e3 * el / steps, "steps": steps,
            "pipeline": "CPU (host state tensors: H2D set; fetch_results(sim, True) stages the refreshed kinds in one "
                        "D2H round trip, mg_fetch_host_state; the refreshes copy from it)",
            "timed_loop": "eager Python loop (host tensors)",
            "bytes_over_pcie_per_step": n * 2 * 13 * 4 * 3}


# --------------------------------------------------------------------------- dry run (no GPU)
def dry_run(args, world, rank):
    """Launcher / sharding rehearsal without a GPU: every rank builds its shard of
    the servo scene (CPU pipeline, no simulate), the root-state tensors are
    gathered over gloo, and rank 0 checks them against one sim of all envs."""
    import numpy as np
    import torch.distributed as dist
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes, sharding
    gym = gymapi.acquire_gym()
    n = args.envs
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=False, env_offset=rank * n, grid_envs=world * n)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    g = sharding.all_gather_rows(root) if world > 1 else root
    if rank == 0:
        ref, _ = scenes.servo_scene(gym, world * n, use_gpu_pipeline=False)
        want = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(ref)).numpy()
        print(json.dumps({"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": world,
                          "dry_run": True, "backend": dist.get_backend() if world > 1 else None,
                          "envs_per_rank": n, "gathered_rows": int(g.shape[0]),
                          "layout_matches_single_sim": bool(np.array_equal(g.numpy(), want))}), flush=True)
    if world > 1:
        dist.barrier()


# --------------------------------------------------------------------------- main
def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not under torch.distributed.run: start one process per GPU ourselves,
        # before this process touches HIP
        rc, codes = _launcher().spawn_ranks([os.path.abspath(__file__)] + sys.argv[1:], args.gpus)
        if rc != 0:
            print("*** bench: rank exit codes %s" % codes, file=sys.stderr)
        sys.exit(rc)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    from test_isaacgym_amd import sharding
    ndev = 0 if args.dry_run else torch.cuda.device_count()
    backend = args.backend if args.backend != "auto" else sharding.backend_for(world, ndev)
    if args.dry_run:
        backend = "gloo"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    if args.dry_run:
        dry_run(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    if ndev <= 0:
        raise SystemExit("bench: no GPU visible (use --dry-run for the host rehearsal)")
    dev_index = local % ndev
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    cdev = dev if backend == "nccl" else torch.device("cpu")      # where collective operands live

    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes

    gym = gymapi.acquire_gym()
    n = args.envs
    # rank k owns global envs [k n, (k+1) n), placed at their global grid cells
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=True, device=dev_index, env_offset=rank * n,
                                grid_envs=world * n)
    gym.prepare_sim(sim)
    fuse_in_capture(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gym.acquire_rigid_body_state_tensor(sim)
    gym.acquire_dof_state_tensor(sim)
    chunk = graph_chunk(args.steps)
    acts = scenes.servo_actions(n, bank_slots(chunk), dev, seed=rank)
    gathered = args.allgather and world > 1

    def step(k, gather=gathered):
        root[:, 3:10] = acts[k % acts.shape[0]]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, False)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_dof_state_tensor(sim)
        if gather:
            sharding.all_gather_rows(root)      # RCCL over xGMI: (world * 2n, 13) observation

    gym.refresh_actor_root_state_tensor(sim)
    if args.pmc_calibrate:
        every = torch.arange(root.shape[0], dtype=torch.int32, device=dev)
        for _ in range(4):
            gym.set_actor_root_state_tensor_indexed(sim, gymtorch.unwrap_tensor(root), gymtorch.unwrap_tensor(every),
                                                    root.shape[0])
            gym.refresh_actor_root_state_tensor(sim)
    k = 0
    for _ in range(args.warmup):
        step(k)
        k += 1
    # kernel-timing segment: dispatch timestamps on, >= 100 eager launches
    k0 = k
    kern_ms, kmin, used = kernel_stats(sim, KERNEL_TIMED_LAUNCHES,
                                       lambda: [step(k0 + j) for j in range(KERNEL_TIMED_LAUNCHES)])
    k += KERNEL_TIMED_LAUNCHES
    # eager segment, timing off: what an unmodified script's Python loop costs
    neager = 32
    torch.cuda.synchronize(dev)
    t_e = time.perf_counter()
    for _ in range(neager):
        step(k)
        k += 1
    torch.cuda.synchronize(dev)
    eager_ms = 1e3 * (time.perf_counter() - t_e) / neager

    # hipGraph replay: graphs of `chunk` consecutive captured steps (step j applies
    # acts[j]), sharing one memory pool; the replayed sequence is exactly the eager
    # loop's, and one graph launch is paid per `chunk` steps instead of per step
    graphs = None
    if not args.eager and not gathered:
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for j in range(3):
                    step(k + j)
            torch.cuda.current_stream(dev).wait_stream(side)
            graphs = capture_chunks(step, acts.shape[0], chunk)
            # capture does not run the work: replay one chunk to settle, then
            # time from the next chunk-aligned slot
            k = -(-(k + 3) // chunk) * chunk
            graphs[(k // chunk) % len(graphs)].replay()
            k += chunk
        except Exception as ex:          # capture unsupported here: time the eager loop
            print("*** bench: hipGraph capture failed (%s); timing the eager loop" % ex, file=sys.stderr)
            graphs = None

    def run_steps(k_first, nsteps):
        if graphs is not None:
            for i in range(nsteps // chunk):
                graphs[(k_first // chunk + i) % len(graphs)].replay()
        else:
            for j in range(nsteps):
                step(k_first + j)

    def timed(fn, reps):
        """Each repeat bracketed by barrier + synchronize; returns the per-repeat
        elapsed seconds of every rank, shape (world, reps)."""
        els = []
        for r in range(reps):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn(r)
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            els.append(time.perf_counter() - t0)
        t = torch.tensor(els, dtype=torch.float64, device=cdev)
        if world > 1:
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
            return [p.cpu().tolist() for p in parts]
        return [els]

    reps = max(1, args.repeats)
    per_rank = timed(lambda r: run_steps(k + r * args.steps, args.steps), reps)
    k += reps * args.steps
    el_max = [max(per_rank[q][r] for q in range(world)) for r in range(reps)]
    el = statistics.median(el_max)
    value = world * n * args.steps / el
    ms_per_step = 1e3 * el / args.steps

    # optional RCCL all-gather of the observation (N > 1): the gather alone and
    # the eager step loop with one gather per step
    gather_leg = None
    if world > 1 and not gathered:
        gsteps = max(args.steps, 20)
        g_el = timed(lambda r: [sharding.all_gather_rows(root) for _ in range(gsteps)], 3)
        g_ms = 1e3 * statistics.median([max(g_el[q][r] for q in range(world)) for r in range(3)]) / gsteps
        s_el = timed(lambda r: [step(k + j, gather=True) for j in range(gsteps)], 1)
        s_ms = 1e3 * max(s_el[q][0] for q in range(world)) / gsteps
        k += gsteps
        rb = root.numel() * root.element_size()
        gather_leg = {"backend": backend, "bytes_per_rank": rb, "bytes_gathered": rb * world,
                      "ms_per_gather": g_ms, "GB_per_s_received": rb * (world - 1) / (g_ms * 1e-3) / 1e9,
                      "step_with_gather_ms": s_ms,
                      "env_steps_per_s_with_gather": world * n / (s_ms * 1e-3),
                      "loop": "eager Python loop: step + all_gather_into_tensor of the (2n, 13) root state"}

    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded random root-state teleports, SURVEY.md §8d S1)",
            "config": {
                "workload": "S1 servo vecenv: test10_servo_vecenv.py scene (UAV + ground vehicle per env, "
                            "ground plane, dt 1/60, 2 substeps, TGS 6/1), random quat + linvel teleports "
                            "every step, full tensor-API loop",
                "envs_per_gpu": n,
                "global_envs": world * n,
                "parallelism": "env-sharded, one process per GPU (%s)%s" % (
                    backend if world > 1 else "single rank",
                    ", all-gather of root state in the loop" if gathered else ", no collectives in the loop"),
                "timed_loop": ("hipGraph replay: %d captured tensor-API steps per graph (every step's full "
                               "kernel sequence, action slot by slot), %d graph launches per timed region"
                               % (chunk, args.steps // chunk)) if graphs is not None
                              else "eager Python loop",
                "graph_chunk": chunk if graphs is not None else None,
                "action_slots": int(acts.shape[0]),
                "repeats": reps,
                "ms_per_step_runs": [1e3 * e / args.steps for e in el_max],
                "ms_per_step_per_rank": [[1e3 * e / args.steps for e in row] for row in per_rank],
                "eager_ms_per_step": eager_ms,
                "eager_note": "eager Python loop with kernel timing off (timing is opt-in: mg_set_kernel_timing)",
                "step_fusion": STEP_FUSION_NOTE,
            },
            "roofline": dict(rigid_roofline(n, kern_ms, kmin, used,
                                            "a %d-step eager segment after the warm-up" % KERNEL_TIMED_LAUNCHES),
                             note="working set of 4096 envs (~2.8 MB) sits in L2/MALL: the step is "
                                  "latency bound at this size (SURVEY.md §0.10); see large_n"),
        }
        if gather_leg:
            out["allgather"] = gather_leg
    if world == 1:
        # the secondary legs, each announced on stderr with its wall time (the one
        # JSON line stays the only stdout; a long default run keeps printing)
        legs = []
        if not args.no_large_n:
            legs.append(("large_n", lambda: large_n_rate(args.large_n, 64, dev, not args.eager)))
        if not args.no_default_legs:
            legs.append(("s1_default", lambda: s1_rate(ENVS_PER_GPU, min(args.steps, 300), dev, not args.eager,
                                                       fused=False, seed=3)))
            legs.append(("s1_cpu_pipeline", lambda: s1_cpu_pipeline_rate(1024, 100, 10)))
        if not args.no_gimbal:
            legs.append(("s2_servo_arm", lambda: gimbal_rate(ENVS_PER_GPU, min(args.steps, 300), 30, dev,
                                                             not args.eager)))
            if not args.no_large_n:
                legs.append(("s2_servo_arm.large_n", lambda: gimbal_rate(S2_LARGE_N, 64, 10, dev, not args.eager)))
        if not args.no_franka:
            legs.append(("s3_franka", lambda: franka_rate(ENVS_PER_GPU, min(args.steps, 300), 30, dev,
                                                          not args.eager)))
        if not args.no_cameras:
            legs.append(("s5_cameras", lambda: camera_rate(args.camera_envs, min(args.steps, 100), 10, dev,
                                                           not args.eager)))
        if not args.no_piles:
            legs.append(("s6_piles", lambda: pile_rate(args.pile_envs, min(args.steps, 300), 90, dev,
                                                       not args.eager)))
        if not args.no_cpu_baseline:
            legs.append(("cpu_baseline", lambda: cpu_baseline(args.cpu_seconds)))
        leg_s = {}
        for name, fn in legs:
            t_leg = time.perf_counter()
            res = fn()
            if "." in name:
                a, b = name.split(".")
                out[a][b] = res
            else:
                out[name] = res
            leg_s[name] = round(time.perf_counter() - t_leg, 2)
            print("bench: %s done in %.1f s" % (name, leg_s[name]), file=sys.stderr, flush=True)
        out["leg_wall_s"] = leg_s
    if rank == 0:
        print(json.dumps(out), flush=True)
    gym.destroy_sim(sim)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
