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
Weak scaling: every rank owns 4096 envs on its own GPU (one process per GPU,
launched by torch.distributed.run); envs never interact, so there is no
collective on the data path. --allgather adds the optional RCCL
all-gather of the root-state observation.

Prints ONE JSON line (rank 0). `roofline` prices the dominant kernel
(k_rigid_step, one launch per simulate) at SURVEY.md §8d's algorithmic bytes:
376 B per env per simulate (2 bodies x (state in 52 + state out 52 + mass
properties 44 + shape 40)), over its average duration taken from the kernel's own
dispatch timestamps (hipExtLaunchKernelGGL start / stop events on the simulate
stream; the interval rocprofv3 reports).
`cpu_baseline` times the C restatement (oracle/, "port") on the host cores (16 threads on the GPU box) on a
bounded sample of the same workload.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import _native as N  # noqa: E402
from test_isaacgym_amd import scenes, sharding  # noqa: E402

METRIC = "env-steps/sec (whole node), 4096 servo envs; 1/2/4/8-GPU scaling"
ENVS_PER_GPU = 4096
SIM_BYTES_PER_ENV = 376          # simulate share of the 688 B/env-step
STEP_BYTES_PER_ENV = 688         # whole tensor-API step
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec


def cpu_baseline(seconds=10.0, threads=None):
    """The oracle (C restatement) on the same 4096-env scene, on `threads` host
    cores: each step splits the bodies into contiguous ranges, one per thread
    (oracle.step's body_range; ctypes releases the GIL, envs are independent),
    plus a single-thread figure on the same sample for reference."""
    import concurrent.futures as cf
    import oracle
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, ENVS_PER_GPU, use_gpu_pipeline=False)
    sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    nb = st.shape[0]
    roots = sim.model_arrays["actor_root_body"]
    acts = scenes.servo_actions(ENVS_PER_GPU, 16, "cpu", seed=0).numpy()
    dof = np.zeros((0, 2), np.float32)
    cforce = np.zeros((nb, 3), np.float32)
    threads = threads or max(1, min(16, os.cpu_count() or 1))    # 16 = the GPU box's CPU share

    def run(nthr, budget):
        cuts = [nb * k // nthr for k in range(nthr + 1)]
        cuts = [c - (c % 2) for c in cuts]              # an env's two bodies stay in one range
        cuts[-1] = nb
        steps = 0
        with cf.ThreadPoolExecutor(nthr) as pool:
            t0 = time.perf_counter()
            while True:
                st[roots, 3:10] = acts[steps % len(acts)]
                list(pool.map(lambda k: oracle.step(p, m, st, dof, cforce=cforce,
                                                    body_range=(cuts[k], cuts[k + 1])), range(nthr)))
                steps += 1
                el = time.perf_counter() - t0
                if el >= budget and steps >= 5:
                    return steps, el

    s1, e1 = run(1, seconds * 0.3)
    sn, en = run(threads, seconds * 0.7) if threads > 1 else (s1, e1)
    return {"value": ENVS_PER_GPU * sn / en, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "single_thread_value": ENVS_PER_GPU * s1 / e1,
            "sample": "%d simulate() steps of the 4096-env servo scene with random root teleports, "
                      "oracle/migym_oracle.c on %d host threads, bodies split into contiguous ranges (%.1f s); "
                      "single thread: %d steps (%.1f s)" % (sn, threads, en, s1, e1)}


GRAPH_CHUNK = 8      # tensor-API steps captured per hipGraph (amortizes the graph launch)


def graph_chunk(steps, slots):
    """Steps per captured graph: GRAPH_CHUNK when it divides both the timed step
    count and the action-slot cycle, else the largest common divisor."""
    return math.gcd(math.gcd(steps, slots), GRAPH_CHUNK)


def capture_chunks(step, slots, chunk):
    """hipGraphs of `chunk` consecutive steps each, covering the action slots
    0..slots-1 in order (graph c runs step(c * chunk) .. step(c * chunk + chunk - 1)),
    sharing one memory pool. Replaying graph (k / chunk) % len runs exactly the
    steps the eager loop would run for k .. k + chunk - 1."""
    graphs, pool = [], None
    for c in range(slots // chunk):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            for j in range(c * chunk, (c + 1) * chunk):
                step(j)
        pool = g.pool()
        graphs.append(g)
    return graphs


def gimbal_rate(n, steps, warmup, dev, use_graph=True):
    """S2 servo-arm: n fixed-base 3-DOF gimbals under random PD
    position targets; one step = set_dof_position_target_tensor -> simulate ->
    refresh DOF + rigid-body state. Returns env-steps/s and the step kernel time."""
    gym = gymapi.acquire_gym()
    sim, _ = scenes.gimbal_scene(gym, n, use_gpu_pipeline=True, device=dev.index or 0)
    gym.prepare_sim(sim)
    gym.acquire_dof_state_tensor(sim)
    gym.acquire_rigid_body_state_tensor(sim)
    tg = scenes.gimbal_targets(n, 64, dev, seed=0)

    def step(k):
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k % 64]))
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)

    for k in range(warmup):
        step(k)
    torch.cuda.synchronize(dev)
    avg = ctypes.c_float()
    used = N.lib.mg_step_time_stats(sim.native, min(warmup // 2, 512), ctypes.byref(avg), None, None)
    # hipGraph replay, `chunk` captured steps per graph (as the S1 loop)
    graphs = None
    chunk = graph_chunk(steps, tg.shape[0])
    base = -(-(warmup + chunk) // chunk) * chunk       # chunk-aligned slot of the first timed step
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
    return {"envs": n, "env_steps_per_s": n * steps / el, "ms_per_step": 1e3 * el / steps,
            "timed_loop": ("hipGraph replay, %d steps per graph" % chunk) if graphs is not None else "eager Python loop",
            "kernel": "k_artic_world<4>", "kernel_ms_avg": avg.value if used > 0 else None,
            "algorithmic_bytes_per_env": 532}


def franka_rate(n, steps, warmup, dev, use_graph=True):
    """S3 Franka cube pick: examples/franka_cube_ik_osc.py's
    loop at n envs, OSC controller: simulate -> fetch_results -> refresh rigid-body /
    DOF / Jacobian / mass-matrix tensors -> the script's controller on the device
    (test_isaacgym_amd.franka_control) -> set DOF position targets and efforts.
    Returns env-steps/s and the coupled-step kernel time."""
    from test_isaacgym_amd import franka_control
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
    torch.cuda.synchronize(dev)
    avg = ctypes.c_float()
    used = N.lib.mg_step_time_stats(sim.native, min(warmup // 2, 512), ctypes.byref(avg), None, None)
    t_e = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize(dev)
    eager_ms = 1e3 * (time.perf_counter() - t_e) / 10
    graph = None
    chunk = math.gcd(steps, GRAPH_CHUNK)
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
    out = {"envs": n, "env_steps_per_s": n * steps / el, "ms_per_step": 1e3 * el / steps,
           "kernel": "k_env_step<16>", "kernel_ms_avg": avg.value if used > 0 else None,
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
    gym = gymapi.acquire_gym()
    sim, envs = scenes.servo_scene(gym, n, use_gpu_pipeline=True, device=dev.index or 0)
    imgs = scenes.attach_servo_cameras(gym, sim, envs, width, height, 30.0)
    gym.prepare_sim(sim)
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
    rms = []
    for k in range(warmup):
        step(k)
        if k >= warmup // 2:
            rms.append(N.lib.mg_last_render_ms(sim.native))
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
                graphs[(warmup + j) % len(graphs)].replay()
        except Exception as ex:
            print("*** bench: S5 hipGraph capture failed (%s); timing the eager loop" % ex, file=sys.stderr)
            graphs = None
    base = warmup + 2
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
    gym.destroy_sim(sim)
    rk = float(np.mean(rms)) if rms else float("nan")
    wbytes = n * width * height * 4
    ach = wbytes / (rk * 1e-3) / 1e9
    traffic = None        # HBM bytes per launch, committed rocprofv3 WRITE_SIZE pass (tools/gpu_render_pmc.sh)
    pmc = os.path.join(ROOT, "profiles", "r01_pmc_render_%dx%dx%d.json" % (n, width, height))
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("write_bytes_per_launch_from_WRITE_SIZE_KB")
    return {"envs": n, "cameras": n, "resolution": [width, height], "env_steps_per_s": n * steps / el,
            "ms_per_step": 1e3 * el / steps, "timed_loop": "hipGraph replay" if graphs is not None else "eager",
            "kernel": "k_render", "kernel_ms_avg": rk, "image_bytes_per_launch": wbytes,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": traffic},
            "env0_non_sky_fraction": lit}


def load_traffic(envs):
    """HBM bytes per k_rigid_step launch at this env count from the committed
    rocprofv3 PMC passes (profiles/r01_pmc_rigid_<envs>.json, written by
    profiles/collect_pmc.py), else None."""
    path = os.path.join(ROOT, "profiles", "r01_pmc_rigid_%d.json" % envs)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--envs", type=int, default=ENVS_PER_GPU, help="envs per GPU")
    ap.add_argument("--allgather", action="store_true", help="RCCL all-gather of the root state every step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-gimbal", action="store_true", help="skip the secondary S2 servo-arm measurement")
    ap.add_argument("--no-franka", action="store_true", help="skip the secondary S3 Franka cube-pick measurement")
    ap.add_argument("--no-cameras", action="store_true", help="skip the secondary S5 camera-render measurement")
    ap.add_argument("--camera-envs", type=int, default=1024)
    ap.add_argument("--eager", action="store_true",
                    help="time the Python loop itself instead of a hipGraph replay of the step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    gym = gymapi.acquire_gym()
    n = args.envs
    # rank k owns global envs [k n, (k+1) n), placed at their global grid cells
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=True, device=local, env_offset=rank * n,
                                grid_envs=world * n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gym.acquire_rigid_body_state_tensor(sim)
    gym.acquire_dof_state_tensor(sim)
    acts = scenes.servo_actions(n, 64, dev, seed=rank)
    gathered = args.allgather and world > 1

    def step(k):
        root[:, 3:10] = acts[k % acts.shape[0]]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, False)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_dof_state_tensor(sim)
        if gathered:
            sharding.all_gather_rows(root)      # RCCL over xGMI: (world * 2n, 13) observation

    gym.refresh_actor_root_state_tensor(sim)
    for k in range(args.warmup):
        step(k)
    # eager reference timing (the warmup's last half) and the kernel durations
    torch.cuda.synchronize(dev)
    t_e = time.perf_counter()
    neager = max(args.warmup // 2, 1)
    for k in range(neager):
        step(args.warmup + k)
    torch.cuda.synchronize(dev)
    eager_ms = 1e3 * (time.perf_counter() - t_e) / neager
    avg = ctypes.c_float()
    lo = ctypes.c_float()
    hi = ctypes.c_float()
    used = N.lib.mg_step_time_stats(sim.native, min(neager, 512), ctypes.byref(avg),
                                    ctypes.byref(lo), ctypes.byref(hi))
    # hipGraph replay: graphs of `chunk` consecutive captured steps (step j applies
    # acts[j]), sharing one memory pool; the replayed sequence is exactly the eager
    # loop's, and one graph launch is paid per `chunk` steps instead of per step
    graphs = None
    chunk = graph_chunk(args.steps, acts.shape[0])
    if not args.eager and not gathered:
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for j in range(3):
                    step(args.warmup + neager + j)
            torch.cuda.current_stream(dev).wait_stream(side)
            graphs = capture_chunks(step, acts.shape[0], chunk)
            # capture does not run the work: replay one chunk to settle, then
            # time from the next chunk-aligned slot
            base = -(-(args.warmup + neager + 3) // chunk) * chunk
            graphs[(base // chunk) % len(graphs)].replay()
            base += chunk
        except Exception as ex:          # capture unsupported here: time the eager loop
            print("*** bench: hipGraph capture failed (%s); timing the eager loop" % ex, file=sys.stderr)
            graphs = None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if graphs is not None:
        for i in range(args.steps // chunk):
            graphs[(base // chunk + i) % len(graphs)].replay()
    else:
        for k in range(args.steps):
            step(args.warmup + neager + k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if graphs is None:
        used = N.lib.mg_step_time_stats(sim.native, min(args.steps, 512), ctypes.byref(avg), ctypes.byref(lo),
                                        ctypes.byref(hi))

    kern_ms = avg.value if used > 0 else float("nan")

    ms_per_step = 1e3 * el / args.steps
    value = world * n * args.steps / el
    bytes_launch = SIM_BYTES_PER_ENV * n
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9 if used > 0 else None
    traffic = load_traffic(n)
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
                "parallelism": "env-sharded, one process per GPU%s" % (", RCCL all-gather of root state"
                                                                        if gathered else
                                                                        ", no collectives"),
                "timed_loop": ("hipGraph replay: %d captured tensor-API steps per graph (every step's full "
                               "kernel sequence, action slot by slot)" % chunk) if graphs is not None
                              else "eager Python loop",
                "eager_ms_per_step": eager_ms,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_rigid_step",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": bytes_launch,
                "kernel_ms_avg": kern_ms,
                "kernel_ms_min": lo.value if used > 0 else None,
                "kernel_launches_timed": int(used),
                "kernel_timing": "dispatch timestamps of k_rigid_step (hipExtLaunchKernelGGL start/stop events, "
                                 "the interval rocprofv3 reports) for every simulate() of the eager %s" % (
                    "segment after the warmup (graph replays carry no events)" if graphs is not None
                    else "timed loop"),
                "note": "working set of 4096 envs (~2.8 MB) sits in L2/MALL: the step is launch/latency "
                        "bound at this size (SURVEY.md §0.10)",
            },
        }
        if world == 1 and not args.no_gimbal:
            out["s2_servo_arm"] = gimbal_rate(ENVS_PER_GPU, min(args.steps, 300), 30, dev, not args.eager)
        if world == 1 and not args.no_franka:
            out["s3_franka"] = franka_rate(ENVS_PER_GPU, min(args.steps, 300), 30, dev, not args.eager)
        if world == 1 and not args.no_cameras:
            out["s5_cameras"] = camera_rate(args.camera_envs, min(args.steps, 100), 10, dev, not args.eager)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(out), flush=True)
    gym.destroy_sim(sim)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
