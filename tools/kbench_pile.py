"""Kernel microbenchmark of the S6 pile step:
examples/1080_balls_of_solitude.py's 30-ball pyramids at n envs; the average
k_pile_step time (dispatch timestamps) over frames [warm, warm + steps) — the
warm-up lets the pyramids fall and collapse (the layers land at frame ~60).
Library from MIGYM_LIB (default in-tree). Usage: kbench_pile.py [n ...]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from isaacgym import gymapi  # noqa: E402
from test_isaacgym_amd import _native as N, scenes  # noqa: E402


def run(n, steps=120, warm=90):
    gym = gymapi.acquire_gym()
    sim, _ = scenes.ball_pile_scene(gym, n)
    gym.prepare_sim(sim)
    for _ in range(warm):
        gym.simulate(sim)
    torch.cuda.synchronize()
    N.lib.mg_set_kernel_timing(sim.native, 1)
    for _ in range(steps):
        gym.simulate(sim)
    torch.cuda.synchronize()
    avg, lo = ctypes.c_float(), ctypes.c_float()
    used = N.lib.mg_step_time_stats(sim.native, steps, ctypes.byref(avg), ctypes.byref(lo), None)
    out = {"lib": os.path.basename(N.LIB_PATH), "envs": n, "frames": [warm, warm + steps],
           "kernel_us_avg": 1e3 * avg.value, "kernel_us_min": 1e3 * lo.value, "launches": used,
           "pile_envs": int(N.lib.mg_num_pile_envs(sim.native)),
           "env_steps_per_s_kernel": n / (avg.value * 1e-3)}
    gym.destroy_sim(sim)
    return out


if __name__ == "__main__":
    for a in sys.argv[1:] or ["4096"]:
        print(json.dumps(run(int(a))), flush=True)
