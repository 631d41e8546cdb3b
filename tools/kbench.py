"""Kernel microbenchmark: average k_rigid_step duration (HIP events around each
launch) for the servo scene at several env counts, for the library selected
by MIGYM_LIB (default: the in-tree build). KB_FUSION sets gym.set_step_fusion's
flags (default 15; 31 adds the refresh fused into the step, as bench.py). Prints one JSON line per size."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import _native as N, scenes  # noqa: E402


def run(n, steps=200, warm=20):
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    N.lib.mg_set_kernel_timing(sim.native, 1)
    gym.set_step_fusion(sim, int(os.environ.get("KB_FUSION", "15")))   # bench.py's setting
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))   # bound: KB_FUSION=31 fuses the refresh
    acts = scenes.servo_actions(n, 32, "cuda:0", seed=0)
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(warm + steps):
        root[:, 3:10] = acts[k % 32]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_actor_root_state_tensor(sim)
    torch.cuda.synchronize()
    avg, lo = ctypes.c_float(), ctypes.c_float()
    used = N.lib.mg_step_time_stats(sim.native, steps, ctypes.byref(avg), ctypes.byref(lo), None)
    gym.destroy_sim(sim)
    return {"lib": os.path.basename(N.LIB_PATH), "envs": n, "kernel_us_avg": 1e3 * avg.value,
            "kernel_us_min": 1e3 * lo.value, "launches": used, "fusion": os.environ.get("KB_FUSION", "default")}


if __name__ == "__main__":
    sizes = [int(x) for x in (sys.argv[1:] or ["4096", "65536", "262144"])]
    for n in sizes:
        print(json.dumps(run(n)), flush=True)
