"""Where k_rigid_step's time goes at the headline size, without instrumenting
the kernel: the same 4096-env servo step timed (dispatch timestamps, 200
launches) under solver settings that remove one part of the work at a time —
  default        substeps 2, TGS 6/1 (the bench)
  iters_1_0      substeps 2, TGS 1/0    -> cost of 5 position + 1 velocity iterations
  sub_1          substeps 1, TGS 6/1    -> cost of one substep
  airborne       the default with every body 100 m up (no contacts)
Prints one JSON line per setting.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import _native as N, scenes  # noqa: E402


def run(n, label, substeps=2, npos=6, nvel=1, airborne=False, steps=200, warm=20):
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n)
    p = sim.params
    p.substeps = substeps
    p.physx.num_position_iterations = npos
    p.physx.num_velocity_iterations = nvel
    gym.prepare_sim(sim)
    gym.set_sim_params(sim, p)
    N.lib.mg_set_kernel_timing(sim.native, 1)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    acts = scenes.servo_actions(n, 32, "cuda:0", seed=0)
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(warm + steps):
        root[:, 3:10] = acts[k % 32]
        if airborne:
            root[:, 2] = 100.0
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_actor_root_state_tensor(sim)
    torch.cuda.synchronize()
    avg, lo = ctypes.c_float(), ctypes.c_float()
    used = N.lib.mg_step_time_stats(sim.native, steps, ctypes.byref(avg), ctypes.byref(lo), None)
    gym.destroy_sim(sim)
    return {"setting": label, "envs": n, "kernel_us_avg": 1e3 * avg.value, "kernel_us_min": 1e3 * lo.value,
            "launches": used}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    for label, kw in (("default", {}), ("iters_1_0", {"npos": 1, "nvel": 0}), ("sub_1", {"substeps": 1}),
                      ("airborne", {"airborne": True})):
        print(json.dumps(run(n, label, **kw)), flush=True)
