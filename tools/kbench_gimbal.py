"""Kernel microbenchmark of the S2 gimbal step: 4096 gimbals
under random PD position targets; average simulate() kernel time (HIP events).
Library from MIGYM_LIB (default in-tree)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import _native as N, scenes  # noqa: E402


def run(n, steps=200, warm=20, fused=False):
    """fused: STEP_FUSION_ALL and the S2 loop's refreshes (the kernel reads the
    targets from the set tensor and writes the DOF / rigid-body rows itself)."""
    gym = gymapi.acquire_gym()
    sim, _ = scenes.gimbal_scene(gym, n)
    gym.prepare_sim(sim)
    if fused:
        gym.set_step_fusion(sim, gymapi.STEP_FUSION_ALL)
    gym.acquire_dof_state_tensor(sim)
    gym.acquire_rigid_body_state_tensor(sim)
    N.lib.mg_set_kernel_timing(sim.native, 1)
    tg = scenes.gimbal_targets(n, 64, "cuda:0", seed=0)
    for k in range(warm + steps):
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k % 64]))
        gym.simulate(sim)
        if fused:
            gym.refresh_dof_state_tensor(sim)
            gym.refresh_rigid_body_state_tensor(sim)
    torch.cuda.synchronize()
    avg, lo = ctypes.c_float(), ctypes.c_float()
    used = N.lib.mg_step_time_stats(sim.native, steps, ctypes.byref(avg), ctypes.byref(lo), None)
    out = {"lib": os.path.basename(N.LIB_PATH), "envs": n, "fused": fused, "kernel_us_avg": 1e3 * avg.value,
           "kernel_us_min": 1e3 * lo.value, "coupled_envs": int(N.lib.mg_num_coupled_envs(sim.native))}
    gym.destroy_sim(sim)
    return out


if __name__ == "__main__":
    fused = os.environ.get("MIGYM_KB_FUSED", "0") == "1"
    for n in [int(x) for x in (sys.argv[1:] or ["4096"])]:
        print(json.dumps(run(n, fused=fused)), flush=True)
