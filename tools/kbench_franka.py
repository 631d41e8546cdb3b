"""Kernel microbenchmark of the coupled per-env step (k_env_step): the S3
Franka cube-pick loop (OSC controller) at n envs; warm frames bring the arms to
the cubes (grasp contacts), then the average simulate() kernel time over the
timed frames (HIP events), then the loop continues to KB_FRAMES (default 600)
frames for the fraction of cubes lifted above 0.55 m and the cubes at rest
inside the table. Library from MIGYM_LIB (default in-tree)."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import _native as N, franka_control, scenes  # noqa: E402


def run(n, warm=150, steps=100):
    gym = gymapi.acquire_gym()
    sim, info = scenes.franka_scene(gym, n, asset_file=os.environ.get("MIGYM_FRANKA_ASSET", "franka/franka_proxy.urdf"))
    gym.prepare_sim(sim)
    N.lib.mg_set_kernel_timing(sim.native, 1)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    jac = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, "franka"))
    mm = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, "franka"))
    ctl = franka_control.CubePick(n, info["init_pos"], info["init_rot"], info["default_dof_pos"], "cuda:0")
    h = info["hand_index"]
    bi = torch.tensor(info["box_idxs"], device="cuda:0")
    hi = torch.tensor(info["hand_idxs"], device="cuda:0")
    total = max(warm + steps, int(os.environ.get("KB_FRAMES", "600")))
    maxz = torch.zeros(n, device="cuda:0")
    avg, lo = ctypes.c_float(), ctypes.c_float()
    used = 0
    for k in range(total):
        gym.simulate(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_jacobian_tensors(sim)
        gym.refresh_mass_matrix_tensors(sim)
        pa, ea = ctl.step(rb, dof[:, 0].view(n, 9, 1), dof[:, 1].view(n, 9, 1), jac[:, h - 1, :, :7],
                          mm[:, :7, :7], bi, hi)
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(pa))
        gym.set_dof_actuation_force_tensor(sim, gymtorch.unwrap_tensor(ea))
        maxz = torch.maximum(maxz, rb[bi, 2])
        if k == warm + steps - 1:      # the timed window: frames [warm, warm + steps)
            used = N.lib.mg_step_time_stats(sim.native, steps, ctypes.byref(avg), ctypes.byref(lo), None)
            phases = None
            if hasattr(N.lib, "mg_debug_env_phase"):
                buf = (ctypes.c_ulonglong * 24)()
                N.lib.mg_debug_env_phase(buf)
                waves = (n + 3) // 4
                names = ["unconstrained", "narrowphase_rest", "crba_minv", "rows", "tgs", "integrate", "setup",
                         "outputs", "np_screen", "np_collide", "pairs_tested", "pairs_with_hull",
                         "coop_vertices", "coop_edges", "coop_merge", "coop_edge_passes",
                         "coop_pairs_no_contact", "np_kernel_setup_fk", "np_setup_and_one_lane_tests", "np_coop_loop",
                         "np_placement", "np_kernel_patches_out"]
                phases = {nm: buf[i] / waves / steps for i, nm in enumerate(names)}   # cycles per wave per frame
        if k == warm - 1 and hasattr(N.lib, "mg_debug_env_phase_reset"):
            torch.cuda.synchronize()
            N.lib.mg_debug_env_phase_reset()
    torch.cuda.synchronize()
    if os.environ.get("KB_DUMP"):
        # the grasp-phase state and targets, for replaying one step on the host restatement
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_dof_state_tensor(sim)
        np.savez(os.environ["KB_DUMP"], rb=rb.cpu().numpy(), dof=dof.cpu().numpy(), pa=pa.cpu().numpy(),
                 ea=ea.cpu().numpy())
    lifted = float((maxz > 0.55).float().mean())
    bz = rb[bi, 2]
    rel = rb[bi, 0:2] - rb[bi - 1, 0:2]       # from the table centre (tests/test_franka_gpu.py)
    over = (rel[:, 0].abs() < 0.3 - 0.0225) & (rel[:, 1].abs() < 0.5 - 0.0225)
    sunk = int(((bz > 0.3) & (bz < 0.4225 - 0.005) & (rb[bi, 7:10].norm(dim=1) < 0.05) & over).sum())
    gym.destroy_sim(sim)
    return {"lib": os.path.basename(N.LIB_PATH), "envs": n, "kernel_us_avg": 1e3 * avg.value,
            "kernel_us_min": 1e3 * lo.value, "launches": used, "window": [warm, warm + steps],
            "frames": total, "cubes_lifted_frac": lifted, "cubes_sunk": sunk, "phase_cycles_per_wave": phases}


if __name__ == "__main__":
    sizes = [int(x) for x in (sys.argv[1:] or ["4096"])]
    for n in sizes:
        print(json.dumps(run(n)), flush=True)
