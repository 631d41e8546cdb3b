"""Where a quad-kernel wave's time goes at the S2 size: reads the s_memtime
stamps of a diagnostic build (MIGYM_LIB=tools/variants/libmigym_stamps.so,
tools/build_variant.sh stamps "-DMG_CHAIN_STAMPS": k_artic_chain_q's lane 0
stamps its wave at kernel entry, inputs in registers, after each substep,
output rows formed, stores issued, stores complete) after the 4096-gimbal
fused step loop of tools/kbench_gimbal.py. Prints per-phase cycles (median
and max over the launch's waves) and the entry skew across waves."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import _native as N, scenes  # noqa: E402

PHASES = ["inputs", "substep0", "substep1", "output_fk", "stores_issue", "stores_drain"]


def run(n, steps=100):
    gym = gymapi.acquire_gym()
    sim, _ = scenes.gimbal_scene(gym, n)
    gym.prepare_sim(sim)
    gym.set_step_fusion(sim, gymapi.STEP_FUSION_ALL)
    gym.acquire_dof_state_tensor(sim)
    gym.acquire_rigid_body_state_tensor(sim)
    tg = scenes.gimbal_targets(n, 64, "cuda:0", seed=0)
    for k in range(steps):
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(tg[k % 64]))
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
    torch.cuda.synchronize()
    nw = (n * 4 + 63) // 64
    buf = (ctypes.c_ulonglong * (nw * 8))()
    fn = N.lib.mg_debug_chain_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    assert fn(buf, nw) == 0
    st = np.frombuffer(buf, np.uint64).reshape(nw, 8).astype(np.int64)
    d = np.diff(st[:, :7], axis=1)
    out = {"envs": n, "waves": nw,
           "phase_cycles_median": {p: int(np.median(d[:, i])) for i, p in enumerate(PHASES)},
           "phase_cycles_max": {p: int(d[:, i].max()) for i, p in enumerate(PHASES)},
           "wave_cycles_median": int(np.median(st[:, 6] - st[:, 0])),
           "entry_skew_cycles": int(st[:, 0].max() - st[:, 0].min()),
           "launch_span_cycles": int(st[:, 6].max() - st[:, 0].min())}
    gym.destroy_sim(sim)
    return out


if __name__ == "__main__":
    for n in [int(x) for x in (sys.argv[1:] or ["4096"])]:
        print(json.dumps(run(n)), flush=True)
