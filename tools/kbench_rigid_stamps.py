"""Where a k_rigid_step1 wave's time goes at the S1 headline size: reads the
s_memtime stamps of a diagnostic build (MIGYM_LIB=tools/variants/
libmigym_rstamps.so, tools/build_variant.sh rstamps "-DMG_RIGID1_STAMPS":
lane 0 stamps its wave at entry, inputs in registers, patch record read, and
per substep after the free-flight velocity, the candidates, the patch update,
the row constants, the solver sweeps and the pose update; then stores issued
and stores complete) after the 4096-env servo loop of tools/kbench.py with
the refresh fused (KB_FUSION 31). Per-phase shader cycles, median over the
UAV waves (first half of the launch: the airborne template is ordered first)
and over the vehicle waves."""
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

NAMES = ["inputs", "patch_read"] + ["%s_%d" % (p, s) for s in (0, 1)
                                    for p in ("freeflight", "candidates", "patch", "constants", "solver", "pose")] \
    + ["stores_issue", "stores_drain"]
IDX = [(0, 1), (1, 2)] + [(2 + 6 * s + k, 3 + 6 * s + k) for s in (0, 1) for k in range(6)] + [(14, 15), (15, 16)]


def run(n, steps=60):
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    gym.set_step_fusion(sim, 31)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    acts = scenes.servo_actions(n, 32, "cuda:0", seed=0)
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(steps):
        root[:, 3:10] = acts[k % 32]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_actor_root_state_tensor(sim)
    torch.cuda.synchronize()
    nw = (2 * n + 63) // 64
    buf = (ctypes.c_ulonglong * (nw * 18))()
    fn = N.lib.mg_debug_rigid_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    assert fn(buf, nw) == 0
    st = np.frombuffer(buf, np.uint64).reshape(nw, 18).astype(np.int64)
    out = {"envs": n, "waves": nw}
    for name, rows in (("uav_waves", st[: nw // 2]), ("vehicle_waves", st[nw // 2:])):
        out[name] = {nm: int(np.median(rows[:, b] - rows[:, a])) for nm, (a, b) in zip(NAMES, IDX)}
        out[name]["wave"] = int(np.median(rows[:, 16] - rows[:, 0]))
    gym.destroy_sim(sim)
    return out


if __name__ == "__main__":
    for n in [int(x) for x in (sys.argv[1:] or ["4096"])]:
        print(json.dumps(run(n)), flush=True)
