"""Where a k_pile_step wave's time goes (the S6 ball-pile frame): reads the
s_memtime stamps of a diagnostic build (MIGYM_LIB=tools/variants/
libmigym_pstamps.so, tools/build_variant.sh pstamps "-DMG_PILE_STAMPS": lane 0
of each env's wave stamps entry, inputs loaded, and in the (last) substep the
free flight, narrow phase, row constants, colouring, sort, solver sweeps and
pose / contact-force pass; then the stores) after `frames` frames of
examples/1080_balls_of_solitude.py's scene, with the wave's counts (candidate
pairs, active pairs, contact points, colours). Per-phase shader cycles, median
and 90th percentile over the waves."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from isaacgym import gymapi  # noqa: E402
from test_isaacgym_amd import _native as N, scenes  # noqa: E402

NAMES = ["inputs", "gap", "freeflight", "narrow", "constants", "colour", "links", "solver", "pose_force", "stores"]
IDX = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7), (7, 8), (8, 9), (9, 10)]


def run(n, frames):
    gym = gymapi.acquire_gym()
    sim, _ = scenes.ball_pile_scene(gym, n)
    gym.prepare_sim(sim)
    for _ in range(frames):
        gym.simulate(sim)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (n * 16))()
    fn = N.lib.mg_debug_pile_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    assert fn(buf, n) == 0
    st = np.frombuffer(buf, np.uint64).reshape(n, 16).astype(np.int64)
    out = {"envs": n, "frame": frames, "lib": os.path.basename(N.LIB_PATH)}
    for name, (a, b) in zip(NAMES, IDX):
        d = st[:, b] - st[:, a]
        out[name] = [int(np.median(d)), int(np.percentile(d, 90))]
    out["total"] = [int(np.median(st[:, 10] - st[:, 0])), int(np.percentile(st[:, 10] - st[:, 0], 90))]
    for name, k in (("pairs", 12), ("active_pairs", 13), ("points", 14), ("colours", 15)):
        out[name] = [int(np.median(st[:, k])), int(st[:, k].max())]
    gym.destroy_sim(sim)
    return out


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    for f in (30, 61, 90, 150):
        print(json.dumps(run(n, f)), flush=True)
