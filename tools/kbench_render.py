"""k_render micro-benchmark (S5 scene: servo envs, one camera per env on the
UAV): prints one JSON line per resolution with the kernel's average duration
(dispatch timestamps) and its image-write bandwidth. Short enough to run under
rocprofv3 --pmc.  Usage: python tools/kbench_render.py [envs] [WxH ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import _native as N  # noqa: E402
from test_isaacgym_amd import scenes  # noqa: E402


def run(n, w, h, warm=10, reps=20):
    """The bench's own S5 sequence (bench.py camera_rate): actions
    servo_actions(n, 16, seed=5), `warm` steps, then `reps` timed renders."""
    gym = gymapi.acquire_gym()
    sim, envs = scenes.servo_scene(gym, n)
    imgs = scenes.attach_servo_cameras(gym, sim, envs, w, h, 30.0)
    gym.prepare_sim(sim)
    N.lib.mg_set_kernel_timing(sim.native, 1)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    acts = scenes.servo_actions(n, 16, "cuda:0", seed=5)
    gym.refresh_actor_root_state_tensor(sim)
    ms = []
    for k in range(warm + reps):
        root[:, 3:10] = acts[k % 16]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_actor_root_state_tensor(sim)
        gym.render_all_camera_sensors(sim)
        if k >= warm:
            ms.append(N.lib.mg_last_render_ms(sim.native))
    torch.cuda.synchronize()
    sky = float((imgs[0][0][..., :3].amax(-1) == 0).float().mean())
    lit = float(np.mean([float((imgs[i][0][..., :3].amax(-1) > 0).float().mean())
                         for i in range(0, n, max(1, n // 16))]))
    gym.destroy_sim(sim)
    avg = float(np.mean(ms))
    return {"envs": n, "w": w, "h": h, "kernel_ms": avg, "write_GBps": n * w * h * 4 / (avg * 1e-3) / 1e9,
            "env0_sky_frac": sky, "sampled_cameras_non_sky_fraction": lit}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    sizes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[2:]] or [(1600, 900)]
    for w, h in sizes:
        print(json.dumps(run(n, w, h)), flush=True)
