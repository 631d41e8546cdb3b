"""Reads a phase-stamped build of k_rigid_step1 (MIGYM_LIB=tools/variants/
libmigym_phase.so, a local instrumentation build whose kernel writes
[loads, substep 1, whole wave] s_memtime cycle counts into the net contact
force tensor) on the 4096-env servo scene: per-phase cycles of the wave,
averaged over bodies, for the default and the airborne settings."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import scenes  # noqa: E402


def run(n, airborne):
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    acts = scenes.servo_actions(n, 32, "cuda:0", seed=0)
    gym.refresh_actor_root_state_tensor(sim)
    rows = []
    for k in range(60):
        root[:, 3:10] = acts[k % 32]
        if airborne:
            root[:, 2] = 100.0
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        if k >= 20:
            rows.append(ncf.clone())
    torch.cuda.synchronize()
    t = torch.stack(rows)                      # (steps, bodies, 3)
    out = {"airborne": airborne, "envs": n}
    for name, sel in (("uav", slice(0, None, 2)), ("car", slice(1, None, 2))):
        c = t[:, sel, :]
        out[name] = {"loads_cyc": float(c[..., 0].mean()), "substep1_cyc": float(c[..., 1].mean()),
                     "wave_cyc": float(c[..., 2].mean()), "wave_cyc_max": float(c[..., 2].max())}
    gym.destroy_sim(sim)
    return out


if __name__ == "__main__":
    for air in (False, True):
        print(json.dumps(run(4096, air)), flush=True)
