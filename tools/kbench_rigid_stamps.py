"""Reads a phase-stamped local build of k_rigid_step1 (MIGYM_LIB=tools/variants/
libmigym_phase.so: an instrumentation build, not committed, whose kernel writes
s_memtime cycle counts instead of its outputs: velocity columns = [entry ->
substep 0 start, Iw / COM, free-flight velocity, candidates, contact constants,
TGS], net contact force = [pose update, whole wave]) on the 4096-env servo
scene; per-phase cycles averaged over UAV and vehicle lanes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import scenes  # noqa: E402

NAMES = ["load", "iw_com", "freeflight", "candidates", "constants", "tgs", "pose", "wave"]


def run(n, airborne):
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    acts = scenes.servo_actions(n, 32, "cuda:0", seed=0)
    gym.refresh_actor_root_state_tensor(sim)
    rows = []
    for k in range(60):
        gym.refresh_actor_root_state_tensor(sim)
        root[:, 3:10] = acts[k % 32]
        root[:, 7:13] = acts[k % 32][:, 4:7].repeat(1, 2)   # velocities rewritten (the kernel overwrote them)
        if airborne:
            root[:, 2] = 100.0
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        if k >= 20:
            rows.append(torch.cat([rb[:, 7:13], ncf[:, 0:2]], 1).clone())
    torch.cuda.synchronize()
    t = torch.stack(rows)
    out = {"airborne": airborne, "envs": n}
    for name, sel in (("uav", slice(0, None, 2)), ("car", slice(1, None, 2))):
        c = t[:, sel, :].mean((0, 1))
        out[name] = {k: round(float(v), 1) for k, v in zip(NAMES, c)}
    gym.destroy_sim(sim)
    return out


if __name__ == "__main__":
    for air in (False, True):
        print(json.dumps(run(4096, air)), flush=True)
