"""Where test10's CPU-pipeline step spends its time (host tensors, 1024 envs):
per-call wall time of the tensor-API loop, averaged over `steps` steps.
usage: cpu_pipeline_breakdown.py [envs] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=False)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    gym.acquire_rigid_body_state_tensor(sim)
    gym.acquire_dof_state_tensor(sim)
    acts = scenes.servo_actions(n, 16, "cpu", seed=2)
    names = ["write_actions", "set_root", "simulate", "fetch_results", "refresh_root", "refresh_rb", "refresh_dof"]
    acc = dict.fromkeys(names, 0.0)
    calls = [lambda k: root[:, 3:10].copy_(acts[k % 16]),
             lambda k: gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root)),
             lambda k: gym.simulate(sim),
             lambda k: gym.fetch_results(sim, True),
             lambda k: gym.refresh_actor_root_state_tensor(sim),
             lambda k: gym.refresh_rigid_body_state_tensor(sim),
             lambda k: gym.refresh_dof_state_tensor(sim)]
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(30):
        for c in calls:
            c(k)
    t_all = time.perf_counter()
    for k in range(steps):
        for name, c in zip(names, calls):
            t = time.perf_counter()
            c(k)
            acc[name] += time.perf_counter() - t
    el = time.perf_counter() - t_all
    out = {"envs": n, "steps": steps, "us_per_step": 1e6 * el / steps,
           "us_per_call": {k: round(1e6 * v / steps, 2) for k, v in acc.items()},
           "env_steps_per_s": n * steps / el}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
