"""Wall time of the S1 scene at N envs, by stage: the Python scene build
(create_env / create_actor), build_model (packing), prepare_sim (the native
upload and classification), the first simulate. usage: time_scene_build.py N"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    import torch
    from isaacgym import gymapi
    from test_isaacgym_amd import scenes
    gym = gymapi.acquire_gym()
    t = [time.perf_counter()]
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=True)
    t.append(time.perf_counter())
    sim.build_model()
    t.append(time.perf_counter())
    gym.prepare_sim(sim)
    torch.cuda.synchronize()
    t.append(time.perf_counter())
    gym.simulate(sim)
    gym.fetch_results(sim, True)
    t.append(time.perf_counter())
    print(json.dumps({"envs": n, "scene_s": t[1] - t[0], "build_model_s": t[2] - t[1], "prepare_sim_s": t[3] - t[2],
                      "first_simulate_s": t[4] - t[3]}), flush=True)


if __name__ == "__main__":
    main()
