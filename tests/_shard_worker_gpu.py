"""One rank of tests/test_config4_gpu.py (BASELINE config 4 on one MI355X):
started by test_isaacgym_amd.launch.spawn_ranks, the launcher `bench.py --gpus N`
uses. All ranks share GPU 0, so the process group is gloo (RCCL refuses two
ranks on one device); the physics is the real device step.

Rank k builds envs [k n, (k+1) n) of a `world * n`-env servo scene on cuda:0
(env grid laid out for the whole job, sharding.py), applies the global action
bank's rows for its envs and steps `frames` frames through the gymapi tensor
API (test10_servo_vecenv.py:376-456), then the ranks all-gather their root and
rigid-body state tensors and rank 0 saves them to <out>_root.npy / <out>_rb.npy.

With backend "nccl" (one rank only: RCCL refuses two ranks on one device) the
same job runs over RCCL, so sharding.all_gather_rows takes its device branch
(all_gather_into_tensor), the one the 8-GPU node runs.

usage: _shard_worker_gpu.py <envs per rank> <frames> <out prefix> [gloo|nccl]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    n, frames, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    backend = sys.argv[4] if len(sys.argv) > 4 else "gloo"
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    assert dist.get_backend() == backend
    rank, world = dist.get_rank(), dist.get_world_size()
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes, sharding
    gym = gymapi.acquire_gym()
    start, end = sharding.env_range(rank, world, world * n)
    sim, _ = scenes.servo_scene(gym, end - start, use_gpu_pipeline=True, device=0, env_offset=start,
                                grid_envs=world * n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    acts = scenes.servo_actions(world * n, frames, "cpu", seed=11)[:, 2 * start:2 * end].to("cuda:0")
    gym.refresh_actor_root_state_tensor(sim)
    for f in range(frames):
        root[:, 3:10] = acts[f]
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
    torch.cuda.synchronize()
    g_root = sharding.all_gather_rows(root)
    g_rb = sharding.all_gather_rows(rb)
    if rank == 0:
        np.save(out + "_root.npy", g_root.cpu().numpy())
        np.save(out + "_rb.npy", g_rb.cpu().numpy())
    dist.barrier()
    gym.destroy_sim(sim)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
