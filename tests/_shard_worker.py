"""One rank of tests/test_sharding.py's stepped-shard check, started by
test_isaacgym_amd.launch.spawn_ranks (the launcher bench.py --gpus N uses).

Rank k builds envs [k n, (k+1) n) of a `world * n`-env servo scene, applies the
global action bank's rows for its envs and steps its shard `frames` times with
the C restatement (the host stand-in for the device step: this container has no
GPU), then the ranks all-gather their body states over gloo and rank 0 saves
the gathered (world * 2n, 13) state to argv[3].

usage: _shard_worker.py <envs per rank> <frames> <out.npy>
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
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import oracle
    from isaacgym import gymapi
    from test_isaacgym_amd import scenes, sharding
    gym = gymapi.acquire_gym()
    start, end = sharding.env_range(rank, world, world * n)
    sim, _ = scenes.servo_scene(gym, end - start, use_gpu_pipeline=False, env_offset=start, grid_envs=world * n)
    sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    roots = sim.model_arrays["actor_root_body"]
    acts = scenes.servo_actions(world * n, frames, "cpu", seed=3).numpy()
    dof = np.zeros((0, 2), np.float32)
    for f in range(frames):
        st[roots, 3:10] = acts[f, 2 * start:2 * end]
        oracle.step(p, m, st, dof)
    rb = torch.from_numpy(st)          # rigid-body tensor order (env-major, actor, body)
    g = sharding.all_gather_rows(rb)
    if rank == 0:
        np.save(out, g.numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
