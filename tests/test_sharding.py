"""Multi-GPU path on the host (gloo, world size 2): each rank builds its shard
of the servo scene; the all-gathered root-state tensors equal the single-sim
layout bit for bit. The device step needs no collective."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_isaacgym_amd import sharding


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes
    gym = gymapi.acquire_gym()
    start, end = sharding.env_range(rank, world, n)
    sim, _ = scenes.servo_scene(gym, end - start, use_gpu_pipeline=False, env_offset=start, grid_envs=n)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    g_root = sharding.all_gather_rows(root)
    g_rb = sharding.all_gather_rows(rb)
    if rank == 0:
        q.put((g_root.numpy().copy(), g_rb.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_layout_matches_single_sim():
    n, world = 32, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    g_root, g_rb = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from isaacgym import gymapi, gymtorch
    from test_isaacgym_amd import scenes
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, n, use_gpu_pipeline=False)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim)).numpy()
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim)).numpy()
    assert np.array_equal(g_root, root)
    assert np.array_equal(g_rb, rb)


def test_env_range_partition():
    for n in (1, 7, 32, 4096, 32768):
        for w in (1, 2, 3, 8):
            rs = [sharding.env_range(r, w, n) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(e - s for s, e in rs) - min(e - s for s, e in rs) <= 1
