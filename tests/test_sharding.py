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


def test_launcher_stepped_shards_match_single_sim(tmp_path):
    """bench.py's launcher (launch.spawn_ranks) starts 2 gloo ranks; each steps its
    shard 6 frames under the global action bank; the all-gathered body state
    equals one 2n-env sim stepped the same way, bit for bit."""
    import sys
    import oracle
    from isaacgym import gymapi
    from test_isaacgym_amd import launch, scenes
    n, world, frames = 24, 2, 6
    out = str(tmp_path / "gathered.npy")
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_shard_worker.py")
    rc, codes = launch.spawn_ranks([worker, str(n), str(frames), out], world, timeout=240)
    assert rc == 0, codes
    got = np.load(out)
    gym = gymapi.acquire_gym()
    sim, _ = scenes.servo_scene(gym, world * n, use_gpu_pipeline=False)
    sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = sim.model_arrays["body_state0"].copy()
    roots = sim.model_arrays["actor_root_body"]
    acts = scenes.servo_actions(world * n, frames, "cpu", seed=3).numpy()
    for f in range(frames):
        st[roots, 3:10] = acts[f]
        oracle.step(p, m, st, np.zeros((0, 2), np.float32))
    assert got.shape == st.shape
    assert not np.array_equal(st, sim.model_arrays["body_state0"])      # the shards did step
    assert np.array_equal(got, st)


def test_bench_dry_run_two_ranks():
    """`python bench.py --gpus 2 --dry-run` (no WORLD_SIZE): the bench starts its
    own two ranks, which report n_gpus 2 and the single-sim layout."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--envs", "8"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["gathered_rows"] == 32 and d["layout_matches_single_sim"]
