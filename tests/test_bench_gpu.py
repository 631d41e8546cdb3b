"""bench.py's multi-process path on the GPU box (one MI355X): `--gpus 2` without
torch.distributed.run starts its own two rank processes. Both ranks share GPU 0,
which RCCL does not allow, so the launcher picks gloo for the barrier / max /
all-gather; each rank steps its own 512-env shard on the device through the same
timed hipGraph loop the 8-GPU run uses."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_share_one_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "16",
                        "--warmup", "4", "--repeats", "2", "--envs", "512"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_envs"] == 1024
    assert d["value"] > 0 and len(d["config"]["ms_per_step_per_rank"]) == 2
    assert d["roofline"]["kernel_launches_timed"] >= 100
    g = d["allgather"]
    assert g["backend"] == "gloo" and g["bytes_gathered"] == 2 * 1024 * 13 * 4
    assert g["env_steps_per_s_with_gather"] > 0
