"""One process per GPU, started by the parent before it touches the GPU
(envs shard with no interaction, rank k owning its own sim on its
own device). `bench.py --gpus N` uses this when it is not already running under
`torch.distributed.run`; the children see the same environment torchrun would
give them (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR /
MASTER_PORT) and run the same script with the same arguments.

The parent never initialises HIP (it imports nothing GPU-related), so starting
the children is an ordinary fork + exec of a fresh interpreter.
"""
import os
import signal
import socket
import subprocess
import sys
import time


def free_port(host="127.0.0.1"):
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank, world, port, base=None, host="127.0.0.1"):
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                "MASTER_ADDR": host, "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(argv, world, timeout=None, port=None, stdout=None):
    """Run `python argv...` as `world` ranks of one job and wait for all of them.
    If a rank fails, the others are terminated (by PID) so the job does not hang
    in a collective. Returns the worst exit code (0 when every rank succeeded)."""
    port = port or free_port()
    procs = []
    try:
        for r in range(world):
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=rank_env(r, world, port),
                                          stdout=stdout))
        t0 = time.monotonic()
        while True:
            codes = [p.poll() for p in procs]
            if any(c not in (None, 0) for c in codes) or all(c is not None for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    codes = [p.returncode for p in procs]
    bad = [c for c in codes if c != 0]
    return (max(bad, key=abs) if bad else 0), codes
