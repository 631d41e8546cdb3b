#!/bin/bash
# Round 6: the Franka pick-loop GPU parity at the north-star size — 4096 envs,
# 600 frames (10 s of the script's loop), bit for bit the oracle every frame.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat_franka_long.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
MIGYM_PARITY_ENVS=4096 MIGYM_PARITY_FRAMES=600 timeout -k 10 800 python -u -m pytest tests/test_franka_gpu.py \
  -k "pick_parity_bitexact" -v --timeout 780 --timeout-method thread > gpurun_out/franka_long_parity.log 2>&1
rc=$?
tail -4 gpurun_out/franka_long_parity.log | cut -c1-200
exit $rc
