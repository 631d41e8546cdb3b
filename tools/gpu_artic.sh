#!/bin/bash
# Articulation paths: GPU parity (gimbal, VEL drive, Franka, ant) and the S2 / S3
# kernel micro-benchmarks.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_franka_gpu.py tests/test_ant.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_artic.log 2>&1; rc=$?; tail -5 gpurun_out/pt_artic.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/kbench_gimbal.py 4096 && timeout -k 10 300 python tools/kbench_franka.py
