#!/bin/bash
# Articulation kernels, same box: GPU parity of the gimbal / Franka / ant paths,
# then the S2 (4096 gimbals) and S3 (Franka) micro-benchmarks for the in-tree
# library and tools/variants/libmigym_prev.so, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_franka_gpu.py tests/test_ant.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/pt_ab_artic.log 2>&1 || { tail -30 gpurun_out/pt_ab_artic.log; exit 1; }
tail -2 gpurun_out/pt_ab_artic.log
for r in 1 2; do
  timeout -k 10 120 python tools/kbench_gimbal.py 4096 || exit 1
  MIGYM_LIB=tools/variants/libmigym_prev.so timeout -k 10 120 python tools/kbench_gimbal.py 4096 || exit 1
done
timeout -k 10 300 python tools/kbench_franka.py && MIGYM_LIB=tools/variants/libmigym_prev.so timeout -k 10 300 python tools/kbench_franka.py
