#!/bin/bash
# GPU-box script for the S6 pile step: its parity tests, the kernel
# microbenchmark at 36 .. 16384 envs, and a rocprofv3 kernel-trace summary at
# 4096 envs. Each step has its own time limit; the first failure ends the run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r06pile}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pile_gpu.py -m gpu -x -v --timeout 90 --timeout-method thread \
  > gpurun_out/pytest_gpu_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$tag.log
timeout -k 10 300 python tools/kbench_pile.py 36 1024 4096 16384 > gpurun_out/kpile_$tag.jsonl 2>&1 \
  || { tail -20 gpurun_out/kpile_$tag.jsonl; exit 1; }
cat gpurun_out/kpile_$tag.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o kpile --output-format csv -- python tools/kbench_pile.py 4096 \
  > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kpile_${tag}_kernel_stats.csv
cut -c1-160 gpurun_out/kpile_${tag}_kernel_stats.csv | head -8
if [[ -f tools/variants/libmigym_pstamps.so ]]; then
  MIGYM_LIB=tools/variants/libmigym_pstamps.so timeout -k 10 300 python tools/kbench_pile_stamps.py 4096 \
    > gpurun_out/kpile_stamps_$tag.jsonl 2>&1 || { tail -20 gpurun_out/kpile_stamps_$tag.jsonl; exit 1; }
  cat gpurun_out/kpile_stamps_$tag.jsonl
fi
