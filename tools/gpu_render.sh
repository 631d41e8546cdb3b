#!/bin/bash
# Camera-render iteration: render GPU tests, then the S1 + S5 bench legs and a
# rocprofv3 kernel summary of the same command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-render}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_render.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$tag.log 2>&1 || { tail -60 gpurun_out/pytest_$tag.log; exit 1; }
tail -6 gpurun_out/pytest_$tag.log
B="python bench.py --no-franka --no-gimbal --no-cpu-baseline --steps 200 --warmup 20"
timeout -k 10 300 $B > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- $B \
  > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1); cut -c1-150 "$f" | head -12
