#!/bin/bash
# One GPU iteration: GPU tests, S1 kernel A/B (in-tree vs tools/variants/*.so),
# the S1/S2 bench line and a rocprofv3 kernel summary of it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
shopt -s nullglob
for v in "" tools/variants/*.so; do
  if [ -n "$v" ]; then export MIGYM_LIB=$PWD/$v; else unset MIGYM_LIB; fi
  timeout -k 10 300 python tools/kbench.py ${KB_SIZES:-4096 262144} >> gpurun_out/kbench.log 2>&1 || exit $?
done
unset MIGYM_LIB
grep kernel_us gpurun_out/kbench.log
timeout -k 10 300 python bench.py --no-franka --no-cpu-baseline > gpurun_out/bench_s1.log 2>&1 || { tail -20 gpurun_out/bench_s1.log; exit 1; }
tail -1 gpurun_out/bench_s1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s1 -o run --output-format csv -- python bench.py --no-franka --no-cpu-baseline > gpurun_out/prof_s1.log 2>&1 || exit $?
f=$(find gpurun_out/prof_s1 -name '*kernel_stats.csv' | head -1); cut -c1-160 "$f" | head -12
