#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/kbench.py 4096 262144 > gpurun_out/kbench.log 2>&1 || exit $?
cat gpurun_out/kbench.log | grep kernel
timeout -k 10 300 python bench.py --steps 600 --warmup 60 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1 || exit $?
cut -d, -f1-4 gpurun_out/prof/run_kernel_stats.csv | cut -c1-150
