#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/kbench.py 4096 65536 262144 1048576 > gpurun_out/kbench.log 2>&1 || exit $?
grep kernel gpurun_out/kbench.log
n=262144
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_$n -o run --output-format csv -- python bench.py --envs $n --steps 50 --warmup 5 --no-cpu-baseline --no-gimbal > gpurun_out/pmc_f_$n.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_$n -o run --output-format csv -- python bench.py --envs $n --steps 50 --warmup 5 --no-cpu-baseline --no-gimbal > gpurun_out/pmc_w_$n.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 600 --warmup 60 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
