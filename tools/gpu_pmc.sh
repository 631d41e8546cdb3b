#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 4096 262144; do
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_$n -o run --output-format csv -- python bench.py --envs $n --steps 50 --warmup 5 --no-cpu-baseline --no-gimbal > gpurun_out/pmc_f_$n.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_$n -o run --output-format csv -- python bench.py --envs $n --steps 50 --warmup 5 --no-cpu-baseline --no-gimbal > gpurun_out/pmc_w_$n.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$n -o run --output-format csv -- python bench.py --envs $n --steps 300 --warmup 30 --no-cpu-baseline --no-gimbal > gpurun_out/kt_$n.log 2>&1 || exit $?
done
echo done
