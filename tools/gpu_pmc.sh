#!/bin/bash
# rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, no trace
# domains combined) + a kernel-trace pass of the S1 bench at the given env counts.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in ${PMC_SIZES:-4096}; do
  B="python bench.py --envs $n --steps 48 --warmup 5 --repeats 1 --pmc-calibrate --no-cpu-baseline --no-gimbal --no-franka --no-cameras --no-large-n"
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_$n -o run --output-format csv -- $B > gpurun_out/pmc_f_$n.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_$n -o run --output-format csv -- $B > gpurun_out/pmc_w_$n.log 2>&1 || exit $?
done
echo done
