#!/bin/bash
# GPU-box: tests, bench, kernel trace, PMC (FETCH/WRITE in separate passes), env-count sweep.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-pytest,bench,rocprof,pmc,sweep}
[[ $STEPS == *pytest* ]]  && run pytest_gpu 900 python -m pytest tests -m gpu -q -rf
[[ $STEPS == *bench* ]]   && run bench 600 python bench.py --steps 600 --warmup 60
[[ $STEPS == *rocprof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 300 --warmup 30 --no-cpu-baseline
if [[ $STEPS == *pmc* ]]; then
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline
fi
if [[ $STEPS == *sweep* ]]; then
  for n in 16384 65536 262144 1048576; do
    run sweep_$n 900 python bench.py --envs $n --steps 100 --warmup 10 --no-cpu-baseline
  done
fi
exit 0
