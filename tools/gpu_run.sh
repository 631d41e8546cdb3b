#!/bin/bash
# GPU-box check: smoke, parity tests, bench, rocprof kernel trace.
# Each GPU step has its own time limit; a crash/timeout (exit >= 124 or signal)
# ends the script, a plain test failure (exit 1) does not.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,pytest,bench,rocprof}
[[ $STEPS == *smoke* ]]   && run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *pytest* ]]  && run pytest_gpu 900 python -m pytest tests -m gpu -q -rf
[[ $STEPS == *bench* ]]   && run bench 600 python bench.py --steps 600 --warmup 60
[[ $STEPS == *rocprof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 300 --warmup 30 --no-cpu-baseline
exit 0
