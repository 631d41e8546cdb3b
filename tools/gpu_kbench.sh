#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in tools/variants/*.so; do
  echo "== $v"
  MIGYM_LIB=$PWD/$v timeout -k 10 300 python tools/kbench.py 4096 65536 262144 >> gpurun_out/kbench.log 2>&1
  rc=$?; echo "rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -3 gpurun_out/pytest_gpu.log
grep kernel_us gpurun_out/kbench.log
