#!/bin/bash
# Kernel A/B: tools/kbench.py for the in-tree build and every tools/variants/*.so,
# then the GPU parity tests on the in-tree build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
shopt -s nullglob
for v in "" tools/variants/*.so; do
  echo "== ${v:-in-tree}"
  if [ -n "$v" ]; then export MIGYM_LIB=$PWD/$v; else unset MIGYM_LIB; fi
  timeout -k 10 300 python tools/kbench.py ${KB_SIZES:-4096 65536 262144} >> gpurun_out/kbench.log 2>&1
  rc=$?; echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/kbench.log; exit $rc; fi
done
unset MIGYM_LIB
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -3 gpurun_out/pytest_gpu.log
grep kernel_us gpurun_out/kbench.log
