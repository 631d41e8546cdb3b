#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
shopt -s nullglob
for v in "" tools/variants/*.so; do
  if [ -n "$v" ]; then export MIGYM_LIB=$PWD/$v; else unset MIGYM_LIB; fi
  timeout -k 10 300 python tools/kbench_gimbal.py ${KB_SIZES:-4096} >> gpurun_out/kbench_gimbal.log 2>&1 || exit $?
done
cat gpurun_out/kbench_gimbal.log
