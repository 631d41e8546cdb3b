#!/bin/bash
# k_env_step A/B: tools/kbench_franka.py for the in-tree build and every tools/variants/*.so.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
shopt -s nullglob
for v in "" tools/variants/*.so; do
  echo "== ${v:-in-tree}"
  if [ -n "$v" ]; then export MIGYM_LIB=$PWD/$v; else unset MIGYM_LIB; fi
  timeout -k 10 300 python tools/kbench_franka.py ${KB_SIZES:-4096} >> gpurun_out/kbench_franka.log 2>&1
  rc=$?; echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/kbench_franka.log; exit $rc; fi
done
grep kernel_us gpurun_out/kbench_franka.log
