#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 600 --warmup 60 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
