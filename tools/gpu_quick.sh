#!/bin/bash
# Quick GPU check of selected tests (default: the parity / render / graphics
# files) plus the S1 kernel timings. Usage: gpurun -- bash tools/gpu_quick.sh [test files...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
files=${*:-tests/test_parity_gpu.py tests/test_render.py tests/test_graphics_fixture.py}
timeout -k 10 500 python -u -m pytest $files -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_quick.log 2>&1; rc=$?; tail -15 gpurun_out/pt_quick.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/kbench_rigid_phases.py 4096 && timeout -k 10 200 python tools/kbench.py 4096 262144
