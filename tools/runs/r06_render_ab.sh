#!/bin/bash
# Same-box A/B of the camera renderer: in-tree libmigym.so vs a variant build
# (tools/variants/libmigym_$1.so), k_render at 1024 x 1600x900 twice each, then
# the render parity tests on the variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
v=${1:-rslp}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python tools/kbench_render.py 1024 1600x900 >> gpurun_out/render_ab_$v.jsonl 2>&1 || exit 1
  MIGYM_LIB=tools/variants/libmigym_$v.so timeout -k 10 200 python tools/kbench_render.py 1024 1600x900 \
    >> gpurun_out/render_ab_$v.jsonl 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/render_ab_$v.jsonl | cut -c1-300
MIGYM_LIB=tools/variants/libmigym_$v.so timeout -k 10 300 python -u -m pytest tests/test_render.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_render_$v.log 2>&1; tail -2 gpurun_out/pytest_render_$v.log
