#!/bin/bash
# Round 6 A/B of coupled-step variants (tools/variants/libmigym_$v.so): GPU parity
# (the 240-frame Franka pick and the box stacks) under each variant, then the
# kernel times of tools/kbench_franka.py (600 frames) under a kernel trace for
# the in-tree library and each variant; then the bench's S1 CPU-pipeline leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06j}
for v in ${AB_VARIANTS}; do
  MIGYM_LIB=tools/variants/libmigym_$v.so timeout -k 10 300 python -u -m pytest tests/test_franka_gpu.py \
    -k "parity_bitexact" -v --timeout 280 --timeout-method thread > gpurun_out/ab_parity_${v}_$tag.log 2>&1 \
    || { tail -20 gpurun_out/ab_parity_${v}_$tag.log; exit 1; }
  echo "== parity $v: $(tail -1 gpurun_out/ab_parity_${v}_$tag.log)"
done
AB_VARIANTS="${AB_VARIANTS}" KB_FRAMES=600 bash tools/gpu_round.sh $tag kfprof || exit 1
timeout -k 10 300 python -c "
import json, bench, torch
print(json.dumps(bench.s1_cpu_pipeline_rate(1024, 100, 10)))" > gpurun_out/cpupipe_$tag.json 2> gpurun_out/cpupipe_$tag.err \
  || { tail -10 gpurun_out/cpupipe_$tag.err; exit 1; }
cat gpurun_out/cpupipe_$tag.json
