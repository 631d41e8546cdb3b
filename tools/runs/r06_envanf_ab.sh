#!/bin/bash
# Round 6: the coupled step's sweep order A/B (MG_ENV_SWEEP_ANF, a variant build):
# Franka lift fraction and kernel times over 600 frames (tools/kbench_franka.py
# under a kernel trace), and the hull-in-table summary (tools/diag_franka_env.py)
# for the in-tree library and the variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06e}
for v in intree envanf; do
  lib=""
  [ "$v" != intree ] && lib=tools/variants/libmigym_$v.so
  MIGYM_LIB=$lib KB_FRAMES=600 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kfprof_${v}_$tag -o run \
    --output-format csv -- python tools/kbench_franka.py > gpurun_out/kfprof_${v}_$tag.log 2>&1 \
    || { tail -5 gpurun_out/kfprof_${v}_$tag.log; exit 1; }
  echo "== $v"; grep kernel_us gpurun_out/kfprof_${v}_$tag.log | cut -c1-300
  f=$(find gpurun_out/kfprof_${v}_$tag -name '*kernel_stats.csv' | head -1); grep -E "k_env" "$f" | cut -c1-160
  find gpurun_out/kfprof_${v}_$tag -name '*kernel_trace.csv' -delete
  MIGYM_LIB=$lib timeout -k 10 400 python -u tools/diag_franka_env.py 4096 600 > gpurun_out/diag_franka_${v}_$tag.jsonl \
    2> gpurun_out/diag_franka_${v}_$tag.err || { tail -20 gpurun_out/diag_franka_${v}_$tag.err; exit 1; }
  head -1 gpurun_out/diag_franka_${v}_$tag.jsonl
done
