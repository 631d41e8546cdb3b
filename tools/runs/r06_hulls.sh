#!/bin/bash
# Round 6: the Franka hand's collision hull at the
# importer's 32-vertex cap (in-tree), at 64 vertices and at its full 102 (the
# finger hulls are already exact at 18). The finer two run a library built with
# MG_HULL_MAX_VERTS=128 / MG_HULL_MAX_FACES=256 (tools/variants/libmigym_hull128.so)
# on assets/franka_hand64 and assets/franka_handfull with the importer's caps
# raised for that mesh (MIGYM_HULL_CAPS). Per setting: the 240-frame GPU parity
# test against the oracle, k_env_np / k_env_step times and the lift fraction over
# 600 frames (tools/kbench_franka.py under a kernel trace), the hull-in-table
# summary (tools/diag_franka_env.py). Then the S2 PMC pass at 4096 gimbals.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06f}
run_setting() {   # name lib asset caps
  local v=$1
  export MIGYM_LIB=$2 MIGYM_FRANKA_ASSET=$3 MIGYM_HULL_CAPS=$4
  MIGYM_PARITY_ENVS=${PARITY_ENVS:-64} MIGYM_PARITY_FRAMES=${PARITY_FRAMES:-240} timeout -k 10 400 python -u -m pytest tests/test_franka_gpu.py -k "parity_bitexact" -v --timeout 380 \
    --timeout-method thread > gpurun_out/hull_parity_${v}_$tag.log 2>&1 || { tail -20 gpurun_out/hull_parity_${v}_$tag.log; return 1; }
  tail -1 gpurun_out/hull_parity_${v}_$tag.log
  KB_FRAMES=600 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hull_kf_${v}_$tag -o run \
    --output-format csv -- python tools/kbench_franka.py > gpurun_out/hull_kf_${v}_$tag.log 2>&1 \
    || { tail -5 gpurun_out/hull_kf_${v}_$tag.log; return 1; }
  echo "== $v"; grep kernel_us gpurun_out/hull_kf_${v}_$tag.log | cut -c1-300
  f=$(find gpurun_out/hull_kf_${v}_$tag -name '*kernel_stats.csv' | head -1); grep -E "k_env" "$f" | cut -c1-160
  find gpurun_out/hull_kf_${v}_$tag -name '*kernel_trace.csv' -delete
  timeout -k 10 400 python -u tools/diag_franka_env.py 4096 600 > gpurun_out/hull_diag_${v}_$tag.jsonl \
    2> gpurun_out/hull_diag_${v}_$tag.err || { tail -20 gpurun_out/hull_diag_${v}_$tag.err; return 1; }
  head -1 gpurun_out/hull_diag_${v}_$tag.jsonl | cut -c1-600
  unset MIGYM_LIB MIGYM_FRANKA_ASSET MIGYM_HULL_CAPS
}
run_setting hand32 "" franka/franka_proxy.urdf "" || exit 1
run_setting hand64 tools/variants/libmigym_hull128.so franka_hand64/franka_proxy.urdf \
  "hand.obj=64/128,hand_hull.obj=64/128" || exit 1
run_setting handfull tools/variants/libmigym_hull128.so franka_handfull/franka_proxy.urdf \
  "hand.obj=128/256,hand_hull.obj=128/256" || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  MIGYM_KB_FUSED=1 timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmcg_${c}_4096 -o run --output-format csv -- \
    python tools/kbench_gimbal.py 4096 > gpurun_out/pmcg_${c}_4096.log 2>&1 || { tail -20 gpurun_out/pmcg_${c}_4096.log; exit 1; }
done
echo done
