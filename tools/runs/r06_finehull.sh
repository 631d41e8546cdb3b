#!/bin/bash
# Round 6: hulls past the importer's 32-vertex default on the in-tree library
# (MG_HULL_MAX_VERTS / _FACES = 255, mg_env.hip's chunked cooperative loops; no
# variant build). tests/test_fine_hulls.py's GPU parity (240- and 200-vertex
# prisms), then per Franka hand setting (32 in-tree, 64, the full 102 vertices)
# the 240-frame GPU parity test and k_env_np / k_env_step times at 4096 envs
# (tools/kbench_franka.py under a kernel trace) — against profiles/r06_hulls.log
# (the variant library built with the caps raised at compile time).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06h}
timeout -k 10 300 python -u -m pytest tests/test_fine_hulls.py -m gpu -v --timeout 240 --timeout-method thread \
  > gpurun_out/finehull_pytest_$tag.log 2>&1 || { tail -30 gpurun_out/finehull_pytest_$tag.log; exit 1; }
tail -1 gpurun_out/finehull_pytest_$tag.log
run_setting() {   # name asset caps
  local v=$1
  export MIGYM_FRANKA_ASSET=$2 MIGYM_HULL_CAPS=$3
  timeout -k 10 400 python -u -m pytest tests/test_franka_gpu.py -k "parity_bitexact" -v --timeout 380 \
    --timeout-method thread > gpurun_out/hull_parity_${v}_$tag.log 2>&1 || { tail -20 gpurun_out/hull_parity_${v}_$tag.log; return 1; }
  tail -1 gpurun_out/hull_parity_${v}_$tag.log
  KB_FRAMES=600 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hull_kf_${v}_$tag -o run \
    --output-format csv -- python tools/kbench_franka.py > gpurun_out/hull_kf_${v}_$tag.log 2>&1 \
    || { tail -5 gpurun_out/hull_kf_${v}_$tag.log; return 1; }
  echo "== $v"; grep kernel_us gpurun_out/hull_kf_${v}_$tag.log | cut -c1-300
  f=$(find gpurun_out/hull_kf_${v}_$tag -name '*kernel_stats.csv' | head -1); grep -E "k_env" "$f" | cut -c1-160
  find gpurun_out/hull_kf_${v}_$tag -name '*kernel_trace.csv' -delete
  unset MIGYM_FRANKA_ASSET MIGYM_HULL_CAPS
}
run_setting hand32 franka/franka_proxy.urdf "" || exit 1
run_setting hand64 franka_hand64/franka_proxy.urdf "hand.obj=64/128,hand_hull.obj=64/128" || exit 1
run_setting handfull franka_handfull/franka_proxy.urdf "hand.obj=128/255,hand_hull.obj=128/255" || exit 1
echo done
