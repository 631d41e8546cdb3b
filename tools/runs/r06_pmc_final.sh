#!/bin/bash
# Round 6, final HBM-traffic passes (FETCH_SIZE / WRITE_SIZE in separate runs, no
# trace domains) on this round's kernels: S1 k_rigid_step1 at 4096 and 262,144
# envs (bench.py --pmc-calibrate, gpu_round.sh's pmc step) and S2 k_artic_chain
# at 262,144; S3 k_env_np + k_env_step per frame at 4096 Franka envs
# (tools/kbench_franka.py, 300 frames). profiles/collect_pmc.py turns each pair
# into bytes per launch (per frame for S3) -> gpurun_out/r06_pmc_*.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# the 262k-env scene builds run silent for minutes under the counters: a
# heartbeat file under gpurun_out/ shows the run is alive (ended with the script)
( while sleep 50; do date >> gpurun_out/heartbeat_r06p.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
bash tools/gpu_round.sh r06p pmc || exit 1
csv() { find "$1" -name '*counter_collection.csv' | head -1; }
for n in 4096 262144; do
  python profiles/collect_pmc.py $(csv gpurun_out/pmc_FETCH_SIZE_$n) $(csv gpurun_out/pmc_WRITE_SIZE_$n) $n \
    gpurun_out/r06_pmc_rigid_$n.json || exit 1
done
python profiles/collect_pmc.py $(csv gpurun_out/pmcg_FETCH_SIZE_262144) $(csv gpurun_out/pmcg_WRITE_SIZE_262144) 262144 \
  gpurun_out/r06_pmc_gimbal_262144.json --kernel k_artic_chain --bytes-per-env 532 \
  --factor-from gpurun_out/r06_pmc_rigid_262144.json || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  KB_FRAMES=300 timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmcf_${c} -o run --output-format csv -- \
    python tools/kbench_franka.py > gpurun_out/pmcf_$c.log 2>&1 || { tail -5 gpurun_out/pmcf_$c.log; exit 1; }
done
python profiles/collect_pmc.py $(csv gpurun_out/pmcf_FETCH_SIZE) $(csv gpurun_out/pmcf_WRITE_SIZE) 4096 \
  gpurun_out/r06_pmc_env_step_4096.json --frame-kernels k_env_np,k_env_step --per-frame 2 --bytes-per-env 5844 \
  --factor-from gpurun_out/r06_pmc_rigid_262144.json || exit 1
find gpurun_out/pmc_* gpurun_out/pmcg_* gpurun_out/pmcf_* -name '*.csv' -size +20M -delete
for f in gpurun_out/r06_pmc_*.json; do echo "== $f"; head -c 600 $f; echo; done
