#!/bin/bash
# Round 6, one GPU call: (1) the Franka lift / hull-in-table stats at 256 and
# 4096 envs (tests/test_franka_gpu.py, printed), (2) tools/diag_franka_env.py at
# 4096 envs: deepest envs, longest runs past the 1 mm contact offset, per-frame
# logs and the watched envs' actions for a CPU replay on the oracle, (3) the
# large-N legs past the Infinity Cache: S1 fused at 2^20
# envs (bench.py, timed) and S2 at 2^20 gimbals (tools/kbench_gimbal.py, fused),
# then FETCH_SIZE / WRITE_SIZE passes of both (separate runs).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06d}
timeout -k 10 400 python -u -m pytest tests/test_franka_gpu.py -k lifts_cubes -s -v --timeout 380 \
  --timeout-method thread > gpurun_out/franka_stats_$tag.log 2>&1 || { tail -30 gpurun_out/franka_stats_$tag.log; exit 1; }
grep "hull-in-table" gpurun_out/franka_stats_$tag.log
DIAG_ACTIONS=gpurun_out/franka_actions_$tag.npz timeout -k 10 400 python -u tools/diag_franka_env.py 4096 600 \
  > gpurun_out/diag_franka_$tag.jsonl 2> gpurun_out/diag_franka_$tag.err || { tail -20 gpurun_out/diag_franka_$tag.err; exit 1; }
head -c 1500 gpurun_out/diag_franka_$tag.jsonl; echo
N=1048576
B="python bench.py --envs $N --steps 48 --warmup 5 --repeats 3 --no-cpu-baseline --no-gimbal --no-franka --no-cameras --no-large-n --no-default-legs"
timeout -k 10 300 $B > gpurun_out/bench_s1_${N}_$tag.json 2> gpurun_out/bench_s1_${N}_$tag.err || { tail -20 gpurun_out/bench_s1_${N}_$tag.err; exit 1; }
cut -c1-400 gpurun_out/bench_s1_${N}_$tag.json
MIGYM_KB_FUSED=1 timeout -k 10 300 python tools/kbench_gimbal.py $N > gpurun_out/kgimbal_${N}_$tag.jsonl 2> gpurun_out/kgimbal_${N}_$tag.err \
  || { tail -20 gpurun_out/kgimbal_${N}_$tag.err; exit 1; }
cat gpurun_out/kgimbal_${N}_$tag.jsonl
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${c}_$N -o run --output-format csv -- $B --pmc-calibrate --repeats 1 \
    > gpurun_out/pmc_${c}_$N.log 2>&1 || { tail -20 gpurun_out/pmc_${c}_$N.log; exit 1; }
  MIGYM_KB_FUSED=1 timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmcg_${c}_$N -o run --output-format csv -- \
    python tools/kbench_gimbal.py $N > gpurun_out/pmcg_${c}_$N.log 2>&1 || { tail -20 gpurun_out/pmcg_${c}_$N.log; exit 1; }
done
find gpurun_out/pmc_*_$N gpurun_out/pmcg_*_$N -name '*counter_collection.csv' | head
echo done
