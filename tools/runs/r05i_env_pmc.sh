# The GPU-box command that produced profiles/r05_pmc_env_step_4096.json and the r05 SQ passes of k_env_np / k_env_step (run as: gpurun -- bash tools/runs/r05i_env_pmc.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_round.sh r05i pytest,smoke,bench,prof || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  KB_FRAMES=300 timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmcf_${c} -o run --output-format csv -- python tools/kbench_franka.py > gpurun_out/pmcf_$c.log 2>&1 || { tail -5 gpurun_out/pmcf_$c.log; exit 1; }
done
python profiles/collect_pmc.py $(find gpurun_out/pmcf_FETCH_SIZE -name '*counter_collection.csv' | head -1) $(find gpurun_out/pmcf_WRITE_SIZE -name '*counter_collection.csv' | head -1) 4096 gpurun_out/r05_pmc_env_step_4096.json --frame-kernels k_env_np,k_env_step --per-frame 2 --bytes-per-env 5844 --factor-from profiles/r04_pmc_rigid_262144.json | head -30
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
for k in k_env_np k_env_step; do
  KB_FRAMES=300 timeout -s KILL 200 rocprofv3 --kernel-include-regex "$k" --pmc $SQ1 -d gpurun_out/sq_$k -o run --output-format csv -- python tools/kbench_franka.py > gpurun_out/sq_$k.log 2>&1 || { tail -5 gpurun_out/sq_$k.log; exit 1; }
  python tools/pmc_summary.py $(find gpurun_out/sq_$k -name '*counter_collection.csv' | head -1) $k | tee gpurun_out/r05_sq_$k.json
done
