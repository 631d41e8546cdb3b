cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_gimbal -o run --output-format csv -- python tools/kbench_gimbal.py 4096 > gpurun_out/pmc_gimbal.log 2>&1 || exit 1
f=$(find gpurun_out/pmc_gimbal -name '*counter_collection.csv' | head -1)
python tools/pmc_by_setting.py "$f" k_artic_lanes gimbal4096
