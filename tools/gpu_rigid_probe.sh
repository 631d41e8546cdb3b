#!/bin/bash
# k_rigid_step1 probes at 4096 envs: solver-setting phase timings
# (tools/kbench_rigid_phases.py) and one rocprofv3 SQ counter pass (8 SQ
# counters, no trace domains) over the same four settings, reported per setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-probe}
timeout -k 10 300 python tools/kbench_rigid_phases.py 4096 > gpurun_out/rigid_phases_$tag.jsonl 2>&1 || { tail gpurun_out/rigid_phases_$tag.jsonl; exit 1; }
cat gpurun_out/rigid_phases_$tag.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS \
  -d gpurun_out/pmc_sq_$tag -o run --output-format csv -- python tools/kbench_rigid_phases.py 4096 > gpurun_out/pmc_sq_$tag.log 2>&1 || { tail gpurun_out/pmc_sq_$tag.log; exit 1; }
f=$(find gpurun_out/pmc_sq_$tag -name '*counter_collection.csv' | head -1)
python tools/pmc_by_setting.py "$f" k_rigid_step default iters_1_0 sub_1 airborne | tee gpurun_out/pmc_sq_$tag.json
