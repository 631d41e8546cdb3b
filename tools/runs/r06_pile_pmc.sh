#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs, no trace domains) of the S6
# pile kernel at 4096 envs (tools/kbench_pile.py): profiles/collect_pmc.py turns
# them into per-launch HBM bytes (profiles/r06_pmc_pile_4096.json).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-include-regex k_pile_step --pmc $c -d gpurun_out/pmcp_$c -o run \
    --output-format csv -- python tools/kbench_pile.py 4096 > gpurun_out/pmcp_$c.log 2>&1 \
    || { tail -20 gpurun_out/pmcp_$c.log; exit 1; }
done
F=$(find gpurun_out/pmcp_FETCH_SIZE -name '*counter_collection.csv' | head -1)
W=$(find gpurun_out/pmcp_WRITE_SIZE -name '*counter_collection.csv' | head -1)
cp "$F" gpurun_out/pmcp_fetch.csv && cp "$W" gpurun_out/pmcp_write.csv
find gpurun_out/pmcp_FETCH_SIZE gpurun_out/pmcp_WRITE_SIZE -name '*.csv' -size +20M -delete
echo pmc done
