#!/bin/bash
# Whole-step A/B on one box: the S1 bench line for every tools/variants/*.so, twice, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
shopt -s nullglob
for rep in 1 2; do
  for v in tools/variants/*.so; do
    MIGYM_LIB=$PWD/$v timeout -k 10 200 python bench.py --no-franka --no-gimbal --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab.tmp 2>&1 || { tail -20 gpurun_out/ab.tmp; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab.tmp').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,2), 'us graph', round(d['config'].get('eager_ms_per_step',0)*1e3,2), 'us eager')" | tee -a gpurun_out/ab.log
  done
done
