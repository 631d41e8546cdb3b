#!/bin/bash
# Round 6: the fused S3 controller (csrc/mg_ctrl.hip) against the torch one,
# the Franka tests driven by it, the driver's bench command, then the
# finer-hull measurement again after the cooperative vertex loop's fix (the
# parity run at 256 envs x 300 frames).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06g}
timeout -k 10 600 python -u -m pytest tests/test_franka_ctrl_gpu.py tests/test_franka_gpu.py -s -v --timeout 400 \
  --timeout-method thread > gpurun_out/ctrl_$tag.log 2>&1 || { tail -40 gpurun_out/ctrl_$tag.log; exit 1; }
grep -E "fused vs torch|hull-in-table|passed|failed" gpurun_out/ctrl_$tag.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
  || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_$tag.json').read().strip().splitlines()[-1])
print('S1', d['value'], d['ms_per_step'])
s3=d['s3_franka']; print('S3', s3['env_steps_per_s'], s3['ms_per_step'], s3.get('kernel_ms_avg'), s3.get('cubes_lifted_frac'))"
PARITY_ENVS=256 PARITY_FRAMES=300 bash tools/runs/r06_hulls.sh $tag
