#!/bin/bash
# k_env_step (S3) evidence: the SQ counter passes of tools/gpu_env_pmc.sh and the
# per-phase cycle counters of the phase-timing build (tools/build_variant.sh
# envphase "-DMG_ENV_PHASE_TIMING") on the Franka cube-pick loop.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/gpu_env_pmc.sh ${1:-epmc} || exit 1
MIGYM_LIB=tools/variants/libmigym_envphase.so timeout -k 10 300 python tools/kbench_franka.py 4096 > gpurun_out/env_phase_${1:-epmc}.json || exit 1
cat gpurun_out/env_phase_${1:-epmc}.json
