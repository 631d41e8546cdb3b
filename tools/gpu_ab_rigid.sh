#!/bin/bash
# Same-box A/B of k_rigid_step builds: the in-tree library vs
# tools/variants/libmigym_prev.so (a build of the previous commit), phase
# settings at 4096 envs and the 262k-env kernel, alternating twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python tools/kbench_rigid_phases.py 4096 || exit 1
  MIGYM_LIB=tools/variants/libmigym_prev.so timeout -k 10 200 python tools/kbench_rigid_phases.py 4096 || exit 1
done
timeout -k 10 200 python tools/kbench.py 262144 && MIGYM_LIB=tools/variants/libmigym_prev.so timeout -k 10 200 python tools/kbench.py 262144
