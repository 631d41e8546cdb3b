#!/bin/bash
# Same-box A/B: in-tree libmigym.so vs tools/variants/libmigym_$1.so with
# tools/kbench.py at the env counts given after the variant name.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
v=$1; shift
for r in 1 2; do
  for n in "$@"; do
    timeout -k 10 200 python tools/kbench.py $n || exit 1
    MIGYM_LIB=tools/variants/libmigym_$v.so timeout -k 10 200 python tools/kbench.py $n || exit 1
  done
done
