cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in "" sub1 nodyn nokin; do
  if [ -z "$v" ]; then timeout -k 10 120 python tools/kbench_gimbal.py 4096 || exit 1
  else MIGYM_LIB=tools/variants/libmigym_$v.so timeout -k 10 120 python tools/kbench_gimbal.py 4096 || exit 1; fi
done
