cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py 4096 65536 262144 1048576 && MIGYM_LIB=tools/variants/libmigym_narrow.so timeout -k 10 300 python tools/kbench.py 65536 262144 1048576
