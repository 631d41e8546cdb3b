cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_render.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt_g3.log 2>&1; rc=$?; tail -15 gpurun_out/pt_g3.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/kbench_rigid_phases.py 4096 && timeout -k 10 200 python tools/kbench.py 4096 262144
