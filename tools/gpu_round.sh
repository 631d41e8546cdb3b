#!/bin/bash
# The one GPU-box script: GPU tests, smoke(), the default bench line, and a
# rocprofv3 kernel-trace summary of the same bench command. Every GPU step has
# its own time limit and the steps are chained: the first failure ends the run.
# Usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_round.sh [tag] [steps]
#   steps: comma list of pytest,smoke,bench,prof (default: all)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r02}
steps=${2:-pytest,smoke,bench,prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ $steps == *pytest* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$tag.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$tag.log
fi
if [[ $steps == *smoke* ]]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 \
    || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
  tail -1 gpurun_out/smoke_$tag.log
fi
if [[ $steps == *bench* ]]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
    || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
  cat gpurun_out/bench_$tag.json
fi
if [[ $steps == *prof* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv \
    -- python bench.py --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
  tail -1 gpurun_out/prof_$tag.log
  f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1); cut -c1-150 "$f" | head -16
fi
