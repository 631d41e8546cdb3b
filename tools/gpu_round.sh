#!/bin/bash
# The one GPU-box script: GPU tests, smoke(), the bench line (the driver's own
# command and the 600-step default), a rocprofv3 kernel-trace summary of the
# bench, PMC passes and the kernel microbenchmarks. Every GPU step has its own
# time limit and the steps are chained: the first failure ends the run.
# Usage (from this container):
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh <tag> [steps] [pytest -k expr]
#   steps: comma list of
#     probe      host facts (CPU count, affinity, cgroup quota)
#     pytest     python -m pytest tests -m gpu (optionally -k "$3")
#     smoke      __graft_entry__.smoke()
#     bench      python bench.py --gpus 1 --steps 20 --warmup 5 (the driver's command)
#     bench600   python bench.py (defaults: 600 steps)
#     prof       rocprofv3 --kernel-trace --stats of the driver's bench command
#     pmc        rocprofv3 FETCH_SIZE / WRITE_SIZE passes of the S1 bench (PMC_SIZES, default 4096 262144)
#     kbench     tools/kbench.py sweep (k_rigid_step1, 2^12 .. 2^21 envs)
#     kgimbal    tools/kbench_gimbal.py (S2 kernel at 4096 .. 262144 gimbals)
#     kfranka    tools/kbench_franka.py (S3 kernel at 4096 Franka envs; and $AB_VARIANT's library if set)
#     sqrigid    SQ counter pass of k_rigid_step1 (tools/kbench_rigid_phases.py 4096, per setting)
#     sqenv      SQ counter passes of k_env_step (tools/kbench_franka.py 4096) + the phase-timing
#                variant (tools/build_variant.sh envphase "-DMG_ENV_PHASE_TIMING", built beforehand)
#     sqgimbal   SQ counter pass of k_artic_chain (tools/kbench_gimbal.py 4096 262144)
#     sqgimbal4k SQ passes + kernel trace of k_artic_chain at 4096 gimbals alone
#     sqrender   SQ + WRITE_SIZE passes of k_render (tools/kbench_render.py 1024 1600x900)
#     kfprof     rocprofv3 kernel trace of tools/kbench_franka.py (KB_FRAMES, default 300) for the
#                in-tree library and each tools/variants/libmigym_$v.so of $AB_VARIANTS
#     rphases    tools/kbench_rigid_phases.py 4096 (k_rigid_step1 under settings that drop one part)
#     ab         same-box A/B: in-tree libmigym.so vs tools/variants/libmigym_$AB_VARIANT.so on
#                tools/kbench.py at $AB_SIZES (default 4096 262144), twice
#   default: pytest,smoke,bench,prof
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-r04}
steps=${2:-pytest,smoke,bench,prof}
kexpr=${3:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS="--gpus 1 --steps 20 --warmup 5"
has() { [[ ",$steps," == *",$1,"* ]]; }
if has probe; then
  { echo "nproc $(nproc)"; python -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))";
    cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > gpurun_out/probe_$tag.txt 2>&1
  cat gpurun_out/probe_$tag.txt
fi
if has pytest; then
  kargs=()
  [[ -n $kexpr ]] && kargs=(-k "$kexpr")
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread "${kargs[@]}" \
    > gpurun_out/pytest_gpu_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$tag.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$tag.log
fi
if has smoke; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 \
    || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
  tail -1 gpurun_out/smoke_$tag.log
fi
if has bench; then
  timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
    || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
  cut -c1-600 gpurun_out/bench_$tag.json
fi
if has bench600; then
  timeout -k 10 400 python bench.py > gpurun_out/bench600_$tag.json 2> gpurun_out/bench600_$tag.err \
    || { tail -20 gpurun_out/bench600_$tag.err; exit 1; }
  cut -c1-600 gpurun_out/bench600_$tag.json
fi
if has prof; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv \
    -- python bench.py $BENCH_ARGS --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 \
    || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
  tail -1 gpurun_out/prof_$tag.log | cut -c1-300
  f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1); cut -c1-150 "$f" | head -16
  find gpurun_out/prof_$tag -name '*kernel_trace.csv' -delete   # the summary is kept (gpurun_out <= 64 MiB)
fi
if has pmc; then
  # FETCH_SIZE and WRITE_SIZE in separate runs (one counter block each, no trace
  # domains combined); profiles/collect_pmc.py turns the CSVs into per-launch bytes
  for n in ${PMC_SIZES:-4096 262144}; do
    B="python bench.py --envs $n --steps 48 --warmup 5 --repeats 1 --pmc-calibrate --no-cpu-baseline --no-gimbal --no-franka --no-cameras --no-large-n --no-default-legs --no-piles"
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${c}_$n -o run --output-format csv -- $B \
        > gpurun_out/pmc_${c}_$n.log 2>&1 || { tail -20 gpurun_out/pmc_${c}_$n.log; exit 1; }
    done
  done
  for n in ${PMC_GIMBAL_SIZES:-262144}; do          # S2: k_artic_chain (tools/kbench_gimbal.py, fused as bench.py)
    for c in FETCH_SIZE WRITE_SIZE; do
      MIGYM_KB_FUSED=1 timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmcg_${c}_$n -o run --output-format csv -- \
        python tools/kbench_gimbal.py $n > gpurun_out/pmcg_${c}_$n.log 2>&1 || { tail -20 gpurun_out/pmcg_${c}_$n.log; exit 1; }
    done
  done
  echo pmc done
fi
if has kbench; then
  timeout -k 10 300 python tools/kbench.py 4096 32768 262144 524288 1048576 2097152 \
    > gpurun_out/kbench_$tag.jsonl 2> gpurun_out/kbench_$tag.err || { tail -20 gpurun_out/kbench_$tag.err; exit 1; }
  cat gpurun_out/kbench_$tag.jsonl
fi
if has kgimbal; then
  timeout -k 10 300 python tools/kbench_gimbal.py 4096 32768 262144 \
    > gpurun_out/kgimbal_$tag.jsonl 2> gpurun_out/kgimbal_$tag.err || { tail -20 gpurun_out/kgimbal_$tag.err; exit 1; }
  MIGYM_KB_FUSED=1 timeout -k 10 300 python tools/kbench_gimbal.py 4096 32768 262144 \
    >> gpurun_out/kgimbal_$tag.jsonl 2>> gpurun_out/kgimbal_$tag.err || { tail -20 gpurun_out/kgimbal_$tag.err; exit 1; }
  cat gpurun_out/kgimbal_$tag.jsonl
fi
if has kfranka; then
  timeout -k 10 300 python tools/kbench_franka.py > gpurun_out/kfranka_$tag.jsonl 2> gpurun_out/kfranka_$tag.err \
    || { tail -20 gpurun_out/kfranka_$tag.err; exit 1; }
  if [ -n "$AB_VARIANT" ]; then
    MIGYM_LIB=tools/variants/libmigym_$AB_VARIANT.so timeout -k 10 300 python tools/kbench_franka.py \
      >> gpurun_out/kfranka_$tag.jsonl 2>> gpurun_out/kfranka_$tag.err || { tail -20 gpurun_out/kfranka_$tag.err; exit 1; }
  fi
  cut -c1-400 gpurun_out/kfranka_$tag.jsonl
fi
# one SQ counter pass (<= 8 SQ counters, no trace domains): sq_pass NAME KERNEL "COUNTERS" CMD...
sq_pass() {
  local name=$1 kern=$2 ctrs=$3; shift 3
  timeout -s KILL 200 rocprofv3 --kernel-include-regex "$kern" --pmc $ctrs -d gpurun_out/sq_${name}_$tag -o run \
    --output-format csv -- "$@" > gpurun_out/sq_${name}_$tag.log 2>&1 || { tail -5 gpurun_out/sq_${name}_$tag.log; return 1; }
  local f
  f=$(find gpurun_out/sq_${name}_$tag -name '*counter_collection.csv' | head -1)
  python tools/pmc_summary.py "$f" "$kern" | tee gpurun_out/sq_${name}_$tag.json
}
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
if has sqrigid; then
  sq_pass rigid k_rigid_step1 "$SQ1" python tools/kbench_rigid_phases.py 4096 || exit 1
fi
if has sqenv; then
  sq_pass env k_env_step "$SQ1" python tools/kbench_franka.py 4096 || exit 1
  if [ -f tools/variants/libmigym_envphase.so ]; then
    MIGYM_LIB=tools/variants/libmigym_envphase.so timeout -k 10 300 python tools/kbench_franka.py 4096 \
      > gpurun_out/env_phase_$tag.json || exit 1
    cat gpurun_out/env_phase_$tag.json
  fi
fi
if has sqgimbal; then
  sq_pass gimbal k_artic_chain "$SQ1" python tools/kbench_gimbal.py 4096 262144 || exit 1
fi
if has sqgimbal4k; then
  sq_pass gimbal4k k_artic_chain "$SQ1" python tools/kbench_gimbal.py 4096 || exit 1
  sq_pass gimbal4k_b k_artic_chain "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" python tools/kbench_gimbal.py 4096 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ktr_gimbal4k_$tag -o run --output-format csv \
    -- python tools/kbench_gimbal.py 4096 > gpurun_out/ktr_gimbal4k_$tag.log 2>&1 || { tail -5 gpurun_out/ktr_gimbal4k_$tag.log; exit 1; }
fi
if has sqrender; then
  sq_pass render k_render "$SQ1" python tools/kbench_render.py 1024 1600x900 || exit 1
  sq_pass render_w k_render "WRITE_SIZE GRBM_GUI_ACTIVE" python tools/kbench_render.py 1024 1600x900 || exit 1
fi
if has kfprof; then
  for v in intree ${AB_VARIANTS:-}; do
    lib=""
    [ "$v" != intree ] && lib=tools/variants/libmigym_$v.so
    MIGYM_LIB=$lib KB_FRAMES=${KB_FRAMES:-300} timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      -d gpurun_out/kfprof_${v}_$tag -o run --output-format csv -- python tools/kbench_franka.py \
      > gpurun_out/kfprof_${v}_$tag.log 2>&1 || { tail -5 gpurun_out/kfprof_${v}_$tag.log; exit 1; }
    echo "== $v"; grep kernel_us gpurun_out/kfprof_${v}_$tag.log | cut -c1-200
    f=$(find gpurun_out/kfprof_${v}_$tag -name '*kernel_stats.csv' | head -1); grep -E "k_env" "$f" | cut -c1-160
    find gpurun_out/kfprof_${v}_$tag -name '*kernel_trace.csv' -delete   # large; the stats stay
  done
fi
if has rphases; then
  timeout -k 10 300 python tools/kbench_rigid_phases.py 4096 > gpurun_out/rphases_$tag.jsonl \
    2> gpurun_out/rphases_$tag.err || { tail -20 gpurun_out/rphases_$tag.err; exit 1; }
  cat gpurun_out/rphases_$tag.jsonl
fi
if has ab; then
  for r in 1 2; do
    for n in ${AB_SIZES:-4096 262144}; do
      timeout -k 10 200 python tools/kbench.py $n >> gpurun_out/ab_$tag.jsonl || exit 1
      MIGYM_LIB=tools/variants/libmigym_$AB_VARIANT.so timeout -k 10 200 python tools/kbench.py $n \
        >> gpurun_out/ab_$tag.jsonl || exit 1
    done
  done
  cat gpurun_out/ab_$tag.jsonl
fi
exit 0
