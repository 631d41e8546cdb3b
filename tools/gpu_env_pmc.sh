#!/bin/bash
# k_env_step (S3 Franka) PMC passes on tools/kbench_franka.py: wave-cycle
# breakdown + instruction mix, then the instruction-cache counters.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-epmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
K="python tools/kbench_franka.py 4096"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/avail_$tag.txt 2>&1 || true
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_]*\|SQ_WAIT[A-Z_]*" gpurun_out/avail_$tag.txt | sort -u > gpurun_out/avail_sq_$tag.txt || true
timeout -s KILL 200 rocprofv3 --kernel-include-regex k_env_step \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM \
  -d gpurun_out/pmc1_$tag -o run --output-format csv -- $K > gpurun_out/pmc1_$tag.log 2>&1 || { tail -5 gpurun_out/pmc1_$tag.log; exit 1; }
P2=${P2:-SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_BRANCH}
timeout -s KILL 200 rocprofv3 --kernel-include-regex k_env_step --pmc $P2 \
  -d gpurun_out/pmc2_$tag -o run --output-format csv -- $K > gpurun_out/pmc2_$tag.log 2>&1 || { tail -5 gpurun_out/pmc2_$tag.log; exit 1; }
for d in pmc1 pmc2; do
  f=$(find gpurun_out/${d}_$tag -name '*counter_collection.csv' | head -1)
  python - "$f" <<'EOF'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_env_step" in r.get("Kernel_Name", "")]
acc = collections.defaultdict(list)
for r in rows:
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print("%-22s per-dispatch mean %.4g (n=%d)" % (k, sum(v) / len(v), len(v)))
EOF
done
