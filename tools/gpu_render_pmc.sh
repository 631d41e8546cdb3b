#!/bin/bash
# k_render iteration: render GPU tests, the micro-benchmark, and two PMC passes
# (SQ instruction / wave-cycle counters; HBM write bytes + GPU clock) on it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-rpmc}
files=${2:-tests/test_render.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $files -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_$tag.log
timeout -k 10 200 python tools/kbench_render.py 1024 1600x900 > gpurun_out/kb_$tag.jsonl 2>&1 || { tail gpurun_out/kb_$tag.jsonl; exit 1; }
cat gpurun_out/kb_$tag.jsonl
K="python tools/kbench_render.py 1024 1600x900"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
  -d gpurun_out/pmc1_$tag -o run --output-format csv -- $K > gpurun_out/pmc1_$tag.log 2>&1 || { tail -5 gpurun_out/pmc1_$tag.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE \
  -d gpurun_out/pmc2_$tag -o run --output-format csv -- $K > gpurun_out/pmc2_$tag.log 2>&1 || { tail -5 gpurun_out/pmc2_$tag.log; exit 1; }
for d in pmc1 pmc2; do
  f=$(find gpurun_out/${d}_$tag -name '*counter_collection.csv' | head -1)
  python - "$f" <<'EOF'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_render" in r.get("Kernel_Name", "")]
acc = collections.defaultdict(list)
for r in rows:
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print("%-22s per-dispatch mean %.4g (n=%d)" % (k, sum(v) / len(v), len(v)))
EOF
done
