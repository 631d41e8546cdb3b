#!/bin/bash
# FETCH_SIZE of k_rigid_step1 at 262k envs with the fused root-state read and
# without it (KB_FUSION=0): raw KiB per launch, same box, separate passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
n=${1:-262144}
for fu in 3 0; do
  KB_FUSION=$fu timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcfu_$fu -o run --output-format csv -- python tools/kbench.py $n > gpurun_out/pmcfu_$fu.log 2>&1 || { tail -5 gpurun_out/pmcfu_$fu.log; exit 1; }
  f=$(find gpurun_out/pmcfu_$fu -name '*counter_collection.csv' | head -1)
  python - "$f" $fu <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "k_rigid_step1" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
print("fusion", sys.argv[2], "k_rigid_step1 FETCH_SIZE KiB per launch: %.1f (n=%d)" % (sum(v) / len(v), len(v)))
PY
done
