"""Per-dispatch means of every counter of one kernel in a rocprofv3
counter_collection.csv (one --pmc pass), plus per-wave ratios when SQ_WAVES is
present. Prints one JSON object.

usage: pmc_summary.py counter_collection.csv KERNEL_SUBSTR
"""
import collections
import csv
import json
import sys


def main():
    path, kern = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kern in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: sum(v) / len(v) for k, v in sorted(acc.items())}
    out["dispatches"] = max((len(v) for v in acc.values()), default=0)
    w = out.get("SQ_WAVES")
    if w:
        out["per_wave"] = {k: v / w for k, v in out.items() if k.startswith("SQ_") and k != "SQ_WAVES"}
    if out.get("SQ_WAVE_CYCLES"):
        out["wait_any_frac"] = out.get("SQ_WAIT_ANY", 0.0) / out["SQ_WAVE_CYCLES"]
    print(json.dumps({"kernel": kern, "csv": path, "counters": out}))


if __name__ == "__main__":
    main()
