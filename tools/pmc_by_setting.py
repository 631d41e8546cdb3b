"""Per-setting means of rocprofv3 counter_collection.csv rows of one kernel,
the dispatches split in order into equal consecutive groups, one per setting
name given (tools/kbench_rigid_phases.py runs its settings back to back with
the same launch count). Prints JSON: setting -> counter -> mean, plus per-wave
ratios.

usage: pmc_by_setting.py counter_collection.csv KERNEL_SUBSTR NAME...
"""
import collections
import csv
import json
import sys


def main():
    path, kern, names = sys.argv[1], sys.argv[2], sys.argv[3:]
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if kern not in r["Kernel_Name"]:
            continue
        per.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    rows = list(per.values())
    g = len(rows) // len(names)
    out = {}
    for k, name in enumerate(names):
        grp = rows[k * g:(k + 1) * g]
        m = {c: sum(r.get(c, 0.0) for r in grp) / len(grp) for c in grp[0]}
        w = m.get("SQ_WAVES", 0.0) or 1.0
        m["per_wave"] = {c: v / w for c, v in m.items() if c != "SQ_WAVES"}
        m["dispatches"] = len(grp)
        out[name] = m
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
