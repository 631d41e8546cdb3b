"""Turns rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs, as
MI355X_MICROARCH.md §rocprofv3 PMC slots requires) of `bench.py` into per-launch
HBM traffic of the step kernel.

Units and gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE
are KiB; FETCH_SIZE under-reads wide coalesced loads by exactly 2x and other
widths are uncalibrated, so the read factor is calibrated here on a kernel of
the same run with a known read volume and the same access width (dword loads):
k_scatter_rows of bench.py --pmc-calibrate's indexed set_actor_root_state of
every actor reads the (2N, 13) f32 root tensor once (fully coalesced) plus the
int32 selection and root-body index per row.

usage: python profiles/collect_pmc.py FETCH.csv WRITE.csv ENVS OUT.json
       python profiles/collect_pmc.py FETCH.csv WRITE.csv ENVS OUT.json --kernel k_artic_chain \
              --bytes-per-env 532 --factor-from profiles/r03_pmc_rigid_262144.json
(the second form: another kernel of a run without a calibration kernel, its
FETCH_SIZE scaled by the read factor calibrated in the named S1 summary of the
same GPU session — dword SoA loads like the step kernel's)
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for key in ("k_rigid_step", "k_scatter_rows", "k_gather_rb_root", "k_gather_rows", "k_artic_step",
                    "k_artic_chain", "k_env_step", "k_env_np", "k_pile_step"):
            if key in name:
                name = key
        acc[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def other_kernel(f, nf, w, envs, out, kernel, bpe, factor_from):
    cal = json.load(open(factor_from))
    factor = cal["read_factor_calibrated"]
    key = [k for k in f if kernel in k][0]
    read = f[key] * 1024.0 * factor
    write = w[[k for k in w if kernel in k][0]] * 1024.0
    res = {"envs": envs, "kernel": kernel, "fetch_kib_raw": f[key], "write_kib_raw": write / 1024.0,
           "read_factor_calibrated": factor, "calibration": "from %s (%s)" % (factor_from, cal["calibration"]),
           "hbm_bytes_per_launch": read + write, "algorithmic_bytes_per_launch": bpe * envs, "launches": nf[key]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


def frame_kernels(f, nf, w, envs, out, kernels, per_frame, bpe, factor_from):
    """Several kernels that make up one frame (the S3 coupled step: k_env_np and
    k_env_step, each launched once per substep): bytes per frame = per_frame x
    the sum of the kernels' per-launch averages."""
    cal = json.load(open(factor_from))
    factor = cal["read_factor_calibrated"]
    parts = {}
    for k in kernels:
        key = [x for x in f if k in x][0]
        wk = [x for x in w if k in x][0]
        parts[k] = {"fetch_kib_raw": f[key], "write_kib_raw": w[wk], "launches": nf[key],
                    "hbm_bytes_per_launch": f[key] * 1024.0 * factor + w[wk] * 1024.0}
    total = per_frame * sum(p["hbm_bytes_per_launch"] for p in parts.values())
    # per FRAME, under its own key: bench.py prices the S3 roofline on
    # the frame's summed kernels, so its `traffic` is this value
    res = {"envs": envs, "kernel": " + ".join(kernels), "launches_per_frame_each": per_frame, "per_kernel": parts,
           "read_factor_calibrated": factor, "read_factor_borrowed": True,
           "calibration": "borrowed from %s (%s): no kernel of known read volume runs in the S3 benchmark, so the "
                          "FETCH_SIZE factor of the same GPU session's S1 calibration kernel (dword SoA loads) "
                          "is applied" % (factor_from, cal["calibration"]),
           "hbm_bytes_per_frame": total, "algorithmic_bytes_per_frame": bpe * envs}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


def main():
    fetch_csv, write_csv, envs, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    f, nf = per_kernel(fetch_csv, "FETCH_SIZE")
    w, _ = per_kernel(write_csv, "WRITE_SIZE")
    if "--frame-kernels" in sys.argv:
        a = sys.argv
        return frame_kernels(f, nf, w, envs, out, a[a.index("--frame-kernels") + 1].split(","),
                             int(a[a.index("--per-frame") + 1]), int(a[a.index("--bytes-per-env") + 1]),
                             a[a.index("--factor-from") + 1])
    if "--kernel" in sys.argv:
        a = sys.argv
        return other_kernel(f, nf, w, envs, out, a[a.index("--kernel") + 1], int(a[a.index("--bytes-per-env") + 1]),
                            a[a.index("--factor-from") + 1])
    # bench.py's S1 kernel: 376 B simulate share + 208 B of rigid-body and root
    # rows with the refresh fused into the step (STEP_FUSION_STEP_OUT, bench default)
    bpe = int(sys.argv[sys.argv.index("--bytes-per-env") + 1]) if "--bytes-per-env" in sys.argv else 584
    actors = 2 * envs
    # bench.py --pmc-calibrate: indexed sets of every actor (the fused step reads a
    # full set itself): the (2N, 13) rows, the int32 selection and root-body index
    known_read = actors * 13 * 4 + 2 * actors * 4
    factor = known_read / (f["k_scatter_rows"] * 1024.0)
    rigid_read = f["k_rigid_step"] * 1024.0 * factor
    rigid_write = w["k_rigid_step"] * 1024.0
    # WRITE_SIZE calibration: the paired refresh gather of
    # the calibration sets writes the (2N, 13) root rows and the (2N, 13)
    # rigid-body rows, 52-B rows in order (the same row pattern the fused step
    # writes), a known volume
    wcal = None
    if "k_gather_rb_root" in w:
        known_write = 2 * actors * 13 * 4
        wcal = {"kernel": "k_gather_rb_root", "known_bytes": known_write,
                "write_size_bytes": w["k_gather_rb_root"] * 1024.0,
                "write_factor": known_write / (w["k_gather_rb_root"] * 1024.0)}
    res = {
        "envs": envs,
        "kernel": "k_rigid_step",
        "fetch_kib_raw": f["k_rigid_step"],
        "write_kib_raw": w["k_rigid_step"],
        "read_factor_calibrated": factor,
        "calibration": "k_scatter_rows reads %d B per launch; FETCH_SIZE %.1f KiB" % (known_read,
                                                                                   f["k_scatter_rows"]),
        "hbm_bytes_per_launch": rigid_read + rigid_write,
        "write_calibration": wcal,
        "algorithmic_bytes_per_launch": bpe * envs,
        "algorithmic_bytes_per_env": bpe,
        "launches": nf["k_rigid_step"],
        "all_kernels_fetch_kib": f,
        "all_kernels_write_kib": w,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
