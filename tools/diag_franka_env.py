"""Diagnostic: the S3 pick loop at n envs (tests/
test_franka_gpu.py::test_franka_pick_lifts_cubes) watched for (a) the hand /
finger hulls reaching into the table box (tests/franka_geom.py: deepest hull
vertex inside the box, every frame, every env) and (b) cubes that end at rest
below the table top beside it. A second, identical run (the step is
deterministic) then logs the selected envs frame by frame around their worst
frame: DOF positions against their limits, the penetration depth, the net
contact forces of cube / hand / fingers, and the contacts k_env_np handed to
the step (mg_debug_copy_env_ctab: participants, separation, normal).
Usage: python tools/diag_franka_env.py [n] [frames] [env ...]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from isaacgym import gymapi, gymtorch  # noqa: E402
from test_isaacgym_amd import _native as N  # noqa: E402
from test_franka_gpu import _setup, _control  # noqa: E402
import franka_geom as FG  # noqa: E402

NAMES = {64: "cube", 80: "table", -1: "ground"}


def who(p):
    if p >= 128:
        return "limit(dof %d)" % (p - 128)
    if p in NAMES:
        return NAMES[p]
    return "link%d" % p


def contacts(sim, e):
    cap = N.lib.mg_env_ctab_floats()
    buf = (ctypes.c_float * cap)()
    n = N.lib.mg_debug_copy_env_ctab(sim.native, e, buf, cap)   # every env of the scene is coupled
    N.check(n if n < 0 else 0, "mg_debug_copy_env_ctab")
    a = np.frombuffer(buf, np.float32)[:n]
    ib = a.view(np.int32)
    nct = min(int(ib[0]), (n - 8) // 24)
    out = []
    for c in range(nct):
        r = 8 + c * 10
        out.append((who(int(ib[r])), who(int(ib[r + 1])), float(a[r + 8]), a[r + 5:r + 8].round(3).tolist()))
    return int(ib[0]), int(ib[1]), out


def run(n, frames, watch=(), around=None, around_run=False):
    gym = gymapi.acquire_gym()
    sim, info, rb, dof, jac, mm, ctl = _setup(gym, n)
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    A = sim.model_arrays
    bi = torch.tensor(info["box_idxs"], device="cuda:0")
    hi = torch.tensor(info["hand_idxs"], device="cuda:0")
    hulls = torch.stack([hi, hi + 1, hi + 2], 1)
    props = torch.tensor(A["dof_props"][:9], device="cuda:0")
    lo, up = props[:, 5], props[:, 6]
    worst = torch.zeros(n, dtype=torch.float64, device="cuda:0")
    worst_f = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    log = {e: [] for e in watch}
    run_1mm = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    best_run = torch.zeros_like(run_1mm)
    best_run_end = torch.zeros_like(run_1mm)
    acts = {e: [] for e in watch}   # the controller's targets / efforts (tools/replay_franka_env.py)
    for f in range(frames):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        pa, ea = _control(gym, sim, info, rb, dof, jac, mm, ctl, n)
        gym.refresh_net_contact_force_tensor(sim)
        d = FG.penetration_depth(A, rb, hulls, bi - 1)
        upd = d > worst
        worst = torch.where(upd, d, worst)
        worst_f = torch.where(upd, torch.full_like(worst_f, f), worst_f)
        run_1mm = torch.where(d > 0.001, run_1mm + 1, torch.zeros_like(run_1mm))
        longer = run_1mm > best_run
        best_run = torch.where(longer, run_1mm, best_run)
        best_run_end = torch.where(longer, torch.full_like(best_run_end, f), best_run_end)
        for e in watch:
            acts[e].append(np.stack([pa.view(n, 9)[e].cpu().numpy(), ea.view(n, 9)[e].cpu().numpy()]))
            if around is not None and abs(f - around[e]) > 12 and not (around_run and float(d[e]) > 0.0005):
                continue
            q = dof[:, 0].view(n, 9)[e]
            nct, nanc, cl = contacts(sim, e)
            log[e].append({
                "frame": f, "depth_mm": round(1e3 * float(d[e]), 3),
                "q_minus_lo_deg": torch.rad2deg(q - lo).round(decimals=2).tolist(),
                "up_minus_q_deg": torch.rad2deg(up - q).round(decimals=2).tolist(),
                "hand_z": round(float(rb[hi[e], 2]), 4), "cube_z": round(float(rb[bi[e], 2]), 4),
                "ncf": {k: round(float(ncf[b].norm()), 2) for k, b in
                        (("cube", bi[e]), ("hand", hi[e]), ("fingerA", hi[e] + 1), ("fingerB", hi[e] + 2))},
                "contacts": nct, "anchors": nanc, "list": cl})
    z = rb[bi, 2]
    still = rb[bi, 7:10].norm(dim=1) < 0.05
    rel = rb[bi, 0:2] - rb[bi - 1, 0:2]
    overlap = (rel[:, 0].abs() < 0.3225) & (rel[:, 1].abs() < 0.5225)
    loose = ((z > 0.3) & (z < 0.4175) & still & ~overlap).nonzero().flatten().tolist()
    gym.destroy_sim(sim)
    run.runs = (best_run.cpu().numpy(), best_run_end.cpu().numpy())
    run.acts = {e: np.stack(a) for e, a in acts.items()}
    return worst.cpu().numpy(), worst_f.cpu().numpy(), loose, log


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    worst, wf, loose, _ = run(n, frames)
    order = np.argsort(-worst)
    summary = {"envs": n, "frames": frames,
               "deeper_than_contact_offset": int((worst > 0.001).sum()),
               "deeper_than_5mm": int((worst > 0.005).sum()),
               "depth_mm_quantiles": {q: round(1e3 * float(np.quantile(worst, q)), 3) for q in (0.5, 0.9, 0.99, 1.0)},
               "deepest": [(int(e), round(1e3 * float(worst[e]), 2), int(wf[e])) for e in order[:8]],
               "loose_cubes": loose}
    runs, run_end = run.runs
    by_run = np.argsort(-runs)
    summary["longest_runs_past_1mm"] = [(int(e), int(runs[e]), int(run_end[e])) for e in by_run[:8]]
    print(json.dumps(summary), flush=True)
    watch = [int(x) for x in sys.argv[3:]] or (loose[:3] + [int(order[0]), int(by_run[0])])
    around = {e: (int(wf[e]) if e not in loose else frames - 6) for e in watch}
    _, _, _, log = run(n, frames, watch, around, around_run=True)
    out = os.environ.get("DIAG_ACTIONS")
    if out:   # the watched envs' per-frame actions, for a CPU replay on the oracle
        np.savez_compressed(out, envs=np.array(watch), acts=np.stack([run.acts[e] for e in watch]))
    for e in watch:
        print(json.dumps({"env": e, "worst_depth_mm": round(1e3 * float(worst[e]), 3), "worst_frame": int(wf[e]),
                          "log": log[e]}), flush=True)


if __name__ == "__main__":
    main()
