"""Diagnostic: the S3 pick loop (tests/test_franka_gpu.py::test_franka_pick_lifts_cubes)
with a per-frame record of every cube's height and speed; prints, for each env
whose cube ends at rest inside the table, the frame it went below the table top
and its trajectory around it (cube z, vz, hand z, finger DOFs, contact force).
Usage: python tools/diag_sunk.py [n] [frames]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from isaacgym import gymapi, gymtorch  # noqa: E402
from test_franka_gpu import _setup, _control  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    gym = gymapi.acquire_gym()
    sim, info, rb, dof, jac, mm, ctl = _setup(gym, n)
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    bi = torch.tensor(info["box_idxs"], device="cuda:0")
    hi = torch.tensor(info["hand_idxs"], device="cuda:0")
    Z, V, H, F, C, XY = [], [], [], [], [], []
    for f in range(frames):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        _control(gym, sim, info, rb, dof, jac, mm, ctl, n)
        gym.refresh_net_contact_force_tensor(sim)
        Z.append(rb[bi, 2].cpu().numpy())
        V.append(rb[bi, 7:10].norm(dim=1).cpu().numpy())
        H.append(rb[hi, 2].cpu().numpy())
        F.append(dof[:, 0].view(n, 9)[:, 7:9].sum(1).cpu().numpy())
        C.append(ncf[bi, 2].cpu().numpy())
        XY.append((rb[bi, 0:2] - rb[bi - 1, 0:2]).cpu().numpy())   # relative to the table (body box - 1)
    Z, V, H, F, C, XY = map(np.stack, (Z, V, H, F, C, XY))
    over = (np.abs(XY[-1, :, 0]) < 0.3 - 0.0225) & (np.abs(XY[-1, :, 1]) < 0.5 - 0.0225)
    low = (Z[-1] > 0.3) & (Z[-1] < 0.4225 - 0.005) & (V[-1] < 0.05)
    print("at rest below the table top: %d, of which over the table (sunk): %d" % (low.sum(), (low & over).sum()))
    sunk = np.where(low)[0]
    print("sunk envs:", sunk.tolist())
    for e in sunk[:6]:
        below = np.where(Z[:, e] < 0.4225 - 0.005)[0]
        f0 = int(below[0]) if len(below) else frames - 1
        print("env %d: below the top from frame %d; cube x, y from the table centre at the end %s (table half extents 0.3, 0.5)"
              % (e, f0, XY[-1, e].tolist()))
        for f in range(max(0, f0 - 12), min(frames, f0 + 6)):
            print("  f%3d cube z %.4f |v| %.3f  hand z %.4f  fingers %.4f  cf_z %.2f"
                  % (f, Z[f, e], V[f, e], H[f, e], F[f, e], C[f, e]))


if __name__ == "__main__":
    main()
