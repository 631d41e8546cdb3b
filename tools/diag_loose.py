"""Diagnostic: the S3 pick loop at 4096 envs (tests/test_franka_gpu.py::
test_franka_pick_lifts_cubes) with, for every cube that ends at rest below the
table top beside the table, its last frames: cube z / |v| / net contact force,
both fingers' distance to the cube and net contact force, the hand height.
Usage: python tools/diag_loose.py [n] [frames]"""
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
    rec = []
    for f in range(frames):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        _control(gym, sim, info, rb, dof, jac, mm, ctl, n)
        gym.refresh_net_contact_force_tensor(sim)
        if f >= frames - 40:
            c = rb[bi, 0:3]
            rec.append(torch.stack([rb[bi, 2], rb[bi, 7:10].norm(dim=1), ncf[bi].norm(dim=1),
                                    (rb[hi + 1, 0:3] - c).norm(dim=1), ncf[hi + 1].norm(dim=1),
                                    (rb[hi + 2, 0:3] - c).norm(dim=1), ncf[hi + 2].norm(dim=1), rb[hi, 2],
                                    dof[:, 0].view(n, 9)[:, 7] + dof[:, 0].view(n, 9)[:, 8]], 1).cpu().numpy())
    R = np.stack(rec)
    z, v = R[-1, :, 0], R[-1, :, 1]
    rel = (rb[bi, 0:2] - rb[bi - 1, 0:2]).cpu().numpy()
    over = (np.abs(rel[:, 0]) < 0.3225) & (np.abs(rel[:, 1]) < 0.5225)
    low = (z > 0.3) & (z < 0.4175) & (v < 0.05) & ~over
    print("at rest below the top beside the table:", np.where(low)[0].tolist())
    for e in np.where(low)[0][:4]:
        print("env %d rel %s" % (e, rel[e].tolist()))
        print("  f   cube_z   |v|    ncf    dA     ncfA    dB     ncfB   hand_z  fingers")
        for k in range(0, 40, 2):
            print("  %2d " % k + " ".join("%7.4f" % x for x in R[k, e]))


if __name__ == "__main__":
    main()
