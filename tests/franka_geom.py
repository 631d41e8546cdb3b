"""Geometry checks for the S3 Franka scene (tests/test_franka_gpu.py,
tools/diag_franka_env.py), in torch on the device: how deep the hand's and the
fingers' convex hulls reach into the table box, from the rigid-body state and
the model's shape / hull tables (_sim.py build_model: shape rows of
MG_SHAPE_STRIDE floats, hull records [nv, nf, ne, 0, verts(3 nv), ...])."""
import numpy as np
import torch


def _qmat(q):
    """(n, 4) xyzw -> (n, 3, 3) rotation matrices."""
    x, y, z, w = q.unbind(-1)
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        torch.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        torch.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)


def body_hull_points(A, body, dev):
    """Body-frame hull vertices of one body's convex shapes, (k, 3)."""
    t = int(A["body_tmpl"][body])
    s0, ns = int(A["tmpl_body_i"][t][0]), int(A["tmpl_body_i"][t][1])
    pts = []
    for s in range(s0, s0 + ns):
        sh = A["shapes"][s]
        if int(sh[0]) != 3:      # MG_SHAPE_CONVEX
            continue
        rec = A["hulls"][int(sh[2]):]
        nv = int(rec[0])
        v = rec[4:4 + 3 * nv].reshape(nv, 3).astype(np.float64)
        qs = torch.tensor(sh[7:11], dtype=torch.float64)[None]
        pts.append(torch.tensor(sh[4:7], dtype=torch.float64) + torch.from_numpy(v) @ _qmat(qs)[0].T)
    return torch.cat(pts).to(dev) if pts else torch.zeros((0, 3), dtype=torch.float64, device=dev)


def box_shape(A, body):
    """(half extents, local position, local quaternion) of a body's first shape (a box)."""
    t = int(A["body_tmpl"][body])
    sh = A["shapes"][int(A["tmpl_body_i"][t][0])]
    return sh[1:4].astype(np.float64), sh[4:7].astype(np.float64), sh[7:11].astype(np.float64)


def penetration_depth(A, rb, hull_bodies, table_bodies):
    """Depth (m, >= 0) of the deepest vertex of each env's hull bodies inside
    its table box: per env (rows of `hull_bodies`, (n, k) body indices, one
    hull template per column) the largest min-distance-to-the-faces of a
    vertex inside the box, 0 when none is inside. rb: (nb, 13) state."""
    dev = rb.device
    tb = table_bodies
    he, lp, lq = box_shape(A, int(tb[0]))
    he = torch.tensor(he, device=dev)
    st = rb.double()
    Rt = _qmat(st[tb, 3:7])                                          # (n, 3, 3)
    ct = st[tb, 0:3] + torch.einsum("nij,j->ni", Rt, torch.tensor(lp, device=dev))
    Rt = Rt @ _qmat(torch.tensor(lq, device=dev)[None])[0]
    depth = torch.zeros(len(tb), dtype=torch.float64, device=dev)
    for col in range(hull_bodies.shape[1]):
        bodies = hull_bodies[:, col]
        P = body_hull_points(A, int(bodies[0]), dev)                   # (k, 3) body frame
        if len(P) == 0:
            continue
        Rb = _qmat(st[bodies, 3:7])
        W = st[bodies, None, 0:3] + torch.einsum("nij,kj->nki", Rb, P)  # (n, k, 3) world
        L = torch.einsum("nji,nkj->nki", Rt, W - ct[:, None, :])       # table frame
        d = (he[None, None, :] - L.abs()).min(-1).values               # > 0 inside
        depth = torch.maximum(depth, d.clamp(min=0.0).max(-1).values)
    return depth
