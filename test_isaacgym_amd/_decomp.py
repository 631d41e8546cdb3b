"""Approximate convex decomposition of a collision mesh (AssetOptions.vhacd_enabled,
gymapi.VhacdParams): the importer's counterpart of PhysX cooking a concave mesh
into several convex hulls instead of one.

The solid the triangle mesh encloses is voxelised (voxel centres classified by
the parity of +x ray crossings, column by column), then split recursively: the
piece whose convex hull exceeds its voxel volume the most (its concavity) is cut
by the axis-aligned plane, among a few candidates per axis, that minimises the
two halves' summed hull volume, until every piece is convex within
`concavity` (relative) or `max_convex_hulls` pieces exist. Each piece becomes the
convex hull of its voxels' corner points (an outer approximation by at most one
voxel), reduced to MG_HULL_MAX_VERTS vertices like any collision mesh.
"""
import heapq

import numpy as np


def mesh_triangles(path):
    """(vertices (n, 3), triangles (m, 3) int) of an OBJ or STL file, or None
    for another format (such a mesh is taken as a single hull)."""
    import os
    ext = os.path.splitext(path)[1].lower()
    if ext == ".obj":
        vs, fs = [], []
        with open(path, "r", errors="ignore") as f:
            for line in f:
                if line.startswith("v "):
                    p = line.split()
                    vs.append([float(p[1]), float(p[2]), float(p[3])])
                elif line.startswith("f "):
                    idx = []
                    for tok in line.split()[1:]:
                        k = int(tok.split("/")[0])
                        idx.append(k - 1 if k > 0 else len(vs) + k)
                    for j in range(1, len(idx) - 1):     # fan
                        fs.append([idx[0], idx[j], idx[j + 1]])
        return np.array(vs, dtype=np.float64).reshape(-1, 3), np.array(fs, dtype=np.int64).reshape(-1, 3)
    if ext == ".stl":
        from ._assets import _mesh_vertices
        v = _mesh_vertices(path)
        m = len(v) // 3
        return v[:3 * m], np.arange(3 * m, dtype=np.int64).reshape(m, 3)
    return None


def voxelize(verts, tris, resolution):
    """Boolean occupancy (nx, ny, nz), grid origin and voxel size: voxel centres
    inside the closed triangle mesh by the parity of +x ray crossings."""
    lo, hi = verts.min(0), verts.max(0)
    ext = np.maximum(hi - lo, 1e-9)
    h = float((np.prod(ext) / max(resolution, 8)) ** (1.0 / 3.0))
    n = np.maximum(np.ceil(ext / h).astype(int), 1)
    lo = lo - 0.5 * (n * h - ext)
    occ = np.zeros(n, dtype=bool)
    a, b, c = verts[tris[:, 0]], verts[tris[:, 1]], verts[tris[:, 2]]
    ys = lo[1] + (np.arange(n[1]) + 0.5) * h
    zs = lo[2] + (np.arange(n[2]) + 0.5) * h
    xs = lo[0] + (np.arange(n[0]) + 0.5) * h
    # per triangle, its (y, z) projection; a column (y, z) crosses it where the
    # 2-D barycentric coordinates are inside (half-open edges against double counts)
    d = (b[:, 1] - a[:, 1]) * (c[:, 2] - a[:, 2]) - (c[:, 1] - a[:, 1]) * (b[:, 2] - a[:, 2])
    ok = np.abs(d) > 1e-18
    a, b, c, d = a[ok], b[ok], c[ok], d[ok]
    for j, y in enumerate(ys):
        for k, z in enumerate(zs):
            w1 = ((b[:, 1] - y) * (c[:, 2] - z) - (c[:, 1] - y) * (b[:, 2] - z)) / d
            w2 = ((c[:, 1] - y) * (a[:, 2] - z) - (a[:, 1] - y) * (c[:, 2] - z)) / d
            w3 = 1.0 - w1 - w2
            hit = (w1 >= 0) & (w2 >= 0) & (w3 > 0)
            if not hit.any():
                continue
            xc = np.sort(w1[hit] * a[hit, 0] + w2[hit] * b[hit, 0] + w3[hit] * c[hit, 0])
            # inside where an odd number of crossings lies left of the centre
            cnt = np.searchsorted(xc, xs)
            occ[:, j, k] = (cnt % 2) == 1
    return occ, lo, h


def _corners(cells, lo, h):
    off = np.array([[i, j, k] for i in (0, 1) for j in (0, 1) for k in (0, 1)], dtype=np.float64)
    return (lo + (cells[:, None, :] + off[None]) * h).reshape(-1, 3)


def _extreme_cells(cells):
    """The cells that are first or last along some axis-parallel line through the
    set: their corners span the same convex hull as all cells' corners."""
    keep = np.zeros(len(cells), dtype=bool)
    for ax in range(3):
        o1, o2 = [a for a in range(3) if a != ax]
        key = cells[:, o1] * 4096 + cells[:, o2]
        order = np.lexsort((cells[:, ax], key))
        k = key[order]
        first = np.ones(len(k), dtype=bool)
        first[1:] = k[1:] != k[:-1]
        last = np.ones(len(k), dtype=bool)
        last[:-1] = k[:-1] != k[1:]
        keep[order[first | last]] = True
    return cells[keep]


def _hull_volume(cells, lo, h):
    from scipy.spatial import ConvexHull
    pts = np.unique(_corners(_extreme_cells(cells), lo, h), axis=0)
    try:
        return float(ConvexHull(pts).volume)
    except Exception:
        return len(cells) * h ** 3


def decompose(verts, tris, max_convex_hulls=64, resolution=100000, concavity=0.0, min_volume_per_ch=0.0,
              candidates=12):
    """Point sets (one (k, 3) array per convex piece) whose hulls approximate the
    solid; a single piece when the mesh is convex within the tolerance."""
    res = int(min(max(resolution, 512), 32 ** 3))        # bounded: pure-numpy voxeliser
    occ, lo, h = voxelize(np.asarray(verts, np.float64), np.asarray(tris, np.int64), res)
    cells = np.argwhere(occ)
    if len(cells) < 8:
        return [np.asarray(verts, np.float64)]
    tol = concavity if concavity > 0.0 else 0.02
    vmin = max(min_volume_per_ch, 0.0)

    def score(cs):
        hv = _hull_volume(cs, lo, h)
        return (hv - len(cs) * h ** 3) / max(hv, 1e-30), hv

    pieces = []           # max-heap on concavity: (-concavity, id, cells, hull volume)
    c0, hv0 = score(cells)
    heapq.heappush(pieces, (-c0, 0, cells, hv0))
    uid = 1
    while len(pieces) < max(max_convex_hulls, 1):
        negc, _, cs, hv = pieces[0]
        if -negc <= tol or len(cs) < 16 or hv <= vmin:
            break
        best = None
        for ax in range(3):
            vals = cs[:, ax]
            lo_i, hi_i = int(vals.min()), int(vals.max())
            if hi_i <= lo_i:
                continue
            cand = np.arange(lo_i + 1, hi_i + 1)
            if len(cand) > candidates:
                cand = np.unique(np.linspace(lo_i + 1, hi_i, candidates).astype(int))
            for t in cand:
                left = cs[vals < t]
                right = cs[vals >= t]
                if len(left) == 0 or len(right) == 0:
                    continue
                tot = _hull_volume(left, lo, h) + _hull_volume(right, lo, h)
                if best is None or tot < best[0]:
                    best = (tot, left, right)
        if best is None:
            break
        heapq.heappop(pieces)
        for part in (best[1], best[2]):
            cp, hp = score(part)
            heapq.heappush(pieces, (-cp, uid, part, hp))
            uid += 1
    return [_corners(_extreme_cells(p[2]), lo, h) for p in sorted(pieces, key=lambda p: p[1])]
