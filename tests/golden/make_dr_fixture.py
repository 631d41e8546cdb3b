"""Extract the ant-at-rest fixture from the reference's own Isaac Gym output.

Source: /root/reference/examples/dr_output_images/rgb_image_NNN_000.png, the 41
images examples/domain_randomization.py:139-197 writes with --save_images:
  - sim (:36-48): Isaac Gym defaults (y-up, gravity -9.8 y), dt 1/60, 2
    substeps, PhysX TGS 4/1, CPU pipeline; default ground plane (:60);
  - scene (:103-128): one env, assets/mjcf/nv_ant.xml at (0, 0.5, 0) rotated
    -90 degrees about x (quat (-0.707107, 0, 0, 0.707107)), every DOF
    DOF_MODE_NONE with zero stiffness and damping; a default camera sensor
    (1600 x 900, 90 degree horizontal FOV) attached to the torso and then
    placed by set_camera_location at (0, 3, 3) looking at (0, 0, -1);
  - loop (:139-197): image NNN is written at frame 100 (NNN + 1), rendered
    before that frame's randomisation, so image 000 shows the white ant from
    the initial camera and image NNN >= 1 the camera moved at frame 100 NNN to
    (0, 3 + y, 3 + z), y, z ~ U(-1, 1) from Python's unseeded `random`, with
    random body colours, textures and light.
The ant lands and settles in the first frames; every image shows it at rest.

Per image this script
  1. solves the camera offsets (y, z) from the checker ground: the 1 m checker
     (parity (floor x + floor z) & 1, the phase the graphics fixture pins) is
     projected through the candidate camera and correlated with the image's
     luminance over all ground pixels; a coarse grid then three refinements to
     0.5 mm (image 000 solves to (0, 0) within 0.5 mm: the camera model and the
     set_camera_location semantics — world frame, attachment dropped — hold);
  2. segments the ant: the ground's colour per parity is fitted by a smooth
     model outside the region the ant can cover, and a pixel is the ant when
     its colour is not a scaled copy of the ground's there (shadows are
     darkened ground: same chromaticity), or is brighter than lit ground;
     the largest connected component is kept;
  3. records the silhouette's bounding box and its four leg tips (the
     silhouette pixel farthest from the mask centroid in each quadrant around
     it), and quality measures; images whose mask fails the checks (area,
     symmetry, camera residual) are marked unusable.
Run in the build container (the reference tree is not on the GPU box); the
JSON it writes is the committed fixture (tests/golden/dr_fixture.json).
usage: make_dr_fixture.py [--debug DIR]
"""
import glob
import json
import os
import sys

import numpy as np
from PIL import Image
from scipy import ndimage

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/examples/dr_output_images"
OUT = os.path.join(HERE, "dr_fixture.json")
W, H = 1600, 900
FX = 800.0                       # (W / 2) / tan(90 deg / 2)
CAM_POS = np.array([0.0, 3.0, 3.0])
CAM_TGT = np.array([0.0, 0.0, -1.0])


def cam_basis(pos, tgt):
    """y-up look-at (test_isaacgym_amd/_render.py look_at): forward f, left l, up u."""
    f = tgt - pos
    f = f / np.linalg.norm(f)
    l = np.cross(np.array([0.0, 1.0, 0.0]), f)
    l = l / np.linalg.norm(l)
    return f, l, np.cross(f, l)


def pixel_rays(pos, tgt, cols, rows):
    """Ray directions of pixel centres (mg_render.hip: a = (cx - c - 1/2) / fx)."""
    f, l, u = cam_basis(pos, tgt)
    a = (W / 2 - cols - 0.5) / FX
    b = (H / 2 - rows - 0.5) / FX
    return f[None, :] + a[:, None] * l[None, :] + b[:, None] * u[None, :]


def ground_hits(pos, tgt, cols, rows):
    d = pixel_rays(pos, tgt, cols, rows)
    ok = d[:, 1] < -1e-6
    t = np.where(ok, -pos[1] / np.where(ok, d[:, 1], -1.0), 0.0)
    X = pos[0] + t * d[:, 0]
    Z = pos[2] + t * d[:, 2]
    par = (np.floor(X).astype(np.int64) + np.floor(Z).astype(np.int64)) & 1
    return par, ok, X, Z, t


def project(pos, tgt, P):
    """World points (n, 3) -> pixel (col, row) of the same camera model."""
    f, l, u = cam_basis(pos, tgt)
    d = P - pos[None, :]
    z = d @ f
    col = W / 2 - 0.5 - FX * (d @ l) / z
    row = H / 2 - 0.5 - FX * (d @ u) / z
    return np.stack([col, row], axis=1)


def solve_camera(Y):
    """Camera offsets (y, z) maximising the correlation of the projected checker
    parity (parity 0 light) with the luminance over the ground pixels."""
    rng = np.random.RandomState(0)
    n = 120000
    cols = rng.randint(0, W, n).astype(np.float64)
    rows = rng.randint(0, H, n).astype(np.float64)
    yv = Y[rows.astype(int), cols.astype(int)].astype(np.float64)
    full = (cols, rows, yv)
    sub = (cols[:12000], rows[:12000], yv[:12000])   # the coarse grid on a tenth of the samples

    def score(yo, zo):
        cols, rows, yv = samp
        pos = CAM_POS + np.array([0.0, yo, zo])
        par, ok, X, Z, t = ground_hits(pos, CAM_TGT, cols, rows)
        m = ok & (t < 12.0) & (np.hypot(X, Z) > 1.6)     # away from the ant
        p, v = par[m], yv[m]
        if p.sum() < 100 or (1 - p).sum() < 100:
            return -9.0
        return (v[p == 0].mean() - v[p == 1].mean()) / (v.std() + 1e-6)

    best = (-9.0, 0.0, 0.0)
    samp = sub
    for yo in np.linspace(-1.0, 1.0, 41):
        for zo in np.linspace(-1.0, 1.0, 41):
            s = score(yo, zo)
            if s > best[0]:
                best = (s, yo, zo)
    samp = full
    best = (score(best[1], best[2]), best[1], best[2])
    for step in (0.01, 0.002, 0.0005):
        _, y0, z0 = best
        for yo in y0 + step * np.arange(-5, 6):
            for zo in z0 + step * np.arange(-5, 6):
                s = score(yo, zo)
                if s > best[0]:
                    best = (s, yo, zo)
    return best


def ant_region(pos):
    """Pixels the ant (within 1.1 m of the origin, below 0.75 m) can cover: the
    bounding box of that cylinder's projection, padded."""
    ang = np.linspace(0, 2 * np.pi, 64, endpoint=False)
    P = np.concatenate([np.stack([1.1 * np.cos(ang), np.full_like(ang, y), 1.1 * np.sin(ang)], 1)
                        for y in (0.0, 0.75)])
    uv = project(pos, CAM_TGT, P)
    return (max(int(uv[:, 0].min()) - 10, 0), min(int(uv[:, 0].max()) + 10, W),
            max(int(uv[:, 1].min()) - 10, 0), min(int(uv[:, 1].max()) + 10, H))


def _basis(x, y):
    return np.stack([np.ones_like(x), x, y, x * x, x * y, y * y, x ** 3, x * x * y, x * y * y, y ** 3], -1)


def _seg_dist(c, a, b):
    """Distance of colours c from the segments [a, b] (all (..., 3))."""
    ab = b - a
    t = np.clip(((c - a) * ab).sum(-1) / np.maximum((ab * ab).sum(-1), 1e-6), 0.0, 1.0)
    return np.linalg.norm(c - (a + t[..., None] * ab), axis=-1)


def segment(img, pos):
    """Ant mask. The ground's colour of parity p lies between its shadow colour
    S_p (ambient light only: one colour over the whole plane) and its lit colour
    L_p(col, row) (a smooth fit: the light's falloff and highlight), the
    penumbra in between; a pixel farther than a threshold from that segment of
    its parity (from both, within 2 px of a square edge) is the ant. The largest
    connected component, holes filled."""
    rr, cc = np.mgrid[0:H, 0:W]
    par, ok, X, Z, t = ground_hits(pos, CAM_TGT, cc.ravel().astype(np.float64), rr.ravel().astype(np.float64))
    par, ok, X, Z = par.reshape(H, W), ok.reshape(H, W), X.reshape(H, W), Z.reshape(H, W)
    edge_d = np.minimum(np.abs(X - np.round(X)), np.abs(Z - np.round(Z)))
    c0, c1, r0, r1 = ant_region(pos)
    inside = np.zeros((H, W), bool)
    inside[r0:r1, c0:c1] = True
    band = np.zeros((H, W), bool)
    band[max(r0 - 200, 0):min(r1 + 200, H), max(c0 - 300, 0):min(c1 + 300, W)] = True
    xs, ys = (cc - W / 2) / W, (rr - H / 2) / H
    B = _basis(xs, ys)
    lit = np.zeros((H, W, 3))
    for p in (0, 1):
        m = band & ~inside & ok & (edge_d > 0.03) & (par == p)
        for _ in range(3):                   # robust: drop shadowed samples and refit
            coef = np.linalg.lstsq(B[m], img[m], rcond=None)[0]
            fitv = B[m] @ coef
            keep = (img[m] > 0.9 * fitv).all(-1)
            idx = np.nonzero(m)
            m2 = np.zeros_like(m)
            m2[idx[0][keep], idx[1][keep]] = True
            m = m2
        lit[par == p] = B[par == p] @ coef
    # shadow colour per parity: the most common colour darker than lit (in every
    # channel) near the ant
    shadow = []
    for p in (0, 1):
        m = band & ok & (edge_d > 0.03) & (par == p)
        c = img[m]
        dark = (c < 0.85 * lit[m]).all(-1)
        c = c[dark]
        if len(c) < 50:
            shadow.append(lit[m].mean(0) * 0.5)
            continue
        q = np.floor(c / 8.0).astype(np.int64)
        key = q[:, 0] * 1024 + q[:, 1] * 32 + q[:, 2]
        vals, cnt = np.unique(key, return_counts=True)
        mode = vals[np.argmax(cnt)]
        shadow.append(c[key == mode].mean(0))
    S = np.where((par == 0)[..., None], shadow[0], shadow[1])
    d = _seg_dist(img, S, lit) / np.maximum(np.linalg.norm(lit, axis=-1), 8.0)
    # near a square edge the pixel may show either parity
    Sx = np.where((par == 1)[..., None], shadow[0], shadow[1])
    litx = np.zeros_like(lit)
    for p in (0, 1):
        m = band & ok & (edge_d > 0.03) & (par == p)
    alt = 1 - par
    # the other parity's lit model: refit by swapping (cheap: evaluate both fits)
    d_alt = np.full((H, W), np.inf)
    near = edge_d < 0.02 * np.maximum(np.abs(Z - pos[2]), 1.0)
    if near.any():
        # use the neighbouring pixel's colours of the other parity as its model
        lit_o = ndimage.grey_dilation(np.where((par == 1)[..., None], lit, 0.0), size=(5, 5, 1)) * (par == 0)[..., None] + \
            ndimage.grey_dilation(np.where((par == 0)[..., None], lit, 0.0), size=(5, 5, 1)) * (par == 1)[..., None]
        d_alt = np.where(near, _seg_dist(img, Sx, lit_o) / np.maximum(np.linalg.norm(lit_o, axis=-1), 8.0), np.inf)
    dist = np.minimum(d, d_alt)
    ant = (dist > 0.12) & inside
    ant = ndimage.binary_opening(ant, iterations=2)
    ant = ndimage.binary_closing(ant, iterations=3)
    lab, n = ndimage.label(ant)
    if n == 0:
        return ant, 0.0
    sizes = ndimage.sum(ant, lab, range(1, n + 1))
    keep = ndimage.binary_fill_holes(lab == (1 + int(np.argmax(sizes))))
    fitm = band & ~inside & ok & (edge_d > 0.03)
    return keep, float(np.median(dist[fitm]))


def features(mask):
    """Bounding box [top, bottom, left, right] and the four leg tips (col, row):
    the silhouette pixel farthest from the mask centroid in each quadrant
    (upper-left, upper-right, lower-left, lower-right around the centroid)."""
    ys, xs = np.nonzero(mask)
    if len(ys) == 0:
        return None
    cy, cx = ys.mean(), xs.mean()
    tips = []
    for qy in (-1, 1):
        for qx in (-1, 1):
            s = ((ys - cy) * qy > 0) & ((xs - cx) * qx > 0)
            if not s.any():
                return None
            d2 = (ys[s] - cy) ** 2 + (xs[s] - cx) ** 2
            i = int(np.argmax(d2))
            tips.append([int(xs[s][i]), int(ys[s][i])])
    return {"bbox": [int(ys.min()), int(ys.max()), int(xs.min()), int(xs.max())], "tips": tips,
            "area": int(len(ys)), "centroid": [float(cx), float(cy)]}


FOOT_R = 0.08     # nv_ant.xml foot capsule radius: a resting foot's end sphere centre is 0.08 m up


def _backproject(pos, px, height):
    """Pixel (col, row) -> the point of its ray at world height y = `height`."""
    d = pixel_rays(pos, CAM_TGT, np.array([px[0]]), np.array([px[1]]))[0]
    t = (height - pos[1]) / d[1]
    return pos + t * d


def _tip_centre_px(pos, tip, centroid, C=None):
    """A tip is the silhouette point farthest from the centroid: the foot's end
    sphere centre lies one projected radius back along that direction."""
    u = np.array(tip, float) - np.array(centroid, float)
    u /= max(np.linalg.norm(u), 1e-9)
    if C is None:
        C = _backproject(pos, tip, FOOT_R)
    f, _, _ = cam_basis(pos, CAM_TGT)
    r_px = FX * FOOT_R / float((C - pos) @ f)
    return np.array(tip, float) - r_px * u, r_px, u


def consensus(out, tol=3.0):
    """Multi-view check of the extracted tips, independent of any simulation:
    the ant is at rest from frame 100 on, so each foot's end-sphere centre is
    one world point. Per image and foot it is back-projected onto y = 0.08 m
    (the feet rest on the ground), the per-foot median over images is the
    consensus centre, and an image is `usable` when its four measured tips lie
    within `tol` px of the consensus centres' predicted tips. The consensus
    centres are recorded too (`foot_centres`, world metres)."""
    imgs = out["images"]
    est = {k: [] for k in range(4)}
    for rec in imgs.values():
        if "tips" not in rec:
            continue
        pos = CAM_POS + np.array([0.0, *rec["cam_offset_yz"]])
        for k in range(4):
            c_px, _, _ = _tip_centre_px(pos, rec["tips"][k], rec["centroid"])
            est[k].append(_backproject(pos, c_px, FOOT_R))
    C = [np.median(np.array(est[k]), axis=0) for k in range(4)]
    for rec in imgs.values():
        rec["usable"] = False
        if "tips" not in rec:
            continue
        pos = CAM_POS + np.array([0.0, *rec["cam_offset_yz"]])
        errs = []
        for k in range(4):
            _, r_px, u = _tip_centre_px(pos, rec["tips"][k], rec["centroid"], C[k])
            pred = project(pos, CAM_TGT, C[k][None, :])[0] + r_px * u
            errs.append(float(np.abs(pred - np.array(rec["tips"][k])).max()))
        rec["consensus_err_px"] = [round(e, 2) for e in errs]
        rec["usable"] = bool(max(errs) <= tol)
    out["foot_centres"] = [[round(float(x), 5) for x in c] for c in C]
    out["usable_images"] = sorted(k for k, r in imgs.items() if r["usable"])


def process(path, debug=None):
    idx = int(os.path.basename(path).split("_")[2])
    img = np.asarray(Image.open(path).convert("RGB")).astype(np.float64)
    s, yo, zo = solve_camera(img.mean(-1))
    pos = CAM_POS + np.array([0.0, yo, zo])
    mask, fit_res = segment(img, pos)
    f = features(mask)
    rec = {"frame": 100 * (idx + 1), "cam_offset_yz": [round(float(yo), 4), round(float(zo), 4)],
           "cam_score": round(float(s), 4), "ground_fit_residual": round(fit_res, 4)}
    if f:
        rec.update(f)
    print(idx, rec.get("cam_offset_yz"), rec.get("cam_score"), rec.get("bbox"), rec.get("tips"), flush=True)
    if debug:
        os.makedirs(debug, exist_ok=True)
        o = img.copy()
        o[mask] = 0.5 * o[mask] + np.array([127.0, 0.0, 0.0])
        for c, r in (f["tips"] if f else []):
            o[max(r - 3, 0):r + 4, max(c - 3, 0):c + 4] = [0, 255, 0]
        Image.fromarray(o.astype(np.uint8)).save(os.path.join(debug, "m%03d.png" % idx))
    return idx, rec


def main():
    if not os.path.isdir(SRC):
        sys.exit("reference images not found at %s" % SRC)
    debug = sys.argv[sys.argv.index("--debug") + 1] if "--debug" in sys.argv else None
    out = {"source": "examples/dr_output_images (Isaac Gym output of examples/domain_randomization.py)",
           "image_size": [W, H], "hfov_deg": 90.0, "cam_pos": CAM_POS.tolist(), "cam_target": CAM_TGT.tolist(),
           "images": {}}
    paths = sorted(glob.glob(os.path.join(SRC, "rgb_image_*_000.png")))
    if os.environ.get("DR_ONLY"):
        only = {int(x) for x in os.environ["DR_ONLY"].split(",")}
        paths = [p for p in paths if int(os.path.basename(p).split("_")[2]) in only]
    import functools
    import multiprocessing
    with multiprocessing.Pool(min(6, os.cpu_count() or 1)) as pool:
        res = pool.map(functools.partial(process, debug=debug), paths)
    for idx, rec in sorted(res):
        out["images"]["%03d" % idx] = rec
    consensus(out)
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print("usable", out["usable_images"], "feet", out["foot_centres"])
    print("wrote", OUT)


if __name__ == "__main__":
    if "--consensus-only" in sys.argv:    # re-run step 3's check on the written fixture
        with open(OUT) as fh:
            o = json.load(fh)
        consensus(o)
        with open(OUT, "w") as fh:
            json.dump(o, fh, indent=1)
        print("usable", o["usable_images"], "feet", o["foot_centres"])
    else:
        main()
