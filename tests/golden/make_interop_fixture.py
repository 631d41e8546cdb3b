"""Extract the camera-render fixture from the reference's own Isaac Gym output.

Source: /root/reference/examples/interop_images/cam-<frame>-<env>.png, written by
examples/interop_torch.py:173-190 (16 envs, a sphere of radius 0.5 dropped from
y = 5 under y-up gravity -9.8, restitution 0.9, camera 128x128 at env-local
(5, 1, 0) looking at (0, 1, 0), default 90-degree horizontal field of view;
the image of frame f is written after the (f+1)-th simulate). Run in the build
container (the reference tree is not on the GPU box); the JSON it writes is the
committed fixture (tests/golden/interop_fixture.json). Features per image:
  ball  : bounding box [top, bottom, left, right] and pixel count of the lit
          pixels above the horizon (rows < 64; the sky is black there), and the
          number of lit blobs above the horizon (1 = no neighbouring env drawn);
  ground: for frame 0, env 0, the checker class of every pixel of rows 70..127
          (1 = light square, 0 = dark), as a hex string of packed bits.
"""
import json
import os
import sys

import numpy as np
from PIL import Image

SRC = "/root/reference/examples/interop_images"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "interop_fixture.json")
FRAMES = [0, 10, 20, 30, 40, 50]
ENVS = 16


def blobs(mask):
    """4-connected components of a boolean mask (small images)."""
    seen = np.zeros_like(mask, dtype=bool)
    n = 0
    for y, x in zip(*np.nonzero(mask)):
        if seen[y, x]:
            continue
        n += 1
        stack = [(y, x)]
        seen[y, x] = True
        while stack:
            cy, cx = stack.pop()
            for dy, dx in ((1, 0), (-1, 0), (0, 1), (0, -1)):
                yy, xx = cy + dy, cx + dx
                if 0 <= yy < mask.shape[0] and 0 <= xx < mask.shape[1] and mask[yy, xx] and not seen[yy, xx]:
                    seen[yy, xx] = True
                    stack.append((yy, xx))
    return n


def main():
    if not os.path.isdir(SRC):
        sys.exit("reference images not found at %s" % SRC)
    out = {"source": "examples/interop_images (Isaac Gym output of examples/interop_torch.py)",
           "frames": FRAMES, "envs": ENVS, "horizon_row": 64, "ball": {}}
    for f in FRAMES:
        for e in range(ENVS):
            im = np.array(Image.open(os.path.join(SRC, "cam-%04d-%04d.png" % (f, e))))
            lit = im[..., :3].max(-1) > 6
            lit[64:] = False
            ys, xs = np.nonzero(lit)
            rec = {"count": int(len(ys)), "blobs": blobs(lit)}
            if len(ys):
                rec["bbox"] = [int(ys.min()), int(ys.max()), int(xs.min()), int(xs.max())]
            out["ball"]["%d/%d" % (f, e)] = rec
    im = np.array(Image.open(os.path.join(SRC, "cam-0000-0000.png"))).astype(int)
    cls = (im[70:128, :, 0] > 125).astype(np.uint8)
    out["ground_rows"] = [70, 128]
    out["ground_light_bits"] = np.packbits(cls.reshape(-1)).tobytes().hex()
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
