"""Extract the contact-rest fixture from the reference's own Isaac Gym output.

Source: /root/reference/examples/graphics_images/, written by
examples/graphics.py:203-236 — 8 envs, eight 0.2 m / 0.5 kg balls per env
(assets/urdf/ball.urdf), ball 0 dropped from y = 6 onto the ground, the others
starting 5 cm above it; PhysX TGS 4/1, y-up defaults; images of frames 0, 30,
60, 90, 120 (the image of frame f follows the (f+1)-th simulate) from
  cam0: 360x240 at env-local (1.5, 1, 1.5) looking at the env origin, and
  cam1: 360x240 attached to ball 0 at (1, 0, -1), 135 degrees about y,
        FOLLOW_TRANSFORM.
Features per env and frame:
  cam0 depth (depth_env*_cam0_frame*.jpg, the reference's uint8 transform of
       the depth image): bounding box [top, bottom, left, right] and pixel
       count of the object mask (scenes.graphics_depth_ball_mask: pixels more
       than 12 grey levels off their row's ground median) — empty at frames
       0 / 30 (ball above the view), the falling ball at frame 60 and the
       ball resting on the ground at frames 90 / 120;
  cam1 color (rgb_env*_cam1_frame*.png): bounding box and count of the
       non-black pixels (the ball seen from below against the sky).
Run in the build container (the reference tree is not on the GPU box); the
JSON it writes is the committed fixture (tests/golden/graphics_fixture.json).
"""
import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from test_isaacgym_amd.scenes import graphics_depth_ball_mask  # noqa: E402

SRC = "/root/reference/examples/graphics_images"
OUT = os.path.join(HERE, "graphics_fixture.json")
FRAMES = [0, 30, 60, 90, 120]
ENVS = 8


def bbox(mask):
    ys, xs = np.nonzero(mask)
    if len(ys) == 0:
        return None, 0
    return [int(ys.min()), int(ys.max()), int(xs.min()), int(xs.max())], int(len(ys))


def main():
    if not os.path.isdir(SRC):
        sys.exit("reference images not found at %s" % SRC)
    out = {"source": "examples/graphics_images (Isaac Gym output of examples/graphics.py)",
           "frames": FRAMES, "envs": ENVS, "cam0_depth": {}, "cam1_color": {}}
    for f in FRAMES:
        for e in range(ENVS):
            d = np.array(Image.open(os.path.join(SRC, "depth_env%d_cam0_frame%d.jpg" % (e, f))))
            b, n = bbox(graphics_depth_ball_mask(d))
            out["cam0_depth"]["%d/%d" % (f, e)] = {"bbox": b, "count": n}
            c = np.array(Image.open(os.path.join(SRC, "rgb_env%d_cam1_frame%d.png" % (e, f))))
            b, n = bbox(c[..., :3].max(-1) > 6)
            out["cam1_color"]["%d/%d" % (f, e)] = {"bbox": b, "count": n}
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
