"""Contact rest pinned to the reference's own output:
examples/graphics_images/ are Isaac Gym's camera images of examples/graphics.py
— eight 0.2 m balls per env under PhysX TGS 4/1, ball 0 dropped from y = 6 —
and tests/golden/graphics_fixture.json holds features extracted from them
(tests/golden/make_graphics_fixture.py).

What they pin:
  * cam0 depth, frames 90 and 120: ball 0 resting on the ground, seen from
    (1.5, 1, 1.5) — its silhouette rows / columns pin the rest height (1 px is
    about 8 mm at 1.4 m), and the identical images at 90 and 120 pin that the
    ball landed without bouncing back up and stays at rest (restitution 0,
    sphere-plane contact, TGS);
  * cam0 depth, frame 60: the ball in flight (gravity, frame cadence), and
    frames 0 / 30: the ball above the view;
  * cam1 color, every frame: the camera attached to the ball
    (FOLLOW_TRANSFORM) sees the ball at the image centre, identically before,
    during and after the landing: no rolling, and the attachment / camera-axis
    convention (a y-up camera looks along its local -z).
Tolerances: +-1 px on every bounding box (at frame 60 the ball falls ~30 px per
frame, so this pins the fall to ~1/30 of a frame; at rest 1 px is ~8 mm of
height); pixel counts within 12 % (the lower rim of the resting ball has the
ground's depth, and the fixture is a JPEG).
The CPU test runs the C restatement (physics + renderer); the GPU test runs the
device path and also checks it bit for bit against the restatement.
"""
import json
import os

import numpy as np
import pytest

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import _render, scenes
import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "graphics_fixture.json")
FRAMES = [0, 30, 60, 90, 120]


def _fixture():
    with open(GOLD) as f:
        return json.load(f)


def _bbox(mask):
    ys, xs = np.nonzero(mask)
    if len(ys) == 0:
        return None, 0
    return [int(ys.min()), int(ys.max()), int(xs.min()), int(xs.max())], int(len(ys))


def _check(fx, f, e, depth0, rgba1):
    ref0 = fx["cam0_depth"]["%d/%d" % (f, e)]
    b0, n0 = _bbox(scenes.graphics_depth_ball_mask(scenes.graphics_depth_u8(depth0)))
    if ref0["bbox"] is None:
        assert n0 == 0, "frame %d env %d: ball visible to cam0 (%s)" % (f, e, b0)
    else:
        assert b0 is not None, "frame %d env %d: ball not visible to cam0" % (f, e)
        assert np.abs(np.array(b0) - ref0["bbox"]).max() <= 1, \
            "frame %d env %d: cam0 ball %s vs Isaac Gym %s" % (f, e, b0, ref0["bbox"])
        assert abs(n0 - ref0["count"]) <= 0.12 * ref0["count"], (f, e, n0, ref0["count"])
    ref1 = fx["cam1_color"]["%d/%d" % (f, e)]
    b1, n1 = _bbox(rgba1[..., :3].max(-1) > 6)
    assert b1 is not None and np.abs(np.array(b1) - ref1["bbox"]).max() <= 1, \
        "frame %d env %d: cam1 ball %s vs Isaac Gym %s" % (f, e, b1, ref1["bbox"])
    assert abs(n1 - ref1["count"]) <= 0.08 * ref1["count"], (f, e, n1, ref1["count"])
    return b0, b1


def _oracle_image(sim, state, cam):
    A = sim.model_arrays
    first, color, seg = _render.body_render_arrays(sim)
    rec = _render.camera_record(sim, cam)
    return oracle.render(sim.mg_params(), state, A["body_tmpl"], A["tmpl_body_i"], A["shapes"], first, color, seg,
                         rec, hulls=A["hulls"])


def test_oracle_rest_matches_isaac_gym_graphics_images(gym):
    fx = _fixture()
    sim, envs, cams = scenes.graphics_scene(gym, 2, use_gpu_pipeline=False)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    seen = {}
    for f in range(FRAMES[-1] + 1):
        oracle.step(p, m, st, dof)           # the image of frame f follows the (f+1)-th simulate
        if f in FRAMES:
            for e in range(2):
                _, depth0, _ = _oracle_image(sim, st, envs[e].cameras[cams[e][0]])
                rgba1, _, _ = _oracle_image(sim, st, envs[e].cameras[cams[e][1]])
                seen[(f, e)] = _check(fx, f, e, depth0, rgba1)
    # at rest: the frame-90 and frame-120 silhouettes agree
    assert seen[(90, 0)] == seen[(120, 0)]
    # the resting ball: centre 0.2 m (+ rest offset) above the ground, still
    balls = st.reshape(2, 8, 13)
    assert np.all(np.abs(balls[:, :, 1] - 0.2) < 0.005), balls[:, :, 1]
    assert np.all(np.abs(balls[:, :, 7:13]) < 0.02)


@pytest.mark.gpu
def test_gpu_rest_matches_isaac_gym_graphics_images(gym):
    fx = _fixture()
    n = 8
    sim, envs, cams = scenes.graphics_scene(gym, n)
    imgs = []
    for e in range(n):
        d0 = gymtorch.wrap_tensor(gym.get_camera_image_gpu_tensor(sim, envs[e], cams[e][0], gymapi.IMAGE_DEPTH))
        c1 = gymtorch.wrap_tensor(gym.get_camera_image_gpu_tensor(sim, envs[e], cams[e][1], gymapi.IMAGE_COLOR))
        imgs.append((d0, c1))
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    A = sim.model_arrays
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    for f in range(FRAMES[-1] + 1):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.render_all_camera_sensors(sim)
        oracle.step(p, m, st, dof)
        if f in FRAMES:
            got = rb.cpu().numpy()
            assert np.array_equal(got, st), "frame %d: max |gpu - oracle| %g" % (f, np.abs(got - st).max())
            for e in range(n):
                d0, c1 = imgs[e][0].cpu().numpy(), imgs[e][1].cpu().numpy()
                _, o_d0, _ = _oracle_image(sim, got, envs[e].cameras[cams[e][0]])
                o_c1, _, _ = _oracle_image(sim, got, envs[e].cameras[cams[e][1]])
                assert np.array_equal(d0.view(np.int32), o_d0.view(np.int32)), "frame %d env %d: depth" % (f, e)
                assert np.array_equal(c1, o_c1), "frame %d env %d: color" % (f, e)
                _check(fx, f, e, d0, c1)
