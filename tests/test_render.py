"""Camera sensors (config 5): the device ray caster
(csrc/mg_render.hip) against its C restatement (oracle/migym_oracle_render.c),
and both against the reference's own rendered output.

Pinning. examples/interop_images/ holds Isaac Gym's camera images of
examples/interop_torch.py (16 envs, a ball dropped from y = 5, a 128x128 camera
at (5, 1, 0) looking at (0, 1, 0)); tests/golden/interop_fixture.json holds
features extracted from them (tests/golden/make_interop_fixture.py). They pin
the camera placement, the projection (90-degree default FOV, square pixels,
principal point at the centre: the ball's silhouette at frame 0 matches to the
pixel), the 1 m ground checker and its phase, that a camera shows only its own
env (no neighbouring ball although envs are 4 m apart), and — through the
ball's height over frames 0..50 — gravity and frame cadence to +-1 px (our
semi-implicit Euler leaves the ball up to 1 px higher from frame 10 on, about
3-4 cm at 5 m; PhysX's integrator is unpinned). Shading values
(light direction, ball colour) are not pinned.

Device vs restatement: the same fp32 expressions in the same order, FMA
contraction off on both sides, so color, depth and segmentation images are
compared bit for bit.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import _render, scenes
import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "interop_fixture.json")
FRAMES = [0, 10, 20, 30, 40, 50]
DEV = "cuda:0"


def _fixture():
    with open(GOLD) as f:
        return json.load(f)


def _oracle_image(sim, state, cam):
    A = sim.model_arrays
    first, color, seg = _render.body_render_arrays(sim)
    rec = _render.camera_record(sim, cam)
    return oracle.render(sim.mg_params(), state, A["body_tmpl"], A["tmpl_body_i"], A["shapes"], first, color, seg,
                         rec, hulls=A["hulls"], light=sim.light)


def _ball_features(rgba):
    lit = rgba[..., :3].max(-1) > 6
    lit[64:] = False
    ys, xs = np.nonzero(lit)
    return [int(ys.min()), int(ys.max()), int(xs.min()), int(xs.max())], len(ys), lit


def _blobs(mask):
    seen = np.zeros_like(mask)
    n = 0
    for y, x in zip(*np.nonzero(mask)):
        if seen[y, x]:
            continue
        n += 1
        stack = [(y, x)]
        seen[y, x] = True
        while stack:
            cy, cx = stack.pop()
            for yy, xx in ((cy + 1, cx), (cy - 1, cx), (cy, cx + 1), (cy, cx - 1)):
                if 0 <= yy < mask.shape[0] and 0 <= xx < mask.shape[1] and mask[yy, xx] and not seen[yy, xx]:
                    seen[yy, xx] = True
                    stack.append((yy, xx))
    return n


def _check_against_fixture(fx, f, e, rgba):
    ref = fx["ball"]["%d/%d" % (f, e)]
    bbox, count, lit = _ball_features(rgba)
    assert _blobs(lit) == ref["blobs"] == 1, "frame %d env %d: a neighbouring env is visible" % (f, e)
    assert np.abs(np.array(bbox) - np.array(ref["bbox"])).max() <= 1, \
        "frame %d env %d: ball bbox %s vs Isaac Gym %s" % (f, e, bbox, ref["bbox"])
    assert abs(count - ref["count"]) <= 0.12 * ref["count"]


def test_oracle_render_matches_isaac_gym_fixture(gym):
    """The restatement (physics + camera) on interop_torch.py's scene vs Isaac
    Gym's own images, on the CPU."""
    fx = _fixture()
    sim, envs, _ = scenes.interop_scene(gym, 16)
    A = sim.build_model()
    p, m = sim.mg_params(), sim.mg_model()
    st = A["body_state0"].copy()
    dof = np.zeros((0, 2), np.float32)
    for f in range(FRAMES[-1] + 1):
        oracle.step(p, m, st, dof)        # the image of frame f follows the (f+1)-th simulate
        if f in FRAMES:
            for e in (0, 5, 15):
                rgba, depth, seg = _oracle_image(sim, st, envs[e].cameras[0])
                _check_against_fixture(fx, f, e, rgba)
                if f == 0 and e == 0:
                    r0, r1 = fx["ground_rows"]
                    cls = (rgba[r0:r1, :, 0] > 125).astype(np.uint8)
                    bits = np.unpackbits(np.frombuffer(bytes.fromhex(fx["ground_light_bits"]), np.uint8))
                    ref = bits[:cls.size].reshape(cls.shape)
                    # checker squares agree except at square edges and the ball's shadow
                    assert (cls == ref).mean() >= 0.97
                    # depth of the ground at the bottom row centre: 1 m ahead (camera 1 m up, 45 deg down)
                    assert depth[127, 64] == pytest.approx(-1.0 / (63.5 / 64.0), rel=1e-5)
                    assert np.isfinite(depth[:64]).sum() == (rgba[:64, :, :3].max(-1) > 0).sum()


def test_camera_intrinsics_and_look_at(gym):
    props = gymapi.CameraProperties()
    props.width, props.height, props.horizontal_fov = 1600, 900, 30.0
    fx, fy, cx, cy = _render.intrinsics(props)
    assert fx == fy == pytest.approx(800.0 / math.tan(math.radians(15.0)))
    assert (cx, cy) == (800.0, 450.0)
    # y-up: the camera's view axis is its local -z (examples/graphics_images cam1);
    # looking down -x, image right = -z (examples/interop_images checker phase)
    t = _render.look_at(gymapi.Vec3(5, 1, 0), gymapi.Vec3(0, 1, 0), gymapi.UP_AXIS_Y)
    f = t.r.rotate(gymapi.Vec3(0, 0, -1))
    up = t.r.rotate(gymapi.Vec3(0, 1, 0))
    right = t.r.rotate(gymapi.Vec3(1, 0, 0))
    assert (right.x, right.y, right.z) == pytest.approx((0, 0, -1), abs=1e-6)
    assert (f.x, f.y, f.z) == pytest.approx((-1, 0, 0), abs=1e-6)
    assert (up.x, up.y, up.z) == pytest.approx((0, 1, 0), abs=1e-6)
    # z-up: no roll, local z stays up
    t = _render.look_at(gymapi.Vec3(0, 0, 10), gymapi.Vec3(10, 5, 0), gymapi.UP_AXIS_Z)
    f = t.r.rotate(gymapi.Vec3(1, 0, 0))
    l = t.r.rotate(gymapi.Vec3(0, 1, 0))
    d = np.array([10, 5, -10.0]) / 15.0
    assert (f.x, f.y, f.z) == pytest.approx(tuple(d), abs=1e-6)
    assert l.z == pytest.approx(0.0, abs=1e-6)


# --------------------------------------------------------------------- GPU
def _gpu_images(gym, sim, env, cam):
    return [gymtorch.wrap_tensor(gym.get_camera_image_gpu_tensor(sim, env, cam, k))
            for k in (gymapi.IMAGE_COLOR, gymapi.IMAGE_DEPTH, gymapi.IMAGE_SEGMENTATION)]


def _assert_same(sim, rb, env, cam, imgs, what):
    rgba, depth, seg = _oracle_image(sim, rb, env.cameras[cam])
    g_rgba, g_depth, g_seg = [t.cpu().numpy() for t in imgs]
    assert np.array_equal(g_rgba, rgba), "%s: color differs in %d px" % (what, int((g_rgba != rgba).any(-1).sum()))
    assert np.array_equal(g_seg, seg), "%s: segmentation differs" % what
    assert np.array_equal(g_depth.view(np.int32), depth.view(np.int32)), \
        "%s: depth differs (max %g)" % (what, float(np.nanmax(np.abs(g_depth - depth))))


@pytest.mark.gpu
def test_render_interop_gpu_bitexact_and_fixture(gym):
    fx = _fixture()
    sim, envs, cams = scenes.interop_scene(gym, 16, colors=[(0.5 + 0.03 * i, 0.6, 0.9 - 0.02 * i) for i in range(16)])
    imgs = [_gpu_images(gym, sim, envs[i], cams[i]) for i in range(16)]
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    for f in range(FRAMES[-1] + 1):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.render_all_camera_sensors(sim)
        gym.start_access_image_tensors(sim)
        if f in FRAMES:
            st = rb.cpu().numpy()
            for e in range(16):
                _assert_same(sim, st, envs[e], cams[e], imgs[e], "frame %d env %d" % (f, e))
                _check_against_fixture(fx, f, e, imgs[e][0].cpu().numpy())
        gym.end_access_image_tensors(sim)


def _servo_with_cameras(gym, n, w, h):
    sim, envs = scenes.servo_scene(gym, n)
    for i, env in enumerate(envs):
        gym.set_rigid_body_segmentation_id(env, 1, 0, 7)          # the vehicle
        gym.set_rigid_body_color(env, 1, 0, gymapi.MESH_VISUAL_AND_COLLISION, gymapi.Vec3(0.9, 0.4, 0.1))
    tens = scenes.attach_servo_cameras(gym, sim, envs, w, h, 30.0,
                                       (gymapi.IMAGE_COLOR, gymapi.IMAGE_DEPTH, gymapi.IMAGE_SEGMENTATION))
    return sim, envs, tens


@pytest.mark.gpu
def test_render_servo_cameras_gpu_bitexact(gym):
    """test11's camera on the UAV (local (5, 0, 0), FOLLOW_TRANSFORM) at 160x90,
    64 envs: half the UAVs pitched down at their vehicle, half at random
    orientations; color / depth / segmentation bit-exact against the oracle."""
    n = 64
    sim, envs, tens = _servo_with_cameras(gym, n, 160, 90)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    acts = scenes.servo_actions(n, 4, DEV, seed=3)
    down = gymapi.Quat.from_euler_zyx(0.0, math.atan2(100.0, 10.0), 0.0)
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(4):
        root[:, 3:10] = acts[k]
        root[0:n:2, 3:7] = torch.tensor([down.x, down.y, down.z, down.w], device=DEV)
        root[0:n:2, 7:13] = 0.0
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_actor_root_state_tensor(sim)
        gym.render_all_camera_sensors(sim)
    st = rb.cpu().numpy()
    seen = 0
    for e in range(n):
        _assert_same(sim, st, envs[e], 0, tens[e], "servo env %d" % e)
        seen += int((tens[e][2] == 7).any())
    assert seen >= n // 2 - 2, "the pitched-down cameras should see their vehicle (%d did)" % seen


@pytest.mark.gpu
def test_get_camera_image_shows_the_render_snapshot(gym, tmp_path):
    """test11 calls set_actor_root_state_tensor between render_all_camera_sensors
    and get_camera_image (:388,456,459): the image is the rendered snapshot."""
    n = 4
    sim, envs = scenes.servo_scene(gym, n, use_gpu_pipeline=False)
    props = gymapi.CameraProperties()
    props.width, props.height = 64, 36
    for env in envs:
        cam = gym.create_camera_sensor(env, props)
        body = gym.get_actor_rigid_body_handle(env, 0, 0)
        local = gymapi.Transform()
        local.p = gymapi.Vec3(5, 0, 0)
        gym.attach_camera_to_body(cam, env, body, local, gymapi.FOLLOW_TRANSFORM)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    assert root.device.type == "cpu"
    down = gymapi.Quat.from_euler_zyx(0.0, 1.4, 0.0)
    root[0::2, 3:7] = torch.tensor([down.x, down.y, down.z, down.w])
    gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
    gym.simulate(sim)
    gym.fetch_results(sim, True)
    gym.render_all_camera_sensors(sim)
    before = [gym.get_camera_image(sim, envs[i], 0, gymapi.IMAGE_COLOR) for i in range(n)]
    assert before[0].shape == (36, 64 * 4) and before[0].dtype == np.uint8
    assert (before[0].reshape(36, 64, 4)[..., :3] > 0).any()           # looking at the ground
    gym.refresh_actor_root_state_tensor(sim)
    root[0::2, 3:7] = torch.tensor([0.0, 0.0, 0.0, 1.0])                # level: horizon view
    gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
    again = [gym.get_camera_image(sim, envs[i], 0, gymapi.IMAGE_COLOR) for i in range(n)]
    for a, b in zip(before, again):
        assert np.array_equal(a, b)
    gym.simulate(sim)
    gym.render_all_camera_sensors(sim)
    after = gym.get_camera_image(sim, envs[0], 0, gymapi.IMAGE_COLOR)
    assert not np.array_equal(after, before[0])
    d = gym.get_camera_image(sim, envs[0], 0, gymapi.IMAGE_DEPTH)
    assert d.dtype == np.float32 and np.isneginf(d[0]).all()           # top row: sky
    # write_camera_image_to_file (domain_randomization.py:192): the same render as PNG
    from PIL import Image
    fc, fd = str(tmp_path / "rgb.png"), str(tmp_path / "depth.png")
    assert gym.write_camera_image_to_file(sim, envs[0], 0, gymapi.IMAGE_COLOR, fc)
    assert gym.write_camera_image_to_file(sim, envs[0], 0, gymapi.IMAGE_DEPTH, fd)
    assert np.array_equal(np.asarray(Image.open(fc)).reshape(36, 64 * 4), after)
    mm = np.asarray(Image.open(fd)).astype(np.int64)
    hit = np.isfinite(d)
    want = np.clip(np.rint(-d[hit].astype(np.float64) * 1000.0), 0, 65535)     # 16-bit: clipped at 65.535 m
    assert (mm[~hit] == 0).all() and np.abs(mm[hit] - want).max() <= 1


@pytest.mark.gpu
def test_render_shapes_and_many_bodies_gpu_bitexact(gym):
    """Boxes, spheres and capsules at random poses (z-up), a fixed camera per
    env, plus the Franka cube-pick scene (13 bodies, ~14 boxes per env) seen by
    a fixed camera: exercises every intersection routine, box normals,
    shadows between bodies and the row culling with many shapes."""
    sp = scenes.servo_sim_params()
    sp.gravity = gymapi.Vec3(0, 0, -9.8)
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    assets = [gym.create_box(sim, 0.4, 0.3, 0.2), gym.create_sphere(sim, 0.25), gym.create_capsule(sim, 0.15, 0.3)]
    rng = np.random.RandomState(7)
    envs = []
    imgs = []
    for i in range(6):
        env = gym.create_env(sim, gymapi.Vec3(-2, -2, 0), gymapi.Vec3(2, 2, 2), 3)
        envs.append(env)
        for j in range(6):
            pose = gymapi.Transform()
            pose.p = gymapi.Vec3(*(rng.uniform(-0.8, 0.8, 2).tolist() + [rng.uniform(0.3, 1.5)]))
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            pose.r = gymapi.Quat(*q)
            h = gym.create_actor(env, assets[j % 3], pose, "s%d" % j, i, -1, j + 1)   # no body-body contacts
            gym.set_rigid_body_color(env, h, 0, gymapi.MESH_VISUAL_AND_COLLISION, gymapi.Vec3(*rng.uniform(0.2, 1, 3)))
        cp = gymapi.CameraProperties()
        cp.width, cp.height = 96 + 4 * i, 72 - 2 * i          # odd sizes: the scalar store path
        cam = gym.create_camera_sensor(env, cp)
        gym.set_camera_location(cam, env, gymapi.Vec3(2.5, 1.5, 1.8), gymapi.Vec3(0, 0, 0.6))
        imgs.append(_gpu_images(gym, sim, env, cam))
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    for f in range(3):
        gym.simulate(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    gym.render_all_camera_sensors(sim)
    st = rb.cpu().numpy()
    for i, env in enumerate(envs):
        _assert_same(sim, st, env, 0, imgs[i], "shapes env %d" % i)
        assert len(np.unique(imgs[i][2].cpu().numpy())) >= 4      # several bodies in view
    gym.destroy_sim(sim)

    sim, info = scenes.franka_scene(gym, 8)
    envs = info["envs"]
    imgs = []
    for env in envs:
        cp = gymapi.CameraProperties()
        cp.width, cp.height = 128, 96
        cam = gym.create_camera_sensor(env, cp)
        gym.set_camera_location(cam, env, gymapi.Vec3(1.6, 1.0, 1.2), gymapi.Vec3(0.3, 0.0, 0.5))
        imgs.append(_gpu_images(gym, sim, env, cam))
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    gym.simulate(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    gym.render_all_camera_sensors(sim)
    st = rb.cpu().numpy()
    for i, env in enumerate(envs):
        _assert_same(sim, st, env, 0, imgs[i], "franka env %d" % i)
        assert np.isfinite(imgs[i][1].cpu().numpy()).mean() > 0.3


@pytest.mark.gpu
def test_render_config5_full_size_sampled_bitexact(gym):
    """Config 5 at full size (test11_servo_vecenv_camerazoom.py:327-335): 1024
    envs, one 1600x900 camera per env on the UAV (FOLLOW_TRANSFORM), 12 frames of
    the bench's S1 step with random teleports and render_all_camera_sensors every
    frame; 6 sampled cameras are compared bit for bit (color, depth, segmentation)
    against the restatement, and the images must show the scene (not only sky)."""
    n, w, h = 1024, 1600, 900
    sim, envs = scenes.servo_scene(gym, n)
    imgs = scenes.attach_servo_cameras(gym, sim, envs, w, h, 30.0,
                                       image_types=(gymapi.IMAGE_COLOR, gymapi.IMAGE_DEPTH, gymapi.IMAGE_SEGMENTATION))
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    acts = scenes.servo_actions(n, 12, DEV, seed=5)
    gym.refresh_actor_root_state_tensor(sim)
    for k in range(12):
        root[:, 3:10] = acts[k]
        gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.render_all_camera_sensors(sim)
    torch.cuda.synchronize()
    st = rb.cpu().numpy()
    lit = []
    for e in (0, 1, 257, 511, 768, 1023):
        _assert_same(sim, st, envs[e], 0, [t for t in imgs[e]], "config5 env %d" % e)
        lit.append(float((imgs[e][0][..., :3].amax(-1) > 0).float().mean()))
    assert max(lit) > 0.05, lit
    gym.destroy_sim(sim)


@pytest.mark.gpu
def test_light_parameters_gpu_bitexact(gym):
    """gym.set_light_parameters (examples/domain_randomization.py:186): a
    coloured, dimmer light from the side changes the bodies' shading and the
    shadows' direction (the checker's colours are fixed), bit for bit the
    oracle renderer with the same light;
    set_light_parameters before prepare_sim applies at prepare."""
    n = 8
    sim, envs, tens = _servo_with_cameras(gym, n, 96, 54)
    gym.set_light_parameters(sim, 0, gymapi.Vec3(0.9, 0.5, 0.2), gymapi.Vec3(0.1, 0.15, 0.2),
                             gymapi.Vec3(1.0, -0.5, 0.4))
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    down = gymapi.Quat.from_euler_zyx(0.0, math.atan2(100.0, 10.0), 0.0)
    gym.refresh_actor_root_state_tensor(sim)
    root[0::2, 3:7] = torch.tensor([down.x, down.y, down.z, down.w], device=DEV)
    root[:, 7:13] = 0.0
    assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
    gym.simulate(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    gym.render_all_camera_sensors(sim)
    st = rb.cpu().numpy()
    lit = [t[0].cpu().numpy().copy() for t in tens]
    for e in range(n):
        _assert_same(sim, st, envs[e], 0, tens[e], "lit env %d" % e)
    # the default light again: the bodies' shading changes (and the shadows move)
    gym.set_light_parameters(sim, 0, gymapi.Vec3(0.7, 0.7, 0.7), gymapi.Vec3(0.3, 0.3, 0.3),
                             gymapi.Vec3(0.3, 0.2, 1.0))
    gym.render_all_camera_sensors(sim)
    body_px = 0
    for e in range(n):
        seg = tens[e][2].cpu().numpy()
        now = tens[e][0].cpu().numpy()
        _assert_same(sim, st, envs[e], 0, tens[e], "default env %d" % e)
        ground = seg == 0
        body_px += int((~ground).sum())
        if (~ground).any():
            assert not np.array_equal(now[~ground], lit[e][~ground])
    assert body_px > 0


@pytest.mark.gpu
def test_destroy_camera_sensor_gpu(gym):
    """destroy_camera_sensor: the camera is no longer rendered (its image
    tensor keeps the last render) and can no longer be read; the env's other
    camera keeps its handle and is still rendered bit for bit."""
    n = 2
    sim, envs = scenes.servo_scene(gym, n)
    props = gymapi.CameraProperties()
    props.width, props.height = 48, 27
    cams = []
    for env in envs:
        pair = []
        for k in range(2):
            c = gym.create_camera_sensor(env, props)
            local = gymapi.Transform()
            local.p = gymapi.Vec3(5, 0, 0)
            gym.attach_camera_to_body(c, env, gym.get_actor_rigid_body_handle(env, 0, 0), local,
                                      gymapi.FOLLOW_TRANSFORM)
            pair.append(c)
        cams.append(pair)
    imgs = [[gymtorch.wrap_tensor(gym.get_camera_image_gpu_tensor(sim, envs[e], c, gymapi.IMAGE_COLOR))
             for c in cams[e]] for e in range(n)]
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    gym.simulate(sim)
    gym.render_all_camera_sensors(sim)
    first = imgs[0][1].clone()
    gym.destroy_camera_sensor(sim, envs[0], cams[0][1])
    gym.refresh_actor_root_state_tensor(sim)
    down = gymapi.Quat.from_euler_zyx(0.0, 1.4, 0.0)
    root[:, 3:7] = torch.tensor([down.x, down.y, down.z, down.w], device=DEV)
    assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
    gym.simulate(sim)
    gym.refresh_rigid_body_state_tensor(sim)
    gym.render_all_camera_sensors(sim)
    assert torch.equal(imgs[0][1], first)                    # not rendered again
    assert not torch.equal(imgs[0][0], first)                 # its sibling is
    with pytest.raises(ValueError):
        gym.get_camera_image(sim, envs[0], cams[0][1], gymapi.IMAGE_COLOR)
    st = rb.cpu().numpy()
    rgba, _, _ = _oracle_image(sim, st, envs[0].cameras[cams[0][0]])
    assert np.array_equal(imgs[0][0].cpu().numpy(), rgba)
