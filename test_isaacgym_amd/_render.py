"""Camera sensors over the device ray caster (csrc/mg_render.hip).

Reference call sites: create_camera_sensor / attach_camera_to_body /
render_all_camera_sensors / get_camera_image (test11_servo_vecenv_camerazoom.py:
327-342,388,458-460), set_camera_location / get_camera_image_gpu_tensor
(examples/interop_torch.py:105-120,173-174).

Semantics kept from Isaac Gym:
  * render_all_camera_sensors renders what the cameras see *at that call*: the
    body poses are snapshotted on the device then, and every image fetched
    afterwards (get_camera_image, or the GPU tensors) shows that snapshot, even
    after set_actor_root_state_tensor (test11 sets roots between the render and
    get_camera_image, :456-460);
  * cameras with a GPU tensor (get_camera_image_gpu_tensor) are rendered in one
    batched launch at render_all_camera_sensors; the others are rendered on
    demand by get_camera_image, so test11's 90 cameras per env cost only the
    one it reads each frame;
  * images: color (H, W*4) uint8 RGBA from get_camera_image, (H, W, 4) as a
    GPU tensor; depth (H, W) float32 = -distance along the view axis, -inf on
    no hit; segmentation (H, W) int32.
Projection (pinned by examples/interop_images/, tests/test_render.py): square
pixels, fx = fy = (W / 2) / tan(horizontal_fov / 2), principal point at the
image centre. Camera axes (local): in a z-up sim the camera looks along +x with
+z as image up; in a y-up sim along -z with +y up (pinned by
examples/graphics_images/*_cam1_*: a camera attached to a ball at offset
(1, 0, -1) rotated 135 degrees about y sees that ball at the image centre).
"""
import ctypes
import math

import numpy as np
import torch

from . import _native as N
from . import _types as T

IMAGE_KINDS = (T.IMAGE_COLOR, T.IMAGE_DEPTH, T.IMAGE_SEGMENTATION)


def intrinsics(props):
    w, h = int(props.width), int(props.height)
    fx = (0.5 * w) / math.tan(math.radians(float(props.horizontal_fov)) * 0.5)
    return fx, fx, 0.5 * w, 0.5 * h


def look_at(pos, target, up_axis):
    """Camera transform at `pos` looking at `target` (gym.set_camera_location):
    the local view axis (+x z-up, -z y-up) -> the view direction, the local up
    axis -> as close to world up as the view allows (no roll)."""
    f = np.array([target.x - pos.x, target.y - pos.y, target.z - pos.z], dtype=np.float64)
    f /= max(np.linalg.norm(f), 1e-12)
    up = np.array([0.0, 0.0, 1.0]) if up_axis == T.UP_AXIS_Z else np.array([0.0, 1.0, 0.0])
    l = np.cross(up, f)
    if np.linalg.norm(l) < 1e-9:          # looking straight up / down
        l = np.cross(np.array([1.0, 0.0, 0.0]) if abs(f[0]) < 0.9 else np.array([0.0, 1.0, 0.0]), f)
    l /= np.linalg.norm(l)
    u = np.cross(f, l)
    if up_axis == T.UP_AXIS_Z:
        F0, L0, U0 = np.eye(3)
    else:
        F0, L0, U0 = np.array([0, 0, -1.0]), np.array([-1.0, 0, 0]), np.array([0, 1.0, 0])
    R = np.outer(f, F0) + np.outer(l, L0) + np.outer(u, U0)
    return T.Transform(T.Vec3(pos.x, pos.y, pos.z), _quat_from_matrix(R))


def _quat_from_matrix(R):
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = math.sqrt(tr + 1.0) * 2
        w, x, y, z = 0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        w, x, y, z = (R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        w, x, y, z = (R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        w, x, y, z = (R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s
    n = math.sqrt(x * x + y * y + z * z + w * w)
    return T.Quat(x / n, y / n, z / n, w / n)


def body_render_arrays(sim):
    """env_body_first [num_envs+1], color [nb, 3], seg [nb] (host), from
    set_rigid_body_color / set_rigid_body_segmentation_id / create_actor's
    segmentationId."""
    sim._assign_indices()
    first = np.zeros(len(sim.envs) + 1, dtype=np.int32)
    color = np.ones((sim.num_bodies, 3), dtype=np.float32)
    seg = np.zeros(sim.num_bodies, dtype=np.int32)
    b = 0
    for i, e in enumerate(sim.envs):
        first[i] = b
        for a in e.actors:
            for k in range(a.num_bodies):
                c = a.body_colors.get(k)
                if c is not None:
                    color[b + k] = [c.x, c.y, c.z]
                seg[b + k] = a.body_segs.get(k, a.segmentation_id)
            b += a.num_bodies
    first[len(sim.envs)] = b
    return first, color, seg


def camera_record(sim, cam, images=None):
    """mg_camera of a CameraSensor; images: {IMAGE_*: device tensor}."""
    c = N.MgCamera()
    p = cam.props
    c.env = cam.env.index
    c.width, c.height = int(p.width), int(p.height)
    c.fx, c.fy, c.cx, c.cy = intrinsics(p)
    c.near_plane, c.far_plane = float(p.near_plane), float(p.far_plane)
    if cam.body is not None:
        a = _body_actor(cam.env, cam.body)
        c.body = a.global_body + (cam.body - a.body_offset)
        c.follow = int(cam.follow)
        t = cam.local
    else:
        c.body = -1
        c.follow = 0
        o = cam.env.origin
        t = T.Transform(T.Vec3(cam.transform.p.x + o[0], cam.transform.p.y + o[1], cam.transform.p.z + o[2]),
                        cam.transform.r)
    c.p[:] = [t.p.x, t.p.y, t.p.z]
    c.q[:] = [t.r.x, t.r.y, t.r.z, t.r.w]
    images = images or {}
    c.color = images[T.IMAGE_COLOR].data_ptr() if T.IMAGE_COLOR in images else None
    c.depth = images[T.IMAGE_DEPTH].data_ptr() if T.IMAGE_DEPTH in images else None
    c.seg = images[T.IMAGE_SEGMENTATION].data_ptr() if T.IMAGE_SEGMENTATION in images else None
    return c


def _body_actor(env, body):
    for a in env.actors:
        if a.body_offset <= body < a.body_offset + a.num_bodies:
            return a
    raise ValueError("camera attached to body %d, which env %d does not have" % (body, env.index))


def image_tensor(sim, cam, kind):
    """The persistent device image of one camera (get_camera_image_gpu_tensor)."""
    t = cam.images.get(kind)
    if t is None:
        h, w = int(cam.props.height), int(cam.props.width)
        dev = torch.device("cuda", sim.compute_device)
        if kind == T.IMAGE_COLOR:
            t = torch.zeros((h, w, 4), dtype=torch.uint8, device=dev)
        elif kind == T.IMAGE_SEGMENTATION:
            t = torch.zeros((h, w), dtype=torch.int32, device=dev)
        else:
            t = torch.full((h, w), -math.inf, dtype=torch.float32, device=dev)
        cam.images[kind] = t
        sim.cam_version += 1
    return t


class Renderer:
    """Per-sim render state: the uploaded body table, the snapshot, the batched
    camera table of the tensor cameras."""

    def __init__(self, sim):
        self.sim = sim
        self.bodies_key = None
        self.snap = False
        self.frame = 0
        self.batch = None          # (ctypes array, count, key) of the tensor cameras

    def _ensure_bodies(self):
        sim = self.sim
        if self.bodies_key == sim.render_version:
            return
        first, color, seg = body_render_arrays(sim)
        N.check(N.lib.mg_set_render_bodies(sim.native, first.ctypes.data, color.ctypes.data, seg.ctypes.data),
                "mg_set_render_bodies")
        self.bodies_key = sim.render_version

    def render_all(self):
        sim = self.sim
        if sim.cam_version == 0:
            return True                     # no camera was ever created
        h = sim.require_native("render_all_camera_sensors")
        self._ensure_bodies()
        st = sim.stream()
        N.check(N.lib.mg_snapshot_render_state(h, st), "render_all_camera_sensors")
        self.snap = True
        self.frame += 1
        if self.batch is None or self.batch[2] != sim.cam_version:
            tcams = [c for e in sim.envs for c in e.cameras if c.images and not c.destroyed]
            arr = (N.MgCamera * max(len(tcams), 1))(*[camera_record(sim, c, c.images) for c in tcams])
            self.batch = (arr, len(tcams), sim.cam_version)
        if self.batch[1]:
            N.check(N.lib.mg_render_cameras(h, self.batch[0], self.batch[1], st), "render_all_camera_sensors")
        return True

    def image(self, cam, kind):
        """get_camera_image: host numpy image of the last render_all snapshot."""
        sim = self.sim
        h = sim.require_native("get_camera_image")
        self._ensure_bodies()
        st = sim.stream()
        if not self.snap:
            N.check(N.lib.mg_snapshot_render_state(h, st), "get_camera_image")
            self.snap = True
        t = cam.images.get(kind)
        if t is None:
            tmp = {}
            hh, ww = int(cam.props.height), int(cam.props.width)
            dev = torch.device("cuda", sim.compute_device)
            if kind == T.IMAGE_COLOR:
                tmp[kind] = torch.empty((hh, ww, 4), dtype=torch.uint8, device=dev)
            elif kind == T.IMAGE_SEGMENTATION:
                tmp[kind] = torch.empty((hh, ww), dtype=torch.int32, device=dev)
            else:
                tmp[kind] = torch.empty((hh, ww), dtype=torch.float32, device=dev)
            rec = camera_record(sim, cam, tmp)
            N.check(N.lib.mg_render_cameras(h, ctypes.byref(rec), 1, st), "get_camera_image")
            t = tmp[kind]
        out = t.cpu().numpy()
        if kind == T.IMAGE_COLOR:
            return out.reshape(out.shape[0], -1)
        return out

