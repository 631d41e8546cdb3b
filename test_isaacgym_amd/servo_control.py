"""GPU-resident servo controller: torch-batched restatement of the reference's
host controller so a test10-style loop never leaves the device (SURVEY.md §8f
rank 4, row a9).

Reference functions (same math, same conventions; no numpy / scipy, any device
and dtype):
  cclvf2            common/controller6.py:92-118 (circular-loiter vector field)
  euler2quaternion  common/controller6.py:46-51  (scipy 'xyz' extrinsic -> xyzw)
  quat_to_matrix    scipy Rotation.from_quat(q).as_matrix()
  CameraController  common/controller6.py:122-253 (pinhole world -> pixel)
  SecondaryControl  common/secondary_control_vecenv.py:8-200 (pixel error ->
                    gimbal roll / pitch / yaw, degrees)
Pinned by tests/golden/controller_golden.npz (outputs of the reference code).
"""
import math

import torch


def cclvf2(current_pos, target_pos, speed, radius):
    """common/controller6.py:92-118. (N,3) positions -> (N,3) velocity command."""
    x_ = current_pos[:, 0] - target_pos[:, 0]
    y_ = current_pos[:, 1] - target_pos[:, 1]
    z_ = current_pos[:, 2] - target_pos[:, 2]
    r = torch.norm(current_pos[:, :2] - target_pos[:, :2], dim=1)
    r = torch.clamp(r, min=0.01)
    rd = radius
    c_ = torch.where(r < rd, r / rd, rd / r)
    r_rd_ = r * r - rd * rd
    factor = speed / torch.sqrt(r ** 4 + (c_ ** 2 - 2) * rd ** 2 * r ** 2 + rd ** 4)
    vx = -factor * (x_ * r_rd_ / r + c_ * rd * y_)
    vy = -factor * (y_ * r_rd_ / r - c_ * rd * x_)
    return torch.stack((vx, vy, -z_), dim=1)


def euler2quaternion(euler):
    """scipy Rotation.from_euler('xyz', e).as_quat(): extrinsic x, y, z -> (x, y, z, w),
    the product q_z q_y q_x of the elementary half-angle quaternions (scipy's sign)."""
    r, p, y = euler[:, 0], euler[:, 1], euler[:, 2]
    cr, sr = torch.cos(0.5 * r), torch.sin(0.5 * r)
    cp, sp = torch.cos(0.5 * p), torch.sin(0.5 * p)
    cy, sy = torch.cos(0.5 * y), torch.sin(0.5 * y)
    return torch.stack([sr * cp * cy - cr * sp * sy,
                        cr * sp * cy + sr * cp * sy,
                        cr * cp * sy - sr * sp * cy,
                        cr * cp * cy + sr * sp * sy], dim=1)


def quat_to_matrix(q):
    """(N,4) xyzw (normalised here, as scipy does) -> (N,3,3) rotation matrices."""
    q = q / torch.norm(q, dim=1, keepdim=True)
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        torch.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        torch.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], dim=1)


def euler_xyz_to_matrix(e):
    """scipy Rotation.from_euler('xyz', e).as_matrix()."""
    return quat_to_matrix(euler2quaternion(e))


def rotvec_to_matrix(rv):
    """scipy Rotation.from_rotvec(rv).as_matrix() (Rodrigues)."""
    th = torch.norm(rv, dim=1)
    small = th < 1e-12
    ths = torch.where(small, torch.ones_like(th), th)
    k = rv / ths[:, None]
    kx, ky, kz = k[:, 0], k[:, 1], k[:, 2]
    zero = torch.zeros_like(kx)
    K = torch.stack([torch.stack([zero, -kz, ky], -1), torch.stack([kz, zero, -kx], -1),
                     torch.stack([-ky, kx, zero], -1)], dim=1)
    s, c = torch.sin(th)[:, None, None], torch.cos(th)[:, None, None]
    eye = torch.eye(3, dtype=rv.dtype, device=rv.device).expand_as(K)
    Rm = eye + s * K + (1 - c) * (K @ K)
    return torch.where(small[:, None, None], eye, Rm)


class CameraController:
    """common/controller6.py:122-253: pinhole projection of the ground target into
    the UAV camera, batched over envs. focal length = zoom * 18 mm on a 36 mm
    sensor, principal point at the image centre."""

    def __init__(self, width, height, device="cpu", dtype=torch.float64):
        self.width = float(width)
        self.height = float(height)
        self.device = device
        self.dtype = dtype
        self.set_zoom(1)

    def set_zoom(self, zoom):
        alpha = self.width / (36 * 0.001)
        fx = alpha * (zoom * 18) * 0.001
        self.camera_matrix = torch.tensor([[fx, 0.0, self.width / 2], [0.0, fx, self.height / 2], [0.0, 0.0, 1.0]],
                                          dtype=self.dtype, device=self.device)

    def world2pixel(self, uav_pos, car_pos, uav_matrix):
        """(N,3), (N,3), (N,3,3) -> (N,3) homogeneous pixel [u, v, 1]."""
        pos_uav = (car_pos - uav_pos)[:, :, None]                      # rot_uav2world = I
        pos_cam = torch.linalg.solve(uav_matrix, pos_uav)             # inv(uav_matrix) @ p
        rot = torch.tensor([[0.0, -1.0, 0.0], [0.0, 0.0, -1.0], [1.0, 0.0, 0.0]], dtype=self.dtype,
                           device=uav_pos.device)
        pos_cam = rot @ pos_cam
        z = torch.clamp(pos_cam[:, 2:3], min=1e-7)
        pos_cam = torch.cat([pos_cam[:, :2], z], dim=1)
        normalized = pos_cam / pos_cam[:, 2:3]
        return (self.camera_matrix.to(uav_pos.device) @ normalized).squeeze(-1)


class SecondaryControl:
    """common/secondary_control_vecenv.py:8-200: gimbal angles (degrees) that
    move the image point `pixel_move` away from the centre."""

    _ROT = ((0.0, 0.0, 1.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0))

    def __init__(self, width=1280, height=760):
        self.width = float(width)
        self.height = float(height)

    def pixel2phy(self, pixel, camera_matrix):
        n = pixel.shape[0]
        p = torch.ones((n, 3), dtype=pixel.dtype, device=pixel.device)
        p[:, :2] = pixel
        a = torch.linalg.solve(camera_matrix.expand(n, 3, 3) if camera_matrix.dim() == 2 else camera_matrix,
                               p[:, :, None])
        rot = torch.tensor(self._ROT, dtype=pixel.dtype, device=pixel.device)
        return rot @ a / torch.norm(a, dim=1)[:, None]

    def servo_ext_pixel(self, camera_matrix, cam_matrix, pixel_move):
        """(3,3) or (N,3,3) intrinsics, (N,3,3) camera attitude, (N,2) pixel move
        -> (N,3) [roll, pitch, yaw] in degrees."""
        dt, dev = pixel_move.dtype, pixel_move.device
        n = pixel_move.shape[0]
        centre = torch.tensor([self.width / 2, self.height / 2], dtype=dt, device=dev)
        target_pixel = pixel_move + centre
        centre_pixel = centre.expand(n, 2)
        cm = camera_matrix.to(dtype=dt, device=dev)
        u_move = self.pixel2phy(target_pixel, cm)          # (N,3,1)
        u_target = self.pixel2phy(centre_pixel, cm)
        u_pos_move = cam_matrix @ u_move
        servo = torch.zeros((n, 3), dtype=dt, device=dev)
        servo[:, 1] = torch.arcsin(u_target[:, 2, 0]) - torch.arcsin(u_pos_move[:, 2, 0])
        on_yaw = u_pos_move[:, :, 0].clone()
        on_yaw[:, 2] = 0
        on_yaw = on_yaw / torch.norm(on_yaw, dim=1, keepdim=True)
        servo[:, 2] = torch.where(on_yaw[:, 1] > 0, torch.arccos(on_yaw[:, 0]), -torch.arccos(on_yaw[:, 0]))
        init_on_yaw = u_move[:, :, 0].clone()
        init_on_yaw[:, 2] = 0
        init_on_yaw = init_on_yaw / torch.norm(init_on_yaw, dim=1, keepdim=True)
        coord_yaw = torch.where(init_on_yaw[:, 1] > 0, torch.arccos(init_on_yaw[:, 0]),
                                -torch.arccos(init_on_yaw[:, 0]))
        e_y = torch.tensor([0.0, 1.0, 0.0], dtype=dt, device=dev)
        e_z = torch.tensor([0.0, 0.0, 1.0], dtype=dt, device=dev)
        unit_y_init = cam_matrix @ e_y
        unit_z_init = cam_matrix @ e_z
        rot_yaw = rotvec_to_matrix(coord_yaw[:, None] * unit_z_init)
        move_view = (rot_yaw @ unit_y_init[:, :, None])[:, :, 0]
        rot_view = euler_xyz_to_matrix(servo) @ e_y
        cosr = torch.clamp((rot_view * move_view).sum(dim=1), -1, 1)
        roll = torch.arccos(cosr)
        servo[:, 0] = torch.where(move_view[:, 2] > 0, roll, -roll)
        return servo * (180.0 / math.pi)
