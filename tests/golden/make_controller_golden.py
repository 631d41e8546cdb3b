"""Generates tests/golden/controller_golden.npz from the reference's host
controller (run in the build container, where /root/reference exists; the
fixture, not this script, travels to the GPU box).

Reference functions evaluated:
  common/controller6.py:92-118   cclvf2 (torch)
  common/controller6.py:46-51    euler2quaternion (scipy 'xyz' -> xyzw)
  common/controller6.py:163-253  CameraController.set_params / world2pixel
  common/secondary_control_vecenv.py:99-200  SecondaryControl.servo_ext_pixel
on seeded inputs shaped like test10_servo_vecenv.py:403-447 (N envs, 1600x900
camera). controller6 imports `isaacgym.gymapi` without using it; this repo's
isaacgym package satisfies that import.

Run: python tests/golden/make_controller_golden.py
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

from scipy.spatial.transform import Rotation as R  # noqa: E402


class _CamProps:
    width = 1600
    height = 900


def main():
    from common.controller6 import CameraController, cclvf2, euler2quaternion  # noqa: E402
    from common.secondary_control_vecenv import SecondaryControl  # noqa: E402

    rng = np.random.RandomState(42)
    n = 64
    car_pos = np.stack([rng.uniform(-80, 80, n), rng.uniform(-80, 80, n), rng.uniform(0.5, 3.0, n)], 1)
    uav_pos = np.stack([car_pos[:, 0] + rng.uniform(-60, 60, n), car_pos[:, 1] + rng.uniform(-60, 60, n),
                        rng.uniform(80, 300, n)], 1)
    # attitude: the servo-law output of test10 is roll/pitch/yaw; sample moderate angles
    uav_euler = np.stack([rng.uniform(-0.6, 0.6, n), rng.uniform(-0.6, 0.6, n), rng.uniform(-np.pi, np.pi, n)], 1)
    uav_quat = R.from_euler("xyz", uav_euler).as_quat()
    uav_matrix = R.from_quat(uav_quat).as_matrix()

    out = {}
    with contextlib.redirect_stdout(io.StringIO()):
        # cclvf2 as test10 calls it (:406, :414)
        cp = torch.tensor(car_pos, dtype=torch.float64)
        out["car_vel"] = cclvf2(cp, torch.ones_like(cp), speed=50, radius=30).numpy()
        tgt = cp.clone()
        tgt[:, 2] = 260
        up = torch.tensor(uav_pos, dtype=torch.float64)
        out["uav_vel"] = cclvf2(up, tgt, speed=50, radius=50).numpy()
        # the r < radius branch and the r -> 0.01 floor
        near = torch.tensor(np.stack([rng.uniform(-5, 5, n), rng.uniform(-5, 5, n), rng.uniform(0, 3, n)], 1))
        near[0, :2] = 1.0
        out["near_vel"] = cclvf2(near, torch.ones_like(near), speed=10, radius=10).numpy()
        # euler2quaternion (:410, :447)
        eul = np.stack([rng.uniform(-np.pi, np.pi, n), rng.uniform(-np.pi / 2, np.pi / 2, n),
                        rng.uniform(-np.pi, np.pi, n)], 1)
        out["euler"] = eul
        out["euler_quat"] = np.asarray(euler2quaternion(eul))
        # world2pixel (:427-429)
        cam = CameraController(_CamProps(), n)
        cam.set_params(np.zeros(3), np.zeros((n, 3)), uav_pos, car_pos, uav_matrix, np.eye(4), np.eye(4), 1)
        out["camera_matrix"] = np.asarray(cam.camera_matrix)
        out["pixel"] = np.asarray(cam.world2pixel())[:, :2]
        # servo_ext_pixel (:432-436)
        sc = SecondaryControl(_CamProps.width, _CamProps.height, n)
        move = np.array([_CamProps.width / 2.0, _CamProps.height / 2.0]) - out["pixel"]
        out["pixel_move"] = move
        out["servo_deg"] = np.asarray(sc.servo_ext_pixel(cam.camera_matrix, uav_matrix, move)).reshape(-1, 3)
        # the reference's own __main__ known answer (secondary_control_vecenv.py:203-231)
        sc2 = SecondaryControl(1600, 900, 2)
        ca = R.from_euler("xyz", np.array([[-10, 90, 45], [10, 90, -45]]), degrees=True).as_matrix()
        cm = np.array([[[800.0, 0, 800], [0, 800.0, 450], [0, 0, 1]]] * 2)
        out["main_servo_deg"] = np.asarray(sc2.servo_ext_pixel(cm, ca, np.array([[25, 46], [85, -96]]))).reshape(-1, 3)
        out["main_cam_matrix"] = ca
    out["car_pos"] = car_pos
    out["uav_pos"] = uav_pos
    out["uav_quat"] = uav_quat
    out["uav_matrix"] = uav_matrix
    out["near_pos"] = near.numpy()
    np.savez(os.path.join(HERE, "controller_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "controller_golden.npz"), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
