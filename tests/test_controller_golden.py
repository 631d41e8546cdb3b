"""Row a9: the torch-batched servo controller (test_isaacgym_amd/servo_control.py)
against golden vectors produced by the reference's own controller code
(tests/golden/make_controller_golden.py: common/controller6.py,
common/secondary_control_vecenv.py). float64 on the CPU: rtol 1e-9 (pixel
coordinates of targets behind the camera reach 1e12 through the reference's
z >= 1e-7 clamp, controller6.py:241, so they get rtol 1e-6); float32 on the GPU:
atol 1e-3 deg / 1e-4 m/s on the well-conditioned rows."""
import os

import numpy as np
import pytest
import torch

from test_isaacgym_amd import servo_control as sc

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "controller_golden.npz"))


def t64(k):
    return torch.tensor(G[k], dtype=torch.float64)


def test_cclvf2_golden():
    car = t64("car_pos")
    np.testing.assert_allclose(sc.cclvf2(car, torch.ones_like(car), 50, 30).numpy(), G["car_vel"], rtol=1e-12)
    uav = t64("uav_pos")
    tgt = car.clone()
    tgt[:, 2] = 260
    np.testing.assert_allclose(sc.cclvf2(uav, tgt, 50, 50).numpy(), G["uav_vel"], rtol=1e-12)
    near = t64("near_pos")
    np.testing.assert_allclose(sc.cclvf2(near, torch.ones_like(near), 10, 10).numpy(), G["near_vel"],
                               rtol=1e-12, atol=1e-12)


def test_euler2quaternion_golden():
    q = sc.euler2quaternion(t64("euler")).numpy()
    np.testing.assert_allclose(q, G["euler_quat"], atol=1e-12)


def test_world2pixel_golden():
    cam = sc.CameraController(1600, 900)
    np.testing.assert_allclose(cam.camera_matrix.numpy(), G["camera_matrix"])
    uav_m = sc.quat_to_matrix(t64("uav_quat"))
    np.testing.assert_allclose(uav_m.numpy(), G["uav_matrix"], atol=1e-12)
    px = cam.world2pixel(t64("uav_pos"), t64("car_pos"), uav_m)[:, :2].numpy()
    np.testing.assert_allclose(px, G["pixel"], rtol=1e-6)


def test_servo_ext_pixel_golden():
    ctl = sc.SecondaryControl(1600, 900)
    got = ctl.servo_ext_pixel(t64("camera_matrix"), t64("uav_matrix"), t64("pixel_move")).numpy()
    ref = G["servo_deg"]
    np.testing.assert_allclose(got, ref, rtol=1e-7, atol=1e-7)


def test_servo_ext_pixel_reference_main():
    """The reference's own known answer (secondary_control_vecenv.py:203-231)."""
    ctl = sc.SecondaryControl(1600, 900)
    cm = torch.tensor([[[800.0, 0, 800], [0, 800.0, 450], [0, 0, 1]]] * 2, dtype=torch.float64)
    got = ctl.servo_ext_pixel(cm, t64("main_cam_matrix"), torch.tensor([[25.0, 46.0], [85.0, -96.0]],
                                                                        dtype=torch.float64)).numpy()
    np.testing.assert_allclose(got, G["main_servo_deg"], atol=1e-9)
    np.testing.assert_allclose(got, [[28.5745, 86.2557, 83.5231], [138.1169, 80.8942, 83.4778]], atol=1e-4)


@pytest.mark.gpu
def test_controller_on_device_fp32():
    dev = "cuda:0"
    f = lambda k: torch.tensor(G[k], dtype=torch.float32, device=dev)  # noqa: E731
    car = f("car_pos")
    v = sc.cclvf2(car, torch.ones_like(car), 50, 30).cpu().numpy()
    np.testing.assert_allclose(v, G["car_vel"], atol=1e-4, rtol=1e-4)
    ctl = sc.SecondaryControl(1600, 900)
    deg = ctl.servo_ext_pixel(f("camera_matrix"), f("uav_matrix"), f("pixel_move")).cpu().numpy()
    ok = np.isfinite(G["servo_deg"]).all(1)
    np.testing.assert_allclose(deg[ok], G["servo_deg"][ok], atol=2e-2)
