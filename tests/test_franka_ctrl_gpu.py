"""GPU: the S3 cube-pick controller as one kernel (csrc/mg_ctrl.hip,
mg_cube_pick_step) against the batched torch restatement it replaced
(test_isaacgym_amd/franka_control.py, fused=False), both restating
examples/franka_cube_ik_osc.py:348-410.

Every frame the fused controller and the torch path see identical inputs (the
sim driven by the float32 torch path's actions; the flag state copied from it
before each call), over the approach, grasp and lift phases of the pick loop.
The grasp state machine's outputs (gripper targets, restart flags) must agree
with the float32 torch path exactly wherever the inputs are not within
rounding of a threshold. The OSC efforts (:59-79) and IK targets (:51-56) are
compared with the torch path evaluated in float64 on the same inputs (the
kernel's linear algebra runs in float64: J M^-1 J^T is badly conditioned near
the arm's singular poses, where the float32 torch evaluation itself is off by
orders of magnitude more — printed for reference), relative to the command's
size. Not bit for bit: the controller is the reference script's own torch
code, not part of the engine the oracle restates.
"""
import numpy as np
import pytest
import torch

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import franka_control, scenes

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("controller", ["osc", "ik"])
def test_fused_controller_matches_torch(gym, controller):
    n, frames = 256, 300
    sim, info = scenes.franka_scene(gym, n, use_gpu_pipeline=True, controller=controller)
    gym.prepare_sim(sim)
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    dof = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    jac = gymtorch.wrap_tensor(gym.acquire_jacobian_tensor(sim, "franka"))
    mm = gymtorch.wrap_tensor(gym.acquire_mass_matrix_tensor(sim, "franka"))
    args = (n, info["init_pos"], info["init_rot"], info["default_dof_pos"], DEV, controller)
    ref = franka_control.CubePick(*args, fused=False)
    r64 = franka_control.CubePick(*args, fused=False)
    for name in ("init_pos", "init_rot", "default_dof_pos", "down_q", "corners", "down_dir", "pos_action",
                 "effort_action", "grip_closed", "grip_open", "eye7"):
        setattr(r64, name, getattr(r64, name).double())      # the torch path in float64 throughout
    fus = franka_control.CubePick(*args, fused=True)
    h = info["hand_index"]
    bi = torch.tensor(info["box_idxs"], device=DEV)
    hi = torch.tensor(info["hand_idxs"], device=DEV)
    j_eef = jac[:, h - 1, :, :7]
    mm7 = mm[:, :7, :7]
    dp = dof[:, 0].view(n, 9, 1)
    dv = dof[:, 1].view(n, 9, 1)
    worst, worst32, restarts, closes, differ = 0.0, 0.0, 0, 0, 0

    def rel(a, b):
        a, b = a.double(), b.double()
        if a.numel() == 0:
            return 0.0
        return float(((a - b).abs() / torch.clamp(b.abs().amax(1, keepdim=True), min=1.0)).max())
    for f in range(frames):
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_jacobian_tensors(sim)
        gym.refresh_mass_matrix_tensors(sim)
        fus.hand_restart.copy_(ref.hand_restart)
        r64.hand_restart.copy_(ref.hand_restart)
        pa_f, ea_f = fus.step(rb, dp, dv, j_eef, mm7, bi, hi)
        pa_f, ea_f = pa_f.clone(), ea_f.clone()
        pa64, ea64 = r64.step(rb.double(), dp.double(), dv.double(), j_eef.double(), mm7.double(), bi, hi)
        pa64, ea64 = pa64.clone(), ea64.clone()
        restart64 = r64.hand_restart.clone()
        pa, ea = ref.step(rb, dp, dv, j_eef, mm7, bi, hi)
        torch.cuda.synchronize()
        # the state machine's discrete outputs: equal in all but (at most) a
        # few envs per frame whose inputs sit on a threshold
        same = (pa_f[:, 7:9] == pa[:, 7:9]).all(1) & (fus.hand_restart == ref.hand_restart)
        differ += int((~same).sum())
        restarts += int(ref.hand_restart.sum())
        closes += int((pa[:, 7] == 0.0).sum())
        # the arm command against float64, on the envs whose state machine agreed
        same64 = same & (pa64[:, 7:9] == pa[:, 7:9]).all(1) & (restart64 == ref.hand_restart)
        if controller == "osc":
            worst = max(worst, rel(ea_f[same64, :7], ea64[same64, :7]))
            worst32 = max(worst32, rel(ea[same64, :7], ea64[same64, :7]))
        else:
            worst = max(worst, rel(pa_f[same64, :7], pa64[same64, :7]))
            worst32 = max(worst32, rel(pa[same64, :7], pa64[same64, :7]))
        gym.set_dof_position_target_tensor(sim, gymtorch.unwrap_tensor(pa))
        gym.set_dof_actuation_force_tensor(sim, gymtorch.unwrap_tensor(ea))
    print("fused vs torch controller:", controller, "worst rel vs float64", worst, "(torch float32 vs float64",
          worst32, ") differing env-frames", differ, "closed-gripper env-frames", closes, "restart env-frames",
          restarts)
    assert closes > n and restarts > 0           # the window reaches the grasp and the return
    assert differ <= frames * n // 1000, differ
    assert worst < 1e-4, worst
