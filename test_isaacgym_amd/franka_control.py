"""GPU-resident cube-pick controller of examples/franka_cube_ik_osc.py (S3).

The reference script computes, every frame, from the refreshed rigid-body,
DOF, Jacobian and mass-matrix tensors (:336-346): the grasp state machine
(:348-401), an operational-space (OSC, :59-79) or damped-least-squares IK
(:51-56) arm command, and gripper targets (:403-407). This module restates that
loop so the S3 bench and the parity tests drive the engine exactly as the
script does, without the viewer. The math follows the cited lines; names
follow the script.

Two implementations behind one step(): on a HIP device, one kernel launch
(csrc/mg_ctrl.hip through mg_cube_pick_step: one lane per env, the inverses as
Cholesky solves in registers; round 6), and the batched torch ops the kernel
replaced (`fused=False`, and on the CPU), ~150 launches per frame. The two
agree to float32 rounding (tests/test_franka_ctrl_gpu.py).
"""
import ctypes
import math

import numpy as np
import torch

from .torch_utils import quat_conjugate, quat_mul


class _CubePickArgs(ctypes.Structure):
    """include/migym.h mg_cube_pick_args."""
    _fields_ = [("n", ctypes.c_int32), ("osc", ctypes.c_int32),
                ("rb", ctypes.c_void_p), ("box_row", ctypes.c_void_p), ("hand_row", ctypes.c_void_p),
                ("dof", ctypes.c_void_p), ("dof_row0", ctypes.c_void_p),
                ("jac", ctypes.c_void_p), ("jac_se", ctypes.c_int64), ("jac_sr", ctypes.c_int64),
                ("jac_sc", ctypes.c_int64),
                ("mm", ctypes.c_void_p), ("mm_se", ctypes.c_int64), ("mm_sr", ctypes.c_int64),
                ("mm_sc", ctypes.c_int64),
                ("init_pos", ctypes.c_void_p), ("init_rot", ctypes.c_void_p), ("default_dof_pos", ctypes.c_void_p),
                ("hand_restart", ctypes.c_void_p), ("pos_action", ctypes.c_void_p),
                ("effort_action", ctypes.c_void_p),
                ("kp", ctypes.c_float), ("kd", ctypes.c_float), ("kp_null", ctypes.c_float),
                ("kd_null", ctypes.c_float), ("damping", ctypes.c_float), ("grasp_offset", ctypes.c_float),
                ("box_size", ctypes.c_float)]


def _inv(a):
    """torch.inverse without the host-side singularity check (linalg.inv_ex), so
    the controller can be captured into a hipGraph; same values."""
    return torch.linalg.inv_ex(a)[0]


def _bmm(a, b):
    """Batched product of tiny matrices, (n, i, k) x (n, k, j), as one broadcast
    multiply and a reduction: rocBLAS batched GEMM tiles cost ~58 us per call at
    4096 x 7x7 on MI355X, this ~5 us."""
    return (a.unsqueeze(-1) * b.unsqueeze(-3)).sum(-2)


def quat_rotate(q, v):
    """torch_utils.quat_rotate with the q_vec . v dot product as an elementwise
    multiply-sum instead of a (n,1,3)x(n,3,1) torch.bmm: same formula, but the
    bmm dispatches a 256x16 hipBLASLt tile at ~56 us per call on MI355X (three
    calls per S3 frame, rocprof r01), this ~5 us."""
    q_w = q[:, -1:]
    q_vec = q[:, :3]
    a = v * (2.0 * q_w * q_w - 1.0)
    b = torch.cross(q_vec, v, dim=-1) * q_w * 2.0
    c = q_vec * (q_vec * v).sum(-1, keepdim=True) * 2.0
    return a + b + c


def quat_axis(q, axis=0):
    """franka_cube_ik_osc.py:28-31."""
    basis = torch.zeros(q.shape[0], 3, device=q.device, dtype=q.dtype)
    basis[:, axis] = 1
    return quat_rotate(q, basis)


def orientation_error(desired, current):
    """franka_cube_ik_osc.py:34-37."""
    q_r = quat_mul(desired, quat_conjugate(current))
    return q_r[:, 0:3] * torch.sign(q_r[:, 3]).unsqueeze(-1)


def cube_grasping_yaw(q, corners):
    """franka_cube_ik_osc.py:40-50: horizontal rotation that aligns the hand with the cube."""
    rc = quat_rotate(q, corners)
    yaw = (torch.atan2(rc[:, 1], rc[:, 0]) - 0.25 * math.pi) % (0.5 * math.pi)
    theta = 0.5 * yaw
    w = theta.cos()
    z = theta.sin()
    zero = torch.zeros_like(w)
    return torch.stack([zero, zero, z, w], dim=-1)


class CubePick:
    """Batched controller state for num_envs Franka cube-pick envs.

    step() takes the refreshed tensors and returns (pos_action, effort_action),
    the (num_envs, 9) tensors the script hands to set_dof_position_target_tensor
    and set_dof_actuation_force_tensor (:409-410)."""

    def __init__(self, num_envs, init_pos, init_rot, default_dof_pos, device, controller="osc",
                 box_size=0.045, damping=0.05, kp=150.0, kp_null=10.0, fused=None):
        self.n = num_envs
        self.device = device
        # fused: the one-kernel controller (csrc/mg_ctrl.hip) on a HIP device;
        # None = there by default, False = the batched torch ops
        self.fused = (torch.device(device).type == "cuda") if fused is None else bool(fused)
        self._args = None
        self.controller = controller
        self.box_size = box_size
        self.damping = damping
        self.kp = kp
        self.kd = 2.0 * np.sqrt(kp)
        self.kp_null = kp_null
        self.kd_null = 2.0 * np.sqrt(kp_null)
        f32 = dict(dtype=torch.float32, device=device)
        self.init_pos = torch.as_tensor(np.asarray(init_pos, dtype=np.float32), **f32).view(num_envs, 3)
        self.init_rot = torch.as_tensor(np.asarray(init_rot, dtype=np.float32), **f32).view(num_envs, 4)
        self.default_dof_pos = torch.as_tensor(np.asarray(default_dof_pos, dtype=np.float32), **f32)
        self.down_q = torch.tensor([1.0, 0.0, 0.0, 0.0], **f32).repeat(num_envs, 1)
        h = 0.5 * box_size
        self.corners = torch.tensor([h, h, h], **f32).repeat(num_envs, 1)
        self.down_dir = torch.tensor([0.0, 0.0, -1.0], **f32).view(1, 3)
        self.hand_restart = torch.zeros(num_envs, dtype=torch.bool, device=device)
        self.pos_action = torch.zeros(num_envs, 9, **f32)
        self.effort_action = torch.zeros(num_envs, 9, **f32)
        self.grip_closed = torch.zeros(num_envs, 2, **f32)
        self.grip_open = torch.full((num_envs, 2), 0.04, **f32)
        self.eye7 = torch.eye(7, **f32).unsqueeze(0)

    def control_ik(self, j_eef, dpose):
        """franka_cube_ik_osc.py:51-56."""
        j_t = torch.transpose(j_eef, 1, 2)
        lmbda = torch.eye(6, device=j_eef.device) * (self.damping ** 2)
        return _bmm(_bmm(j_t, _inv(_bmm(j_eef, j_t) + lmbda)), dpose).view(self.n, 7)

    def control_osc(self, j_eef, mm, dpose, hand_vel, dof_pos, dof_vel):
        """franka_cube_ik_osc.py:59-79."""
        mm_inv = _inv(mm)
        j_t = torch.transpose(j_eef, 1, 2)
        m_eef = _inv(_bmm(_bmm(j_eef, mm_inv), j_t))
        u = _bmm(_bmm(j_t, m_eef), self.kp * dpose - self.kd * hand_vel.unsqueeze(-1))
        j_eef_inv = _bmm(_bmm(m_eef, j_eef), mm_inv)
        u_null = self.kd_null * -dof_vel + self.kp_null * (
            (self.default_dof_pos.view(1, -1, 1) - dof_pos + np.pi) % (2 * np.pi) - np.pi)
        u_null = _bmm(mm, u_null[:, :7])
        u = u + _bmm(self.eye7 - _bmm(j_t, j_eef_inv), u_null)
        return u.squeeze(-1)

    def _fused_args(self, rb_states, dof_pos, dof_vel, j_eef, mm, box_idxs, hand_idxs):
        """The kernel's arguments for these tensors (built on the first call and
        kept while the same tensors come back: a captured hipGraph replays the
        pointers)."""
        key = (rb_states.data_ptr(), dof_pos.data_ptr(), j_eef.data_ptr(), mm.data_ptr(), box_idxs.data_ptr(),
               hand_idxs.data_ptr())
        if self._args is not None and self._args[0] == key:
            return self._args[1]
        n = self.n
        ok = (rb_states.dtype == torch.float32 and rb_states.is_contiguous() and rb_states.shape[1] == 13 and
              dof_pos.shape == (n, 9, 1) and dof_pos.stride(1) == 2 and dof_pos.stride(0) % 2 == 0 and
              dof_vel.data_ptr() == dof_pos.data_ptr() + 4 and dof_vel.stride() == dof_pos.stride() and
              j_eef.shape == (n, 6, 7) and mm.shape == (n, 7, 7) and j_eef.dtype == torch.float32 and
              mm.dtype == torch.float32)
        if not ok:
            raise ValueError("CubePick(fused=True): rb_states (nb, 13) contiguous, dof_pos / dof_vel the (n, 9, 1) "
                             "views of the DOF state's two columns, j_eef (n, 6, 7) and mm (n, 7, 7) float32 views")
        box_row = box_idxs.to(torch.int32).contiguous()
        hand_row = hand_idxs.to(torch.int32).contiguous()
        dof_row0 = torch.arange(n, dtype=torch.int32, device=rb_states.device) * (dof_pos.stride(0) // 2)
        a = _CubePickArgs()
        a.n = n
        a.osc = 1 if self.controller == "osc" else 0
        a.rb = rb_states.data_ptr()
        a.box_row, a.hand_row, a.dof_row0 = box_row.data_ptr(), hand_row.data_ptr(), dof_row0.data_ptr()
        a.dof = dof_pos.data_ptr()
        a.jac = j_eef.data_ptr()
        a.jac_se, a.jac_sr, a.jac_sc = j_eef.stride()
        a.mm = mm.data_ptr()
        a.mm_se, a.mm_sr, a.mm_sc = mm.stride()
        a.init_pos, a.init_rot = self.init_pos.data_ptr(), self.init_rot.data_ptr()
        a.default_dof_pos = self.default_dof_pos.data_ptr()
        a.hand_restart = self.hand_restart.data_ptr()
        a.pos_action, a.effort_action = self.pos_action.data_ptr(), self.effort_action.data_ptr()
        a.kp, a.kd, a.kp_null, a.kd_null = self.kp, self.kd, self.kp_null, self.kd_null
        a.damping = self.damping
        a.grasp_offset = 0.11 if self.controller == "ik" else 0.10
        a.box_size = self.box_size
        self._args = (key, a, (box_row, hand_row, dof_row0))   # the index tensors live with the args
        return a

    def step(self, rb_states, dof_pos, dof_vel, j_eef, mm, box_idxs, hand_idxs):
        """One controller frame (franka_cube_ik_osc.py:348-407).
        rb_states (num_bodies, 13); dof_pos / dof_vel (n, 9, 1); j_eef (n, 6, 7);
        mm (n, 7, 7); box_idxs / hand_idxs: long tensors of body rows."""
        if self.fused:
            from . import _native as N
            a = self._fused_args(rb_states, dof_pos, dof_vel, j_eef, mm, box_idxs, hand_idxs)
            stream = torch.cuda.current_stream(rb_states.device).cuda_stream
            N.check(N.lib.mg_cube_pick_step(ctypes.byref(a), ctypes.c_void_p(stream)), "mg_cube_pick_step")
            return self.pos_action, self.effort_action
        box_pos = rb_states[box_idxs, :3]
        box_rot = rb_states[box_idxs, 3:7]
        hand_pos = rb_states[hand_idxs, :3]
        hand_rot = rb_states[hand_idxs, 3:7]
        hand_vel = rb_states[hand_idxs, 7:]

        to_box = box_pos - hand_pos
        box_dist = torch.norm(to_box, dim=-1).unsqueeze(-1)
        box_dir = to_box / box_dist
        box_dot = (box_dir * self.down_dir).sum(-1, keepdim=True)
        grasp_offset = 0.11 if self.controller == "ik" else 0.10

        gripper_sep = dof_pos[:, 7] + dof_pos[:, 8]
        gripped = (gripper_sep < 0.045) & (box_dist < grasp_offset + 0.5 * self.box_size)

        yaw_q = cube_grasping_yaw(box_rot, self.corners)
        box_yaw_dir = quat_axis(yaw_q, 0)
        hand_yaw_dir = quat_axis(hand_rot, 0)
        yaw_dot = (box_yaw_dir * hand_yaw_dir).sum(-1, keepdim=True)

        to_init = self.init_pos - hand_pos
        init_dist = torch.norm(to_init, dim=-1)
        # in-place state updates: the step can be captured into a hipGraph and replayed
        self.hand_restart.copy_(self.hand_restart & (init_dist > 0.02))
        return_to_start = (self.hand_restart | gripped.squeeze(-1)).unsqueeze(-1)

        above_box = ((box_dot >= 0.99) & (yaw_dot >= 0.95) & (box_dist < grasp_offset * 3)).squeeze(-1)
        grasp_pos = box_pos.clone()
        grasp_pos[:, 2] = torch.where(above_box, box_pos[:, 2] + grasp_offset, box_pos[:, 2] + grasp_offset * 2.5)

        goal_pos = torch.where(return_to_start, self.init_pos, grasp_pos)
        goal_rot = torch.where(return_to_start, self.init_rot, quat_mul(self.down_q, quat_conjugate(yaw_q)))

        pos_err = goal_pos - hand_pos
        orn_err = orientation_error(goal_rot, hand_rot)
        dpose = torch.cat([pos_err, orn_err], -1).unsqueeze(-1)

        if self.controller == "ik":
            self.pos_action[:, :7] = dof_pos.squeeze(-1)[:, :7] + self.control_ik(j_eef, dpose)
        else:
            self.effort_action[:, :7] = self.control_osc(j_eef, mm, dpose, hand_vel, dof_pos, dof_vel)

        close_gripper = (box_dist < grasp_offset + 0.02) | gripped
        self.hand_restart.copy_(self.hand_restart | (box_pos[:, 2] > 0.6))
        keep_going = torch.logical_not(self.hand_restart)
        close_gripper = close_gripper & keep_going.unsqueeze(-1)
        self.pos_action[:, 7:9] = torch.where(close_gripper, self.grip_closed, self.grip_open)
        return self.pos_action, self.effort_action
