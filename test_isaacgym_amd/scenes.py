"""Benchmark / parity scenes, built through the public gymapi exactly as the
reference scripts build them:

  S1 servo   — test10_servo_vecenv.py:117-144 (sim params), :198-206 (ground),
               :227-230 (asset options), :243-247 (env grid), :310-323 (actors:
               UAV at (-10, 0, 102), ground vehicle at (0, 0, 2), group=i,
               filter=-1); no cameras or viewer.
  S2 gimbal  — test12_add_joint.py.py:23-34 (gravity 0, TGS 4/1, 2 substeps),
               :72-88 (fixed base at (0, 2, 3), DOF_MODE_POS), stiffness 50 /
               damping 5 (test13_camera_spherical_joint.py:200-203), filter=1.

and the synthetic random actions of SURVEY.md §8d (seeded torch generators).
"""
import math
import os

import torch

from . import gymapi

ASSET_ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


def servo_sim_params(use_gpu_pipeline=True):
    sp = gymapi.SimParams()
    sp.dt = 1 / 60
    sp.substeps = 2
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0.0, 0.0, -9.8)
    sp.physx.use_gpu = True
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 6
    sp.physx.num_velocity_iterations = 1
    sp.physx.contact_offset = 0.01
    sp.physx.rest_offset = 0.0
    sp.use_gpu_pipeline = use_gpu_pipeline
    return sp


def servo_scene(gym, num_envs, use_gpu_pipeline=True, device=0, uav_height=102.0, asset_root=None,
                asset_files=("servo/uav.urdf", "servo/ground_vehicle.urdf"), env_offset=0, grid_envs=None):
    """Returns (sim, envs). Actor rows alternate UAV, vehicle (test10 :373-374).
    env_offset / grid_envs: this sim holds envs [env_offset, env_offset +
    num_envs) of a grid laid out for grid_envs envs (sharding.py)."""
    sim = gym.create_sim(device, device, gymapi.SIM_PHYSX, servo_sim_params(use_gpu_pipeline))
    sim.env_offset = env_offset
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    plane.distance = 0
    plane.static_friction = 1
    plane.dynamic_friction = 1
    plane.restitution = 0
    gym.add_ground(sim, plane)
    root = asset_root or ASSET_ROOT
    assets = []
    for f in asset_files:
        opts = gymapi.AssetOptions()
        opts.armature = 0.01
        a = gym.load_asset(sim, root, f, opts)
        if a is None:
            raise RuntimeError("failed to load %s" % f)
        assets.append(a)
    per_row = int(math.sqrt(grid_envs or num_envs))
    spacing = 20.0
    lower = gymapi.Vec3(-spacing, -spacing, -spacing)
    upper = gymapi.Vec3(spacing, spacing, spacing)
    envs = []
    for i in range(num_envs):
        env = gym.create_env(sim, lower, upper, per_row)
        envs.append(env)
        uav_pose = gymapi.Transform()
        uav_pose.p = gymapi.Vec3(-10.0, 0.0, uav_height)
        gym.create_actor(env, assets[0], uav_pose, "predator%d" % i, i, -1)
        car_pose = gymapi.Transform()
        car_pose.p = gymapi.Vec3(0.0, 0.0, 2.0)
        gym.create_actor(env, assets[1], car_pose, "fuchs-apc%d" % i, i, -1)
    return sim, envs


def gimbal_scene(gym, num_envs, use_gpu_pipeline=True, device=0, stiffness=50.0, damping=5.0,
                 asset_root=None, asset_file="servo/gimbal.urdf"):
    sp = gymapi.SimParams()
    sp.substeps = 2
    sp.dt = 1.0 / 60.0
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0.0, 0.0, 0.0)
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 4
    sp.physx.num_velocity_iterations = 1
    sp.use_gpu_pipeline = use_gpu_pipeline
    sim = gym.create_sim(device, device, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    opts.default_dof_drive_mode = gymapi.DOF_MODE_POS
    asset = gym.load_asset(sim, asset_root or ASSET_ROOT, asset_file, opts)
    if asset is None:
        raise RuntimeError("failed to load gimbal")
    spacing = 1.0
    lower = gymapi.Vec3(-spacing, -spacing, -spacing)
    upper = gymapi.Vec3(spacing, spacing, spacing)
    per_row = int(math.sqrt(num_envs))
    envs = []
    for i in range(num_envs):
        env = gym.create_env(sim, lower, upper, per_row)
        envs.append(env)
        pose = gymapi.Transform()
        pose.p = gymapi.Vec3(0.0, 2.0, 3.0)
        h = gym.create_actor(env, asset, pose, "gimbal", i, 1)
        props = gym.get_actor_dof_properties(env, h)
        props["driveMode"][:] = gymapi.DOF_MODE_POS
        props["stiffness"][:] = stiffness
        props["damping"][:] = damping
        gym.set_actor_dof_properties(env, h, props)
    return sim, envs


# ------------------------------------------------------------- random actions
def quat_from_euler_xyz(roll, pitch, yaw):
    """scipy Rotation.from_euler('xyz', [r, p, y]).as_quat() in torch (xyzw)."""
    cr, sr = torch.cos(0.5 * roll), torch.sin(0.5 * roll)
    cp, sp = torch.cos(0.5 * pitch), torch.sin(0.5 * pitch)
    cy, sy = torch.cos(0.5 * yaw), torch.sin(0.5 * yaw)
    return torch.stack([sr * cp * cy - cr * sp * sy,
                        cr * sp * cy + sr * cp * sy,
                        cr * cp * sy - sr * sp * cy,
                        cr * cp * cy + sr * sp * sy], dim=-1)


def servo_actions(num_envs, num_batches, device, seed=0):
    """Bank of random root-state actions, (num_batches, 2*num_envs, 7) =
    [quat xyzw, linvel xyz] per actor row: UAV roll, yaw ~
    U(-pi, pi), pitch ~ U(-pi/2, pi/2); vehicle yaw ~ U(-pi, pi); linear
    velocity ~ U(-50, 50)^3 m/s."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    B, n = num_batches, num_envs
    u = lambda *s: torch.rand(*s, generator=g, dtype=torch.float64)  # noqa: E731
    uav_q = quat_from_euler_xyz((u(B, n) * 2 - 1) * math.pi, (u(B, n) * 2 - 1) * math.pi / 2,
                                (u(B, n) * 2 - 1) * math.pi)
    z = torch.zeros(B, n, dtype=torch.float64)
    car_q = quat_from_euler_xyz(z, z, (u(B, n) * 2 - 1) * math.pi)
    vel = (u(B, 2 * n, 3) * 2 - 1) * 50.0
    act = torch.empty(B, 2 * n, 7, dtype=torch.float64)
    act[:, 0::2, 0:4] = uav_q
    act[:, 1::2, 0:4] = car_q
    act[:, :, 4:7] = vel
    return act.to(torch.float32).to(device)


def gimbal_targets(num_envs, num_batches, device, seed=0):
    """(num_batches, 3*num_envs) position targets ~ U(-1.57, 1.57)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    t = (torch.rand(num_batches, 3 * num_envs, generator=g) * 2 - 1) * 1.57
    return t.to(torch.float32).to(device)
