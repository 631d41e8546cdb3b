"""Benchmark / parity scenes, built through the public gymapi exactly as the
reference scripts build them:

  S1 servo   — test10_servo_vecenv.py:117-144 (sim params), :198-206 (ground),
               :227-230 (asset options), :243-247 (env grid), :310-323 (actors:
               UAV at (-10, 0, 102), ground vehicle at (0, 0, 2), group=i,
               filter=-1); no cameras or viewer.
  S2 gimbal  — test12_add_joint.py.py:23-34 (gravity 0, TGS 4/1, 2 substeps),
               :72-88 (fixed base at (0, 2, 3), DOF_MODE_POS), stiffness 50 /
               damping 5 (test13_camera_spherical_joint.py:200-203), filter=1.
  S5 cameras — test11_servo_vecenv_camerazoom.py:274-336: the S1 scene plus one
               camera per env on the UAV (local (5, 0, 0), FOLLOW_TRANSFORM),
               1600x900, horizontal FOV 30 degrees, as a GPU image tensor.
  interop    — examples/interop_torch.py:30-120 (y-up, a 0.5 m ball dropped
               from y = 5 per env, 128x128 camera at (5, 1, 0) looking at
               (0, 1, 0)): the scene of the reference's rendered fixture
               examples/interop_images/.

and the synthetic random actions of SURVEY.md §8d (seeded torch generators).
"""
import math
import numpy as np
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
                 asset_root=None, asset_file="servo/gimbal.urdf", drive_mode=None, link_mass_scale=None):
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
        props["driveMode"][:] = gymapi.DOF_MODE_POS if drive_mode is None else drive_mode
        props["stiffness"][:] = stiffness
        props["damping"][:] = damping
        gym.set_actor_dof_properties(env, h, props)
        if link_mass_scale is not None:   # heavier links (inertia scaled with the mass)
            bp = gym.get_actor_rigid_body_properties(env, h)
            for b in bp:
                b.mass = b.mass * link_mass_scale
            gym.set_actor_rigid_body_properties(env, h, bp, True)
    return sim, envs


def attach_servo_cameras(gym, sim, envs, width=1600, height=900, fov=30.0, image_types=None):
    """One camera per env on the UAV body (test11_servo_vecenv_camerazoom.py:
    274-280,327-336: local (5, 0, 0), FOLLOW_TRANSFORM), each with a GPU image
    tensor per requested type. Returns the list of tensors per env."""
    from . import gymtorch
    props = gymapi.CameraProperties()
    props.width, props.height = width, height
    props.horizontal_fov = fov
    props.enable_tensors = True
    out = []
    for env in envs:
        cam = gym.create_camera_sensor(env, props)
        uav = gym.get_actor_handle(env, 0)
        body = gym.get_actor_rigid_body_handle(env, uav, 0)
        local = gymapi.Transform()
        local.p = gymapi.Vec3(5, 0, 0)
        local.r = gymapi.Quat.from_euler_zyx(0, 0, 0)
        gym.attach_camera_to_body(cam, env, body, local, gymapi.FOLLOW_TRANSFORM)
        out.append([gymtorch.wrap_tensor(gym.get_camera_image_gpu_tensor(sim, env, cam, t))
                    for t in (image_types or (gymapi.IMAGE_COLOR,))])
    return out


def interop_scene(gym, num_envs=16, device=0, colors=None):
    """examples/interop_torch.py:30-120: returns (sim, envs, cams)."""
    sp = gymapi.SimParams()
    sp.gravity = gymapi.Vec3(0.0, -9.8, 0.0)
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 4
    sp.physx.num_velocity_iterations = 1
    sp.use_gpu_pipeline = True
    sim = gym.create_sim(device, device, gymapi.SIM_PHYSX, sp)
    ball = gym.create_sphere(sim, 0.5, None)
    gym.add_ground(sim, gymapi.PlaneParams())
    per_row = int(math.sqrt(num_envs))
    spacing = 2.0
    lower = gymapi.Vec3(-spacing, 0.0, -spacing)
    upper = gymapi.Vec3(spacing, spacing, spacing)
    envs, cams = [], []
    for i in range(num_envs):
        env = gym.create_env(sim, lower, upper, per_row)
        envs.append(env)
        pose = gymapi.Transform()
        pose.p = gymapi.Vec3(0.0, 5.0, 0.0)
        pose.r = gymapi.Quat(0.0, 0.0, 0.0, 1.0)
        h = gym.create_actor(env, ball, pose, "ball", i, 0)
        props = gym.get_actor_rigid_shape_properties(env, h)
        props[0].restitution = 0.9
        gym.set_actor_rigid_shape_properties(env, h, props)
        c = colors[i] if colors is not None else (0.75, 0.75, 0.75)
        gym.set_rigid_body_color(env, h, 0, gymapi.MESH_VISUAL_AND_COLLISION, gymapi.Vec3(*c))
        cp = gymapi.CameraProperties()
        cp.width = 128
        cp.height = 128
        cp.enable_tensors = True
        cam = gym.create_camera_sensor(env, cp)
        gym.set_camera_location(cam, env, gymapi.Vec3(5, 1, 0), gymapi.Vec3(0, 1, 0))
        cams.append(cam)
    return sim, envs, cams


def graphics_scene(gym, num_envs=8, device=0, use_gpu_pipeline=True, asset_root=None):
    """examples/graphics.py:46-180 (y-up defaults, TGS 4/1): per env, eight
    assets/urdf/ball.urdf balls on a 3x3 grid of pitch 4/3 m, ball 0 at y = 6,
    the others at y = 0.25, all rotated by Quat(-0.707107, 0, 0, 0.707107),
    group i, filter 1 (the balls of an env do not collide with each other);
    camera 0: 360x240 at env-local (1.5, 1, 1.5) looking at the env origin;
    camera 1: 360x240 attached to ball 0 at offset (1, 0, -1) rotated 135
    degrees about y, FOLLOW_TRANSFORM. Returns (sim, envs, cams[env] = [c0, c1])."""
    sp = gymapi.SimParams()
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 4
    sp.physx.num_velocity_iterations = 1
    sp.use_gpu_pipeline = use_gpu_pipeline
    sim = gym.create_sim(device, device, gymapi.SIM_PHYSX, sp)
    gym.add_ground(sim, gymapi.PlaneParams())
    ball = gym.load_asset(sim, asset_root or ASSET_ROOT, "urdf/ball.urdf", gymapi.AssetOptions())
    if ball is None:
        raise RuntimeError("failed to load ball.urdf")
    spacing = 2.0
    lower = gymapi.Vec3(-spacing, 0.0, -spacing)
    upper = gymapi.Vec3(spacing, spacing, spacing)
    nb = 8
    grid = math.ceil(math.sqrt(nb))
    d = 2 * spacing / grid
    envs, cams = [], []
    for i in range(num_envs):
        env = gym.create_env(sim, lower, upper, 4)
        envs.append(env)
        for j in range(nb):
            pose = gymapi.Transform()
            pose.p = gymapi.Vec3(d * (0.5 + j % grid), 6.0 if j == 0 else 0.25, d * (0.5 + j // grid))
            pose.r = gymapi.Quat(-0.707107, 0.0, 0.0, 0.707107)
            gym.create_actor(env, ball, pose, "asset_%d" % j, i, 1, 0)
        cp = gymapi.CameraProperties()
        cp.width, cp.height = 360, 240
        cp.enable_tensors = True
        c0 = gym.create_camera_sensor(env, cp)
        gym.set_camera_location(c0, env, gymapi.Vec3(1.5, 1, 1.5), gymapi.Vec3(0, 0, 0))
        c1 = gym.create_camera_sensor(env, cp)
        body = gym.get_actor_rigid_body_handle(env, gym.get_actor_handle(env, 0), 0)
        rot = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 1, 0), math.radians(135.0))
        gym.attach_camera_to_body(c1, env, body, gymapi.Transform(gymapi.Vec3(1, 0, -1), rot),
                                  gymapi.FOLLOW_TRANSFORM)
        cams.append([c0, c1])
    return sim, envs, cams


def graphics_depth_u8(depth):
    """examples/graphics.py:225-236's depth image transform: -inf -> 0, clamp at
    -10 m, -255 depth / min(depth + 1e-4), then numpy's float -> uint8 cast
    (negative values wrap modulo 256 on x86, as in the reference's files)."""
    d = np.array(depth, dtype=np.float32, copy=True)
    d[d == -np.inf] = 0
    d[d < -10] = -10
    n = -255.0 * (d / np.min(d + 1e-4))
    return (n.astype(np.int64) % 256).astype(np.uint8)


def graphics_depth_ball_mask(u8):
    """Ball pixels of a graphics.py camera-0 depth image: the ground's depth is
    constant along an image row (a level camera over a flat ground), so a pixel
    more than 12 grey levels from its row's median that is not sky (0) is an
    object in front of the ground. A 3x3 median filter first removes the JPEG
    ringing of the reference's files along the silhouette."""
    from scipy.ndimage import median_filter
    d = median_filter(u8, size=3, mode="nearest").astype(np.int32)
    med = np.median(d, axis=1)
    return (np.abs(d - med[:, None]) > 12) & (d > 0)


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


# ---------------------------------------------------------------- S3 Franka
FRANKA_TABLE_DIMS = (0.6, 1.0, 0.4)
FRANKA_BOX_SIZE = 0.045


def franka_sim_params(use_gpu_pipeline=True):
    """examples/franka_cube_ik_osc.py:111-128."""
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0.0, 0.0, -9.8)
    sp.dt = 1.0 / 60.0
    sp.substeps = 2
    sp.use_gpu_pipeline = use_gpu_pipeline
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 8
    sp.physx.num_velocity_iterations = 1
    sp.physx.rest_offset = 0.0
    sp.physx.contact_offset = 0.001
    sp.physx.friction_offset_threshold = 0.001
    sp.physx.friction_correlation_distance = 0.0005
    sp.physx.use_gpu = True
    return sp


def franka_scene(gym, num_envs, use_gpu_pipeline=True, device=0, controller="osc", seed=42, asset_root=None,
                 asset_file="franka/franka_proxy.urdf"):
    """S3: the cube-pick scene of examples/franka_cube_ik_osc.py:150-285 — per env a
    fixed table (0.6 x 1.0 x 0.4 at x = 0.5), a 4.5 cm cube placed at random on it
    (np.random.seed(seed), same draws in the same order as :244-249), and a
    fixed-base, gravity-free Franka (armature 0.01) with OSC effort drives on the
    arm and 800 / 40 position drives on the fingers; all three in collision group
    i, the Franka with filter 2. The Franka is assets/franka/franka_proxy.urdf
    (tools/make_franka_asset.py). Returns (sim, info dict)."""
    import numpy as np
    np.random.seed(seed)
    sim = gym.create_sim(device, device, gymapi.SIM_PHYSX, franka_sim_params(use_gpu_pipeline))
    tx, ty, tz = FRANKA_TABLE_DIMS
    opts = gymapi.AssetOptions()
    opts.fix_base_link = True
    table_asset = gym.create_box(sim, tx, ty, tz, opts)
    opts = gymapi.AssetOptions()
    box_asset = gym.create_box(sim, FRANKA_BOX_SIZE, FRANKA_BOX_SIZE, FRANKA_BOX_SIZE, opts)
    opts = gymapi.AssetOptions()
    opts.armature = 0.01
    opts.fix_base_link = True
    opts.disable_gravity = True
    opts.flip_visual_attachments = True
    franka_asset = gym.load_asset(sim, asset_root or ASSET_ROOT, asset_file, opts)
    if franka_asset is None:
        raise RuntimeError("franka asset %s not found" % asset_file)
    props = gym.get_asset_dof_properties(franka_asset)
    lower, upper = props["lower"], props["upper"]
    mids = 0.3 * (upper + lower)
    if controller == "ik":
        props["driveMode"][:7].fill(gymapi.DOF_MODE_POS)
        props["stiffness"][:7].fill(400.0)
        props["damping"][:7].fill(40.0)
    else:
        props["driveMode"][:7].fill(gymapi.DOF_MODE_EFFORT)
        props["stiffness"][:7].fill(0.0)
        props["damping"][:7].fill(0.0)
    props["driveMode"][7:].fill(gymapi.DOF_MODE_POS)
    props["stiffness"][7:].fill(800.0)
    props["damping"][7:].fill(40.0)
    ndof = gym.get_asset_dof_count(franka_asset)
    default_pos = np.zeros(ndof, dtype=np.float32)
    default_pos[:7] = mids[:7]
    default_pos[7:] = upper[7:]
    default_state = np.zeros(ndof, gymapi.DofState.dtype)
    default_state["pos"] = default_pos
    hand_index = gym.get_asset_rigid_body_dict(franka_asset)["panda_hand"]

    per_row = int(math.sqrt(num_envs))
    spacing = 1.0
    lo, hi = gymapi.Vec3(-spacing, -spacing, 0.0), gymapi.Vec3(spacing, spacing, spacing)
    franka_pose = gymapi.Transform()
    franka_pose.p = gymapi.Vec3(0, 0, 0)
    table_pose = gymapi.Transform()
    table_pose.p = gymapi.Vec3(0.5, 0.0, 0.5 * tz)
    box_pose = gymapi.Transform()
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    envs, box_idxs, hand_idxs, init_pos, init_rot = [], [], [], [], []
    for i in range(num_envs):
        env = gym.create_env(sim, lo, hi, per_row)
        envs.append(env)
        gym.create_actor(env, table_asset, table_pose, "table", i, 0)
        box_pose.p.x = table_pose.p.x + np.random.uniform(-0.2, 0.1)
        box_pose.p.y = table_pose.p.y + np.random.uniform(-0.3, 0.3)
        box_pose.p.z = tz + 0.5 * FRANKA_BOX_SIZE
        box_pose.r = gymapi.Quat.from_axis_angle(gymapi.Vec3(0, 0, 1), np.random.uniform(-math.pi, math.pi))
        box = gym.create_actor(env, box_asset, box_pose, "box", i, 0)
        np.random.uniform(0, 1, 3)          # the script's colour draws (:251), kept for the same sequence
        box_idxs.append(gym.get_actor_rigid_body_index(env, box, 0, gymapi.DOMAIN_SIM))
        franka = gym.create_actor(env, franka_asset, franka_pose, "franka", i, 2)
        gym.set_actor_dof_properties(env, franka, props)
        gym.set_actor_dof_states(env, franka, default_state, gymapi.STATE_ALL)
        gym.set_actor_dof_position_targets(env, franka, default_pos)
        hand = gym.find_actor_rigid_body_handle(env, franka, "panda_hand")
        hp = gym.get_rigid_transform(env, hand)
        init_pos.append([hp.p.x, hp.p.y, hp.p.z])
        init_rot.append([hp.r.x, hp.r.y, hp.r.z, hp.r.w])
        hand_idxs.append(gym.find_actor_rigid_body_index(env, franka, "panda_hand", gymapi.DOMAIN_SIM))
    info = dict(envs=envs, box_idxs=box_idxs, hand_idxs=hand_idxs, init_pos=init_pos, init_rot=init_rot,
                hand_index=hand_index, default_dof_pos=default_pos, num_dofs=ndof, controller=controller)
    return sim, info


def ant_sim_params(use_gpu_pipeline=True):
    """examples/apply_forces.py:31-41: z-up, g = -9.81, 1 substep, TGS 4/1."""
    sp = gymapi.SimParams()
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(0.0, 0.0, -9.81)
    sp.substeps = 1
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 4
    sp.physx.num_velocity_iterations = 1
    sp.use_gpu_pipeline = use_gpu_pipeline
    return sp


def ant_scene(gym, num_envs, use_gpu_pipeline=True, device=0, asset_root=None, asset_file="mjcf/ant.xml",
              spacing=2.0, seed=17, height=1.0, sim_params=None, asset_options=None):
    """examples/apply_forces.py:51-100: the MJCF ant (a floating-base
    articulation, 9 bodies, 8 hinge DOFs) at z = `height` in a sqrt(n)-per-row
    grid, collision group i, filter 1, random bright colours; ground plane n = +z.
    Returns (sim, info) with info["num_bodies"], ["envs"], ["actors"]."""
    sp = sim_params or ant_sim_params(use_gpu_pipeline)
    sim = gym.create_sim(device, device, gymapi.SIM_PHYSX, sp)
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1)
    gym.add_ground(sim, plane)
    asset = gym.load_asset(sim, asset_root or ASSET_ROOT, asset_file, asset_options or gymapi.AssetOptions())
    nb = gym.get_asset_rigid_body_count(asset)
    pose = gymapi.Transform()
    pose.p.z = height
    per_row = max(int(np.sqrt(num_envs)), 1)
    lo, hi = gymapi.Vec3(-spacing, -spacing, 0.0), gymapi.Vec3(spacing, spacing, spacing)
    rng = np.random.RandomState(seed)
    envs, actors = [], []
    for i in range(num_envs):
        env = gym.create_env(sim, lo, hi, per_row)
        c = 0.5 + 0.5 * rng.random_sample(3)
        a = gym.create_actor(env, asset, pose, "actor", i, 1)
        gym.set_rigid_body_color(env, a, 0, gymapi.MESH_VISUAL_AND_COLLISION, gymapi.Vec3(*c))
        envs.append(env)
        actors.append(a)
    return sim, {"num_bodies": nb, "envs": envs, "actors": actors, "asset": asset}


# ------------------------------------------------------------ S6 ball piles
def ball_pile_sim_params(use_gpu_pipeline=True):
    """examples/1080_balls_of_solitude.py:41-53: Isaac Gym's default (y-up) sim,
    dt 1/60, 1 substep, PhysX TGS 4/1."""
    sp = gymapi.SimParams()
    sp.substeps = 1
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 4
    sp.physx.num_velocity_iterations = 1
    sp.use_gpu_pipeline = use_gpu_pipeline
    return sp


def ball_pyramid_poses(n=4, radius=0.2):
    """The pyramid of examples/1080_balls_of_solitude.py:102-132: layers of
    n x n, (n-1) x (n-1), ... balls spaced 2.5 radii, the bottom layer at
    y = 1.5 + 4 - 0.75 m (30 balls for n = 4), env-local (x, y, z)."""
    out = []
    spacing = 2.5 * radius
    min_coord = -0.5 * (n - 1) * spacing
    y = min_coord + 4
    while n > 0:
        z = min_coord
        for _ in range(n):
            x = min_coord
            for _ in range(n):
                out.append((x, 1.5 + y, z))
                x += spacing
            z += spacing
        y += spacing
        n -= 1
        min_coord = -0.5 * (n - 1) * spacing
    return out


def ball_pile_scene(gym, num_envs, use_gpu_pipeline=True, device=0, asset_root=None, mode="env",
                    sim_params=None, n=4):
    """S6: examples/1080_balls_of_solitude.py:29-136 — per env a pyramid of 30
    assets/urdf/ball.urdf balls (0.2 m, 0.5 kg), env spacing 1.25, sqrt(n) envs
    per row. mode "env" (the script's default): group i, filter 0, so the balls
    of an env collide with each other — a pile env; "none"
    (--no_collisions): group 0, filter 1, only the ground. Returns (sim, envs)."""
    sim = gym.create_sim(device, device, gymapi.SIM_PHYSX, sim_params or ball_pile_sim_params(use_gpu_pipeline))
    gym.add_ground(sim, gymapi.PlaneParams())
    ball = gym.load_asset(sim, asset_root or ASSET_ROOT, "urdf/ball.urdf", gymapi.AssetOptions())
    if ball is None:
        raise RuntimeError("failed to load ball.urdf")
    per_row = max(int(math.sqrt(num_envs)), 1)
    spacing = 1.25
    lower, upper = gymapi.Vec3(-spacing, 0.0, -spacing), gymapi.Vec3(spacing, spacing, spacing)
    poses = ball_pyramid_poses(n)
    rng = np.random.RandomState(17)
    envs = []
    for i in range(num_envs):
        env = gym.create_env(sim, lower, upper, per_row)
        envs.append(env)
        c = 0.5 + 0.5 * rng.random_sample(3)
        for p in poses:
            pose = gymapi.Transform()
            pose.p = gymapi.Vec3(*p)
            pose.r = gymapi.Quat(0, 0, 0, 1)
            group, filt = (i, 0) if mode == "env" else (0, 1)
            a = gym.create_actor(env, ball, pose, None, group, filt)
            gym.set_rigid_body_color(env, a, 0, gymapi.MESH_VISUAL_AND_COLLISION, gymapi.Vec3(*c))
    return sim, envs


# ------------------------------------------------------ domain randomization
DR_CAM_POS = (0.0, 3.0, 3.0)
DR_CAM_TARGET = (0.0, 0.0, -1.0)


def dr_ant_scene(gym, num_envs=1, device=0, use_gpu_pipeline=False, asset_root=None, cam_offsets=None):
    """examples/domain_randomization.py:36-128, restated as data: Isaac Gym's
    default (y-up) sim with dt 1/60, 2 substeps, PhysX TGS 4/1 (:36-48), the
    default ground plane (:60), per env the MJCF ant (assets/mjcf/ant.xml =
    nv_ant.xml) at (0, 0.5, 0) rotated by Quat(-0.707107, 0, 0, 0.707107),
    group i, filter 1 (:109-112), every DOF DOF_MODE_NONE with zero stiffness
    and damping (:116-120), and a default camera sensor attached to the torso
    at (0, 3, 3) (FOLLOW_TRANSFORM) then placed by set_camera_location at
    (0, 3, 3) looking at (0, 0, -1) (:122-128); cam_offsets[e] = (y, z) moves
    env e's camera to (0, 3 + y, 3 + z) as the loop's randomisation does
    (:168-172). The script's textures, colours and lights are not restated
    (they change no geometry). Returns (sim, envs, actors, cams)."""
    sp = gymapi.SimParams()
    sp.substeps = 2
    sp.dt = 1.0 / 60.0
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = 4
    sp.physx.num_velocity_iterations = 1
    sp.use_gpu_pipeline = use_gpu_pipeline
    sim = gym.create_sim(device, device, gymapi.SIM_PHYSX, sp)
    gym.add_ground(sim, gymapi.PlaneParams())
    ant = gym.load_asset(sim, asset_root or ASSET_ROOT, "mjcf/ant.xml", gymapi.AssetOptions())
    if ant is None:
        raise RuntimeError("failed to load the ant")
    spacing = 0.75
    lower, upper = gymapi.Vec3(-spacing, 0.0, -spacing), gymapi.Vec3(spacing, spacing, spacing)
    envs, actors, cams = [], [], []
    for i in range(num_envs):
        env = gym.create_env(sim, lower, upper, 2)
        pose = gymapi.Transform()
        pose.p = gymapi.Vec3(0, 0.5, 0)
        pose.r = gymapi.Quat(-0.707107, 0.0, 0.0, 0.707107)
        a = gym.create_actor(env, ant, pose, "ant", i, 1)
        props = gym.get_actor_dof_properties(env, a)
        props["driveMode"].fill(gymapi.DOF_MODE_NONE)
        props["stiffness"].fill(0.0)
        props["damping"].fill(0.0)
        gym.set_actor_dof_properties(env, a, props)
        cp = gymapi.CameraProperties()
        cp.enable_tensors = True
        c = gym.create_camera_sensor(env, cp)
        body = gym.get_actor_rigid_body_handle(env, a, 0)
        cam_pos = gymapi.Vec3(*DR_CAM_POS)
        gym.attach_camera_to_body(c, env, body, gymapi.Transform(p=cam_pos), gymapi.FOLLOW_TRANSFORM)
        if cam_offsets is not None:
            cam_pos = cam_pos + gymapi.Vec3(0.0, float(cam_offsets[i][0]), float(cam_offsets[i][1]))
        gym.set_camera_location(c, env, cam_pos, gymapi.Vec3(*DR_CAM_TARGET))
        envs.append(env)
        actors.append(a)
        cams.append(c)
    return sim, envs, actors, cams
