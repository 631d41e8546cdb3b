"""Scenes of the free-body pile step, shared by
tests/test_pile.py (oracle KATs, CPU) and tests/test_pile_gpu.py (device
parity): coupled envs of more than two free bodies and no articulation."""
import math
import os

import numpy as np

from isaacgym import gymapi

G = 9.8


def sim_params(gpu, up="z", substeps=2, npos=6, nvel=1, gravity=True, contact_offset=0.01, rest_offset=0.0):
    sp = gymapi.SimParams()
    if up == "z":
        sp.up_axis = gymapi.UP_AXIS_Z
        sp.gravity = gymapi.Vec3(0, 0, -G if gravity else 0.0)
    else:
        sp.up_axis = gymapi.UP_AXIS_Y
        sp.gravity = gymapi.Vec3(0, -G if gravity else 0.0, 0)
    sp.dt = 1.0 / 60.0
    sp.substeps = substeps
    sp.use_gpu_pipeline = gpu
    sp.physx.solver_type = 1
    sp.physx.num_position_iterations = npos
    sp.physx.num_velocity_iterations = nvel
    sp.physx.contact_offset = contact_offset
    sp.physx.rest_offset = rest_offset
    return sp


def hull_urdf(d, h=0.06):
    """An octahedron hull (6 vertices) as an OBJ mesh behind a URDF in d."""
    with open(os.path.join(d, "octa.obj"), "w") as f:
        for v in ((h, 0, 0), (-h, 0, 0), (0, h, 0), (0, -h, 0), (0, 0, h), (0, 0, -h)):
            f.write("v %g %g %g\n" % v)
    with open(os.path.join(d, "octa.urdf"), "w") as f:
        f.write('<robot name="o"><link name="body"><collision><geometry><mesh filename="octa.obj"/></geometry>'
                '</collision><inertial><mass value="0.2"/><inertia ixx="3e-4" iyy="3e-4" izz="3e-4" ixy="0" '
                'ixz="0" iyz="0"/></inertial></link></robot>')
    return "octa.urdf"


def mixed_pile_scene(gym, n, gpu, d=None, seed=0, counts=None, static=True, up="z"):
    """Per env a heap of spheres, boxes, capsules (and octahedron hulls when d
    is a writable directory) dropped from staggered heights onto the ground and
    a fixed box, one collision group per env (group i, filter 0). counts: free
    bodies per env (ragged); default 3 + (7 i) % 62. Returns (sim, info)."""
    sim = gym.create_sim(0, 0, gymapi.SIM_PHYSX, sim_params(gpu, up=up))
    plane = gymapi.PlaneParams()
    plane.normal = gymapi.Vec3(0, 0, 1) if up == "z" else gymapi.Vec3(0, 1, 0)
    gym.add_ground(sim, plane)
    fixed = gymapi.AssetOptions()
    fixed.fix_base_link = True
    table = gym.create_box(sim, 0.3, 0.3, 0.3, fixed)
    kinds = [gym.create_sphere(sim, 0.05, gymapi.AssetOptions()),
             gym.create_box(sim, 0.08, 0.06, 0.05, gymapi.AssetOptions()),
             gym.create_capsule(sim, 0.03, 0.08, gymapi.AssetOptions())]
    if d is not None:
        kinds.append(gym.load_asset(sim, d, hull_urdf(d), gymapi.AssetOptions()))
    rng = np.random.RandomState(seed)
    per_env = []
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 8)
        if static:
            pos = gymapi.Vec3(0.3, 0.1, 0.15) if up == "z" else gymapi.Vec3(0.3, 0.15, 0.1)
            gym.create_actor(env, table, gymapi.Transform(pos), "table", i, 0)
        c = counts[i] if counts is not None else 3 + (7 * i) % 62
        for k in range(c):
            kind = kinds[(k + i) % len(kinds)]
            x, y = rng.uniform(-0.25, 0.45), rng.uniform(-0.25, 0.35)
            hgt = 0.3 + 0.07 * k + rng.uniform(0, 0.02)
            pos = gymapi.Vec3(x, y, hgt) if up == "z" else gymapi.Vec3(x, hgt, y)
            pose = gymapi.Transform(pos)
            ax = rng.normal(size=3)
            pose.r = gymapi.Quat.from_axis_angle(gymapi.Vec3(*(ax / np.linalg.norm(ax))), rng.uniform(0, math.pi))
            gym.create_actor(env, kind, pose, "b%d" % k, i, 0)
        per_env.append(c + (1 if static else 0))
    return sim, {"bodies_per_env": per_env}
