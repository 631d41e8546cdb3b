"""isaacgym.gymutil mirror: command-line parsing and debug-line geometry.

parse_arguments returns the fields the reference reads (SURVEY.md §2:
physics_engine, compute_device_id, graphics_device_id, use_gpu,
use_gpu_pipeline, sim_device, num_threads) plus per-script custom_parameters
(examples/franka_cube_ik_osc.py:93-101). Line geometry is kept for API
compatibility; drawing is a no-op (headless).
"""
import argparse
import math

import numpy as np

from . import gymapi


def parse_bool(s):
    if isinstance(s, bool):
        return s
    return str(s).lower() in ("true", "t", "yes", "y", "1")


def parse_device_str(device_str):
    device = "cpu"
    device_id = 0
    if device_str == "cpu" or device_str == "cuda":
        device = device_str
    else:
        parts = device_str.split(":")
        device = parts[0]
        device_id = int(parts[1]) if len(parts) > 1 else 0
    if device not in ("cpu", "cuda"):
        raise ValueError("invalid device string %r" % device_str)
    return device, device_id


def parse_arguments(description="Isaac Gym Example", headless=False, no_graphics=False, custom_parameters=None):
    parser = argparse.ArgumentParser(description=description)
    if headless:
        parser.add_argument("--headless", action="store_true", help="Run headless without creating a viewer window")
    if no_graphics:
        parser.add_argument("--nographics", action="store_true", help="Disable graphics context creation")
    parser.add_argument("--sim_device", type=str, default="cuda:0", help="Physics device, e.g. cuda:0")
    parser.add_argument("--pipeline", type=str, default="gpu", help="Tensor API pipeline (cpu/gpu)")
    parser.add_argument("--graphics_device_id", type=int, default=0, help="Graphics device ID")
    physics_group = parser.add_mutually_exclusive_group()
    physics_group.add_argument("--flex", action="store_true", help="Use FleX for physics")
    physics_group.add_argument("--physx", action="store_true", help="Use PhysX for physics")
    parser.add_argument("--num_threads", type=int, default=0, help="Number of cores used by PhysX")
    parser.add_argument("--subscenes", type=int, default=0, help="Number of PhysX subscenes to simulate in parallel")
    parser.add_argument("--slices", type=int, help="Number of client threads that process env slices")
    for arg in custom_parameters or []:
        if "name" not in arg:
            continue
        kw = {k: v for k, v in arg.items() if k in ("type", "default", "help", "action", "nargs", "choices")}
        parser.add_argument(arg["name"], **kw)
    args = parser.parse_args()
    args.sim_device_type, args.compute_device_id = parse_device_str(args.sim_device)
    pipeline = args.pipeline.lower()
    if pipeline not in ("cpu", "gpu", "cuda"):
        raise ValueError("invalid pipeline %r" % args.pipeline)
    args.use_gpu_pipeline = pipeline in ("gpu", "cuda")
    if args.sim_device_type != "cuda" and args.flex:
        args.sim_device = "cuda:0"
        args.sim_device_type, args.compute_device_id = "cuda", 0
    if args.sim_device_type != "cuda" and args.use_gpu_pipeline:
        print("Can't use GPU pipeline with CPU physics; switching to the CPU pipeline.")
        args.use_gpu_pipeline = False
    args.physics_engine = gymapi.SIM_FLEX if args.flex else gymapi.SIM_PHYSX
    args.use_gpu = args.sim_device_type == "cuda"
    if args.slices is None:
        args.slices = args.subscenes
    return args


class LineGeometry:
    def vertices(self):
        return self.verts

    def colors(self):
        return self._colors


class AxesGeometry(LineGeometry):
    def __init__(self, scale=1.0, pose=None):
        verts = np.empty((3, 2), gymapi.Vec3.dtype)
        verts[0][0] = (0, 0, 0)
        verts[0][1] = (scale, 0, 0)
        verts[1][0] = (0, 0, 0)
        verts[1][1] = (0, scale, 0)
        verts[2][0] = (0, 0, 0)
        verts[2][1] = (0, 0, scale)
        self.verts = verts if pose is None else _transform_verts(verts, pose)
        self._colors = np.empty(3, gymapi.Vec3.dtype)
        self._colors[0] = (1.0, 0.0, 0.0)
        self._colors[1] = (0.0, 1.0, 0.0)
        self._colors[2] = (0.0, 0.0, 1.0)


class WireframeBoxGeometry(LineGeometry):
    def __init__(self, xdim=1, ydim=1, zdim=1, pose=None, color=None):
        x, y, z = 0.5 * xdim, 0.5 * ydim, 0.5 * zdim
        c = [(sx * x, sy * y, sz * z) for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]
        edges = [(0, 1), (2, 3), (4, 5), (6, 7), (0, 2), (1, 3), (4, 6), (5, 7), (0, 4), (1, 5), (2, 6), (3, 7)]
        verts = np.empty((len(edges), 2), gymapi.Vec3.dtype)
        for i, (a, b) in enumerate(edges):
            verts[i][0] = c[a]
            verts[i][1] = c[b]
        self.verts = verts if pose is None else _transform_verts(verts, pose)
        self._colors = np.empty(len(edges), gymapi.Vec3.dtype)
        self._colors[:] = color if color is not None else (1.0, 0.0, 0.0)


class WireframeSphereGeometry(LineGeometry):
    def __init__(self, radius=1.0, num_lats=8, num_lons=8, pose=None, color=None, color2=None):
        color = color if color is not None else (1, 0, 0)
        color2 = color2 if color2 is not None else color
        lines = []
        cols = []
        for i in range(num_lats):
            lat0 = math.pi * (-0.5 + i / num_lats)
            lat1 = math.pi * (-0.5 + (i + 1) / num_lats)
            for j in range(num_lons):
                lon = 2 * math.pi * j / num_lons
                p0 = (radius * math.cos(lat0) * math.cos(lon), radius * math.cos(lat0) * math.sin(lon),
                      radius * math.sin(lat0))
                p1 = (radius * math.cos(lat1) * math.cos(lon), radius * math.cos(lat1) * math.sin(lon),
                      radius * math.sin(lat1))
                lines.append((p0, p1))
                cols.append(color)
                lon1 = 2 * math.pi * (j + 1) / num_lons
                p2 = (radius * math.cos(lat0) * math.cos(lon1), radius * math.cos(lat0) * math.sin(lon1),
                      radius * math.sin(lat0))
                lines.append((p0, p2))
                cols.append(color2)
        verts = np.empty((len(lines), 2), gymapi.Vec3.dtype)
        for i, (a, b) in enumerate(lines):
            verts[i][0] = a
            verts[i][1] = b
        self.verts = verts if pose is None else _transform_verts(verts, pose)
        self._colors = np.empty(len(lines), gymapi.Vec3.dtype)
        for i, c in enumerate(cols):
            self._colors[i] = c


def _transform_verts(verts, pose):
    out = np.empty_like(verts)
    for i in range(verts.shape[0]):
        for k in range(2):
            v = verts[i][k]
            p = pose.transform_point(gymapi.Vec3(v["x"], v["y"], v["z"]))
            out[i][k] = (p.x, p.y, p.z)
    return out


def draw_lines(geom, gym, viewer, env, pose):
    """Headless: validates arguments, draws nothing (test10_servo_vecenv.py:305-306)."""
    return None


def draw_line(p1, p2, color, gym, viewer, env):
    return None


def get_property_setter_map(gym):
    return {}


def get_property_getter_map(gym):
    return {}


def get_default_setter_args(gym):
    return {}
