"""gymapi value types: Vec3 / Quat / Transform, enums, parameter structs and the
structured numpy dtypes of Isaac Gym's non-tensor API.

Semantics follow the reference's usage: examples/maths.py:21-140 (operators,
from_axis_angle, from_euler_zyx / to_euler_zyx, rotate, inverse),
examples/projectiles.py:163-168 (RigidBodyState fields pose.p/r, vel.linear/
angular), test13_camera_spherical_joint.py:118-123 (DOF property fields),
test10_servo_vecenv.py:117-144 (SimParams / PhysXParams fields).
Default values that the reference does not show are Isaac Gym Preview 4's
documented defaults; DESIGN.md §6 lists the ones this build had to assume.
"""
import math

import numpy as np

# ---------------------------------------------------------------- enums
SIM_PHYSX = 0
SIM_FLEX = 1
SimType = int

UP_AXIS_Y = 0
UP_AXIS_Z = 1
UpAxis = int

DOF_MODE_NONE = 0
DOF_MODE_POS = 1
DOF_MODE_VEL = 2
DOF_MODE_EFFORT = 3
DofDriveMode = int

DOF_INVALID = -1
DOF_ROTATION = 0
DOF_TRANSLATION = 1
DofType = int

JOINT_INVALID = -1
JOINT_FIXED = 0
JOINT_REVOLUTE = 1
JOINT_PRISMATIC = 2
JOINT_BALL = 3
JOINT_PLANAR = 4
JOINT_FLOATING = 5
JointType = int

STATE_NONE = 0
STATE_POS = 1
STATE_VEL = 2
STATE_ALL = 3

DOMAIN_ACTOR = 0
DOMAIN_ENV = 1
DOMAIN_SIM = 2

ENV_SPACE = 0
LOCAL_SPACE = 1
GLOBAL_SPACE = 2
CoordinateSpace = int

IMAGE_COLOR = 0
IMAGE_DEPTH = 1
IMAGE_SEGMENTATION = 2
IMAGE_OPTICAL_FLOW = 3
ImageType = int

FOLLOW_POSITION = 0
FOLLOW_TRANSFORM = 1
CameraFollowMode = int

MESH_NONE = 0
MESH_COLLISION = 1
MESH_VISUAL = 2
MESH_VISUAL_AND_COLLISION = 3

# viewer keyboard inputs (gymapi.KeyboardInput; subscribe_viewer_keyboard_event,
# examples/1080_balls_of_solitude.py:88). The viewer is headless and raises no
# events, so only their distinctness matters; the values are this build's.
KeyboardInput = int
KEY_SPACE = 32
KEY_APOSTROPHE, KEY_COMMA, KEY_MINUS, KEY_PERIOD, KEY_SLASH = 39, 44, 45, 46, 47
for _i in range(10):
    globals()["KEY_%d" % _i] = 48 + _i
for _i in range(26):
    globals()["KEY_" + chr(65 + _i)] = 65 + _i
KEY_ESCAPE, KEY_ENTER, KEY_TAB, KEY_BACKSPACE, KEY_INSERT, KEY_DEL = 256, 257, 258, 259, 260, 261
KEY_RIGHT, KEY_LEFT, KEY_DOWN, KEY_UP, KEY_PAGE_UP, KEY_PAGE_DOWN, KEY_HOME, KEY_END = (262, 263, 264, 265, 266,
                                                                                        267, 268, 269)
for _i in range(1, 13):
    globals()["KEY_F%d" % _i] = 289 + _i
KEY_LEFT_SHIFT, KEY_LEFT_CONTROL, KEY_LEFT_ALT, KEY_RIGHT_SHIFT, KEY_RIGHT_CONTROL, KEY_RIGHT_ALT = (340, 341, 342,
                                                                                                    344, 345, 346)
del _i

# viewer mouse inputs (gymapi.MouseInput; subscribe_viewer_mouse_event,
# examples/projectiles.py:68): headless viewer, values this build's
MouseInput = int
(MOUSE_LEFT_BUTTON, MOUSE_RIGHT_BUTTON, MOUSE_MIDDLE_BUTTON, MOUSE_FORWARD_BUTTON, MOUSE_BACK_BUTTON,
 MOUSE_SCROLL_RIGHT, MOUSE_SCROLL_LEFT, MOUSE_SCROLL_UP, MOUSE_SCROLL_DOWN,
 MOUSE_MOVE_RIGHT, MOUSE_MOVE_LEFT, MOUSE_MOVE_UP, MOUSE_MOVE_DOWN) = range(13)


def _enum(name, *members):
    """A pybind11-style enum type over this module's int constants: Isaac Gym
    scripts spell both gymapi.UP_AXIS_Z and gymapi.UpAxis.UP_AXIS_Z
    (examples/test_graphics_up.py:43,108); both are the same int here."""
    g = globals()
    return type(name, (int,), {m: g[m] for m in members})


SimType = _enum("SimType", "SIM_PHYSX", "SIM_FLEX")
UpAxis = _enum("UpAxis", "UP_AXIS_Y", "UP_AXIS_Z")
DofDriveMode = _enum("DofDriveMode", "DOF_MODE_NONE", "DOF_MODE_POS", "DOF_MODE_VEL", "DOF_MODE_EFFORT")
DofType = _enum("DofType", "DOF_INVALID", "DOF_ROTATION", "DOF_TRANSLATION")
JointType = _enum("JointType", "JOINT_INVALID", "JOINT_FIXED", "JOINT_REVOLUTE", "JOINT_PRISMATIC", "JOINT_BALL",
                  "JOINT_PLANAR", "JOINT_FLOATING")
CoordinateSpace = _enum("CoordinateSpace", "ENV_SPACE", "LOCAL_SPACE", "GLOBAL_SPACE")
ImageType = _enum("ImageType", "IMAGE_COLOR", "IMAGE_DEPTH", "IMAGE_SEGMENTATION", "IMAGE_OPTICAL_FLOW")
CameraFollowMode = _enum("CameraFollowMode", "FOLLOW_POSITION", "FOLLOW_TRANSFORM")
KeyboardInput = _enum("KeyboardInput", *[k for k in list(globals()) if k.startswith("KEY_")])
MouseInput = _enum("MouseInput", *[k for k in list(globals()) if k.startswith("MOUSE_")])

RIGID_BODY_NONE = 0
RIGID_BODY_DISABLE_GRAVITY = 1
RIGID_BODY_DISABLE_SIMULATION = 2

AXIS_NONE = 0
AXIS_TRANSLATION = 7
AXIS_ROTATION = 56
AXIS_ALL = 63

FROM_ASSET = 0
COMPUTE_PER_VERTEX = 1
COMPUTE_PER_FACE = 2

DTYPE_FLOAT32 = 0
DTYPE_UINT32 = 1
DTYPE_UINT64 = 2
DTYPE_UINT8 = 3
DTYPE_INT16 = 4

CC_NEVER = 0
CC_LAST_SUBSTEP = 1
CC_ALL_SUBSTEPS = 2

INVALID_HANDLE = -1
DEFAULT_VIEWER_WIDTH = 1600
DEFAULT_VIEWER_HEIGHT = 900

_JOINT_TYPE_STRINGS = {
    JOINT_INVALID: "Invalid", JOINT_FIXED: "Fixed", JOINT_REVOLUTE: "Revolute", JOINT_PRISMATIC: "Prismatic",
    JOINT_BALL: "Ball", JOINT_PLANAR: "Planar", JOINT_FLOATING: "Floating",
}
_DOF_TYPE_STRINGS = {DOF_INVALID: "Invalid", DOF_ROTATION: "Rotation", DOF_TRANSLATION: "Translation"}


# ------------------------------------------------------------- math types
class Vec3:
    dtype = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4")])
    __slots__ = ("x", "y", "z")

    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x = float(x)
        self.y = float(y)
        self.z = float(z)

    def __add__(self, o):
        return Vec3(self.x + o.x, self.y + o.y, self.z + o.z)

    def __sub__(self, o):
        return Vec3(self.x - o.x, self.y - o.y, self.z - o.z)

    def __mul__(self, s):
        return Vec3(self.x * s, self.y * s, self.z * s)

    __rmul__ = __mul__

    def __truediv__(self, s):
        return Vec3(self.x / s, self.y / s, self.z / s)

    def __neg__(self):
        return Vec3(-self.x, -self.y, -self.z)

    def dot(self, o):
        return self.x * o.x + self.y * o.y + self.z * o.z

    def cross(self, o):
        return Vec3(self.y * o.z - self.z * o.y, self.z * o.x - self.x * o.z, self.x * o.y - self.y * o.x)

    def length(self):
        return math.sqrt(self.dot(self))

    def length_sq(self):
        return self.dot(self)

    def normalize(self):
        n = self.length()
        return Vec3(self.x / n, self.y / n, self.z / n) if n > 0 else Vec3()

    def to_numpy(self):
        return np.array([self.x, self.y, self.z], dtype=np.float64)

    @staticmethod
    def from_buffer(buf):
        a = np.asarray(buf).reshape(-1)
        if a.dtype.names:
            return Vec3(a["x"][0], a["y"][0], a["z"][0])
        return Vec3(a[0], a[1], a[2])

    def __repr__(self):
        return "Vec3(%f, %f, %f)" % (self.x, self.y, self.z)

    __str__ = __repr__


class Quat:
    dtype = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("w", "<f4")])
    __slots__ = ("x", "y", "z", "w")

    def __init__(self, x=0.0, y=0.0, z=0.0, w=1.0):
        self.x = float(x)
        self.y = float(y)
        self.z = float(z)
        self.w = float(w)

    def __mul__(self, o):
        a, b = self, o
        return Quat(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
                    a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
                    a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w,
                    a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z)

    def rotate(self, v):
        ux, uy, uz, w = self.x, self.y, self.z, self.w
        tx = 2.0 * (uy * v.z - uz * v.y)
        ty = 2.0 * (uz * v.x - ux * v.z)
        tz = 2.0 * (ux * v.y - uy * v.x)
        return Vec3(v.x + w * tx + (uy * tz - uz * ty),
                    v.y + w * ty + (uz * tx - ux * tz),
                    v.z + w * tz + (ux * ty - uy * tx))

    def inverse(self):
        n2 = self.x * self.x + self.y * self.y + self.z * self.z + self.w * self.w
        return Quat(-self.x / n2, -self.y / n2, -self.z / n2, self.w / n2)

    def normalize(self):
        n = math.sqrt(self.x * self.x + self.y * self.y + self.z * self.z + self.w * self.w)
        if n == 0:
            return Quat()
        return Quat(self.x / n, self.y / n, self.z / n, self.w / n)

    def dot(self, o):
        return self.x * o.x + self.y * o.y + self.z * o.z + self.w * o.w

    @staticmethod
    def from_axis_angle(axis, angle):
        a = axis.normalize()
        s = math.sin(0.5 * angle)
        return Quat(a.x * s, a.y * s, a.z * s, math.cos(0.5 * angle))

    @staticmethod
    def from_euler_zyx(roll, pitch, yaw):
        """Intrinsic z-y-x: R = Rz(yaw) Ry(pitch) Rx(roll) (examples/maths.py:44-51)."""
        cr, sr = math.cos(0.5 * roll), math.sin(0.5 * roll)
        cp, sp = math.cos(0.5 * pitch), math.sin(0.5 * pitch)
        cy, sy = math.cos(0.5 * yaw), math.sin(0.5 * yaw)
        return Quat(sr * cp * cy - cr * sp * sy,
                    cr * sp * cy + sr * cp * sy,
                    cr * cp * sy - sr * sp * cy,
                    cr * cp * cy + sr * sp * sy)

    def to_euler_zyx(self):
        """(roll, pitch, yaw) of R = Rz(yaw) Ry(pitch) Rx(roll) (examples/maths.py:53-60)."""
        x, y, z, w = self.x, self.y, self.z, self.w
        roll = math.atan2(2.0 * (w * x + y * z), 1.0 - 2.0 * (x * x + y * y))
        sp = 2.0 * (w * y - z * x)
        pitch = math.copysign(math.pi / 2.0, sp) if abs(sp) >= 1.0 else math.asin(sp)
        yaw = math.atan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z))
        return roll, pitch, yaw

    def to_numpy(self):
        return np.array([self.x, self.y, self.z, self.w], dtype=np.float64)

    @staticmethod
    def from_buffer(buf):
        a = np.asarray(buf).reshape(-1)
        if a.dtype.names:
            return Quat(a["x"][0], a["y"][0], a["z"][0], a["w"][0])
        return Quat(a[0], a[1], a[2], a[3])

    def __repr__(self):
        return "Quat(%f, %f, %f, %f)" % (self.x, self.y, self.z, self.w)

    __str__ = __repr__


class Transform:
    dtype = np.dtype([("p", Vec3.dtype), ("r", Quat.dtype)])
    __slots__ = ("p", "r")

    def __init__(self, p=None, r=None):
        self.p = Vec3(p.x, p.y, p.z) if p is not None else Vec3()
        self.r = Quat(r.x, r.y, r.z, r.w) if r is not None else Quat()

    def __mul__(self, o):
        return Transform(self.p + self.r.rotate(o.p), self.r * o.r)

    def inverse(self):
        ri = self.r.inverse()
        return Transform(-ri.rotate(self.p), ri)

    def transform_point(self, v):
        return self.p + self.r.rotate(v)

    def transform_vector(self, v):
        return self.r.rotate(v)

    def transform_points(self, pts):
        return np.array([self.transform_point(Vec3(*p)).to_numpy() for p in np.asarray(pts).reshape(-1, 3)])

    @staticmethod
    def from_buffer(buf):
        a = np.asarray(buf).reshape(-1)
        if a.dtype.names:
            return Transform(Vec3(a["p"]["x"][0], a["p"]["y"][0], a["p"]["z"][0]),
                             Quat(a["r"]["x"][0], a["r"]["y"][0], a["r"]["z"][0], a["r"]["w"][0]))
        return Transform(Vec3(a[0], a[1], a[2]), Quat(a[3], a[4], a[5], a[6]))

    def __repr__(self):
        return "Transform(p=%r, r=%r)" % (self.p, self.r)

    __str__ = __repr__


class Velocity:
    dtype = np.dtype([("linear", Vec3.dtype), ("angular", Vec3.dtype)])

    def __init__(self, linear=None, angular=None):
        self.linear = linear if linear is not None else Vec3()
        self.angular = angular if angular is not None else Vec3()


class RigidBodyState:
    dtype = np.dtype([("pose", Transform.dtype), ("vel", Velocity.dtype)])


class DofState:
    dtype = np.dtype([("pos", "<f4"), ("vel", "<f4")])


class DofFrame:
    dtype = np.dtype([("origin", Vec3.dtype), ("axis", Vec3.dtype)])

    def __init__(self, origin=None, axis=None):
        self.origin = origin if origin is not None else Vec3()
        self.axis = axis if axis is not None else Vec3(1, 0, 0)


# structured array returned by get_asset_dof_properties / get_actor_dof_properties
DOF_PROPERTIES_DTYPE = np.dtype([
    ("hasLimits", "?"), ("lower", "<f4"), ("upper", "<f4"), ("driveMode", "<i4"),
    ("velocity", "<f4"), ("effort", "<f4"), ("stiffness", "<f4"), ("damping", "<f4"),
    ("friction", "<f4"), ("armature", "<f4"),
])


class RigidBodyProperties:
    def __init__(self, mass=1.0, com=None, inertia=None, flags=0):
        self.mass = float(mass)
        self.invMass = 1.0 / mass if mass > 0 else 0.0
        self.com = com if com is not None else Vec3()
        self.inertia = inertia if inertia is not None else Mat33()
        self.invInertia = Mat33()
        self.flags = flags


class Mat33:
    def __init__(self, x=None, y=None, z=None):
        self.x = x if x is not None else Vec3(1, 0, 0)
        self.y = y if y is not None else Vec3(0, 1, 0)
        self.z = z if z is not None else Vec3(0, 0, 1)


class RigidShapeProperties:
    def __init__(self):
        self.friction = 1.0
        self.rolling_friction = 0.0
        self.torsion_friction = 0.0
        self.restitution = 0.0
        self.compliance = 0.0
        self.thickness = 0.0
        self.contact_offset = -1.0
        self.rest_offset = -1.0
        self.filter = 0

    def __repr__(self):
        return "RigidShapeProperties(friction=%g, restitution=%g, filter=%d)" % (
            self.friction, self.restitution, self.filter)


# --------------------------------------------------------- parameter structs
class _Params:
    def __repr__(self):
        return "%s(%s)" % (type(self).__name__, ", ".join(
            "%s=%r" % (k, getattr(self, k)) for k in sorted(vars(self))))


class PhysXParams(_Params):
    def __init__(self):
        self.num_threads = 4
        self.solver_type = 1
        self.num_position_iterations = 4
        self.num_velocity_iterations = 1
        self.contact_offset = 0.02
        self.rest_offset = 0.001
        self.bounce_threshold_velocity = 0.2
        self.max_depenetration_velocity = 100.0
        self.default_buffer_size_multiplier = 2.0
        self.max_gpu_contact_pairs = 1024 * 1024
        self.num_subscenes = 0
        self.contact_collection = CC_ALL_SUBSTEPS
        self.use_gpu = False
        self.always_use_articulations = False
        self.friction_offset_threshold = 0.04
        self.friction_correlation_distance = 0.025


class FlexParams(_Params):
    def __init__(self):
        self.solver_type = 5
        self.num_outer_iterations = 4
        self.num_inner_iterations = 15
        self.relaxation = 0.75
        self.warm_start = 0.4
        self.shape_collision_margin = 0.0
        self.shape_collision_distance = 0.0
        self.contact_regularization = 1e-7
        self.deterministic_mode = False
        self.friction_mode = 0
        self.geometric_stiffness = 1.0
        self.max_rigid_contacts = 4096
        self.max_soft_contacts = 4096
        self.dynamic_friction = 0.0
        self.static_friction = 0.0
        self.particle_friction = 0.0
        self.return_contacts = False


class SimParams(_Params):
    def __init__(self):
        self.dt = 1.0 / 60.0
        self.substeps = 2
        self.up_axis = UP_AXIS_Y
        self.gravity = Vec3(0.0, -9.8, 0.0)
        self.num_client_threads = 0
        self.use_gpu_pipeline = False
        self.enable_actor_creation_warning = False
        self.stress_visualization = False
        self.stress_visualization_min = 0.0
        self.stress_visualization_max = 1.0e5
        self.physx = PhysXParams()
        self.flex = FlexParams()


class VhacdParams(_Params):
    def __init__(self):
        self.resolution = 100000
        self.max_convex_hulls = 64
        self.max_num_vertices_per_ch = 64
        self.concavity = 0.0
        self.alpha = 0.05
        self.beta = 0.05
        self.mode = 0
        self.pca = 0
        self.plane_downsampling = 4
        self.convex_hull_downsampling = 4
        self.convex_hull_approximation = True
        self.min_volume_per_ch = 0.0001
        self.ocl_acceleration = True


class AssetOptions(_Params):
    def __init__(self):
        self.angular_damping = 0.5
        self.armature = 0.0
        self.collapse_fixed_joints = False
        self.convex_decomposition_from_submeshes = False
        self.default_dof_drive_mode = DOF_MODE_POS
        self.density = 1000.0
        self.disable_gravity = False
        self.enable_gyroscopic_forces = True
        self.fix_base_link = False
        self.flip_visual_attachments = False
        self.linear_damping = 0.0
        self.max_angular_velocity = 64.0
        self.max_linear_velocity = 1000.0
        self.mesh_normal_mode = FROM_ASSET
        self.min_particle_mass = 1e-12
        self.override_com = False
        self.override_inertia = False
        self.replace_cylinder_with_capsule = False
        self.slices_per_cylinder = 20
        self.tendon_limit_stiffness = 1.0
        self.thickness = 0.02
        self.use_mesh_materials = False
        self.use_physx_armature = True
        self.vhacd_enabled = False
        self.vhacd_params = VhacdParams()


class PlaneParams(_Params):
    def __init__(self):
        self.normal = Vec3(0.0, 1.0, 0.0)
        self.distance = 0.0
        self.static_friction = 1.0
        self.dynamic_friction = 1.0
        self.restitution = 0.0
        self.segmentation_id = 0


class CameraProperties(_Params):
    def __init__(self):
        # Isaac Gym's default sensor size: examples/domain_randomization.py:96-99
        # leaves it unset and its images (examples/dr_output_images) are 1600 x 900
        self.width = 1600
        self.height = 900
        self.horizontal_fov = 90.0
        self.near_plane = 0.1
        self.far_plane = 1000.0
        self.supersampling_horizontal = 1
        self.supersampling_vertical = 1
        self.use_collision_geometry = False
        self.enable_tensors = False


class AttractorProperties(_Params):
    def __init__(self):
        self.axes = AXIS_ALL
        self.damping = 0.0
        self.stiffness = 0.0
        self.offset = Transform()
        self.rigid_handle = INVALID_HANDLE
        self.target = Transform()


class TriangleMeshParams(_Params):
    def __init__(self):
        self.nb_vertices = 0
        self.nb_triangles = 0
        self.static_friction = 1.0
        self.dynamic_friction = 1.0
        self.restitution = 0.0
        self.transform = Transform()
