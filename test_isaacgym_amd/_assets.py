"""Asset import: URDF files and primitive assets, mass properties, body / joint /
DOF ordering.

Reference behaviour this mirrors (SURVEY.md §2 "URDF/MJCF/mesh importer", §8a a10):
  - gym.load_asset(sim, root, file, AssetOptions) -> Asset, or None on failure
    (test10_servo_vecenv.py:230-234);
  - gym.create_box(sim, x, y, z, options) (examples/franka_cube_ik_osc.py:156,161),
    create_sphere / create_capsule;
  - bodies in kinematic-tree (depth-first) order from the root link; children in
    the order their joints are declared. dof_test_camera.urdf declares its links
    out of order (base, camera, camera_y, camera_z) with the tree
    base -> z -> y -> camera (assets/urdf/dof_test_camera.urdf:98-119), so its
    bodies come out [base_link, camera_z_link, camera_y_link, camera_link];
  - a link with no <inertial>, no collision and no visual geometry that hangs on
    a fixed joint is merged into its parent (franka's panda_link8: the Jacobian
    of examples/franka_cube_ik_osc.py:306 has 10 = bodies - 1 rows for a fixed
    base, i.e. 11 bodies);
  - missing mass properties are computed from the collision shapes at
    AssetOptions.density; a mass without an inertia tensor (the UAV and ground
    vehicle, assets/urdf/uav/urdf/rq-1-predator-mae-uav.urdf:4-7) keeps the mass
    and takes the shape inertia scaled to it.
Meshes: a collision mesh that exists becomes its convex hull (MG_SHAPE_CONVEX,
as PhysX cooks a convex mesh from it), reduced to at most HULL_MAX_VERTS (32;
MIGYM_HULL_CAPS per mesh, up to PhysX's 255) vertices by farthest-point sampling of the hull vertices; its mass properties
are the hull's at AssetOptions.density. The servo scene's two meshes are missing
from the reference (.MISSING_LARGE_BLOBS:7-8); they get the frozen box proxies
of MESH_PROXIES, expressed in the body frame.
"""
import math
import os
import xml.etree.ElementTree as ET

import numpy as np

from . import _types as T

# body-frame full extents of the frozen proxies for meshes absent from the reference
MESH_PROXIES = {
    "predator.obj": (16.0, 20.0, 3.0),                 # rq-1-predator, URDF scale 2
    "predator_without_sphere.obj": (16.0, 20.0, 3.0),
    "fusch-apc.obj": (7.5, 3.0, 2.5),                  # tpz-fuchs-apc, URDF scale 0.6
}

SPHERE, BOX, CAPSULE, CONVEX = 0, 1, 2, 3
MJCF_MAX_JOINT_VELOCITY = 100.0      # PhysX's default articulation joint speed limit (rad/s, m/s)
# the importer's default hull size; the library takes hulls up to PhysX's own
# limits (255 vertices / 255 faces: MG_HULL_MAX_VERTS / _FACES, include/migym.h)
HULL_MAX_VERTS, HULL_MAX_FACES = 32, 64
# Per-mesh caps (the Franka hand at 64 vertices and at its
# full 102): MIGYM_HULL_CAPS="hand.obj=64/128,finger.obj=128/255" (mesh file
# name = vertices / faces, each at most 255). Unset: every mesh at the defaults.
HULL_CAPS = {}
for _item in filter(None, os.environ.get("MIGYM_HULL_CAPS", "").split(",")):
    _name, _caps = _item.split("=")
    _v, _f = _caps.split("/")
    HULL_CAPS[_name.strip()] = (min(int(_v), 255), min(int(_f), 255))


def _quat_from_rpy(r, p, y):
    # URDF rpy: fixed-axis roll (x), pitch (y), yaw (z) => R = Rz(y) Ry(p) Rx(r)
    q = T.Quat.from_euler_zyx(r, p, y)
    return np.array([q.x, q.y, q.z, q.w], dtype=np.float64)


def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz])


def _qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _mat_to_quat(R):
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        w = 0.25 * s
        x = (R[2, 1] - R[1, 2]) / s
        y = (R[0, 2] - R[2, 0]) / s
        z = (R[1, 0] - R[0, 1]) / s
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        w = (R[2, 1] - R[1, 2]) / s
        x = 0.25 * s
        y = (R[0, 1] + R[1, 0]) / s
        z = (R[0, 2] + R[2, 0]) / s
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        w = (R[0, 2] - R[2, 0]) / s
        x = (R[0, 1] + R[1, 0]) / s
        y = 0.25 * s
        z = (R[1, 2] + R[2, 1]) / s
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        w = (R[1, 0] - R[0, 1]) / s
        x = (R[0, 2] + R[2, 0]) / s
        y = (R[1, 2] + R[2, 1]) / s
        z = 0.25 * s
    q = np.array([x, y, z, w])
    q = q / np.linalg.norm(q)
    return -q if q[3] < 0 else q


class Hull:
    """Convex hull in its shape frame: vertices (nv, 3), face planes (nf, 4) =
    (unit outward n, d) with n . x <= d inside, and unit-density mass
    properties (volume, centroid, inertia about the centroid)."""

    def __init__(self, verts, planes, volume, com, inertia, edge_list=None):
        self.verts = verts
        self.planes = planes
        self.volume = volume
        self.com = com
        self.inertia = inertia
        self.edge_list = edge_list

    def edges(self):
        """(ne, 2) vertex index pairs of the hull's edges: the triangulation's edges
        whose two triangles lie on different merged face planes (diagonals inside a
        merged face dropped); ascending (i, j)."""
        return self.edge_list if self.edge_list is not None else np.zeros((0, 2), np.int64)

    def record(self):
        """The MG_HULL record (include/migym.h) as float32: header (nv, nf, ne, 0),
        vertices, face planes, edges."""
        E = self.edges()
        head = np.array([len(self.verts), len(self.planes), len(E), 0], dtype=np.float32)
        return np.concatenate([head, self.verts.astype(np.float32).reshape(-1),
                               self.planes.astype(np.float32).reshape(-1), E.astype(np.float32).reshape(-1)])


def _farthest_points(pts, k):
    """k of pts by farthest-point sampling, starting from the point farthest
    from their centroid (deterministic)."""
    c = pts.mean(0)
    idx = [int(np.argmax(((pts - c) ** 2).sum(1)))]
    d2 = ((pts - pts[idx[0]]) ** 2).sum(1)
    while len(idx) < k:
        j = int(np.argmax(d2))
        idx.append(j)
        d2 = np.minimum(d2, ((pts - pts[j]) ** 2).sum(1))
    return pts[sorted(idx)]


def make_hull(verts, max_verts=HULL_MAX_VERTS, max_faces=None):
    """Convex hull of a vertex cloud, at most max_verts vertices; coplanar
    triangles merged into one face plane. Mass properties by tetrahedra from
    the vertex centroid."""
    from scipy.spatial import ConvexHull
    pts = np.unique(np.asarray(verts, dtype=np.float64), axis=0)
    h = ConvexHull(pts)
    pts = pts[h.vertices]
    nv = min(max_verts, len(pts))
    while True:
        cand = _farthest_points(pts, nv) if len(pts) > nv else pts
        h = ConvexHull(cand)
        hv = cand[np.sort(h.vertices)]
        h = ConvexHull(hv)
        planes, tri_plane = [], []
        for eq in h.equations:                     # n . x + e <= 0 inside
            n, d = eq[:3], -eq[3]
            match = [k for k, q in enumerate(planes) if abs(np.dot(n, q[:3]) - 1.0) < 1e-6 and abs(d - q[3]) < 1e-6]
            if not match:
                planes.append(np.array([n[0], n[1], n[2], d]))
            tri_plane.append(match[0] if match else len(planes) - 1)
        if len(planes) <= (HULL_MAX_FACES if max_faces is None else max_faces) or nv <= 8:
            break
        nv -= 2
    o = hv.mean(0)
    vol, mom1, C = 0.0, np.zeros(3), np.zeros((3, 3))
    for tri in h.simplices:
        a, b, c = hv[tri[0]] - o, hv[tri[1]] - o, hv[tri[2]] - o
        d6 = abs(float(np.dot(a, np.cross(b, c))))
        s = a + b + c
        vol += d6 / 6.0
        mom1 += d6 / 6.0 * s / 4.0
        C += d6 / 120.0 * (np.outer(a, a) + np.outer(b, b) + np.outer(c, c) + np.outer(s, s))
    r = mom1 / vol
    I_o = np.trace(C) * np.eye(3) - C
    I_c = I_o - vol * (np.dot(r, r) * np.eye(3) - np.outer(r, r))
    inc = {}                                       # triangulation edge -> merged planes of its triangles
    for t, tri in enumerate(h.simplices):
        for u, v in ((tri[0], tri[1]), (tri[1], tri[2]), (tri[2], tri[0])):
            inc.setdefault((min(u, v), max(u, v)), set()).add(tri_plane[t])
    edges = np.array(sorted(e for e, ps in inc.items() if len(ps) > 1), dtype=np.int64).reshape(-1, 2)
    return Hull(hv, np.array(planes), vol, r + o, I_c, edges)


class Shape:
    __slots__ = ("type", "size", "p", "q", "friction", "restitution", "source", "hull", "density")

    def __init__(self, type_, size, p=None, q=None, source="primitive", hull=None):
        self.type = type_
        self.size = tuple(float(s) for s in size)
        self.p = np.zeros(3) if p is None else np.asarray(p, dtype=np.float64)
        self.q = np.array([0, 0, 0, 1.0]) if q is None else np.asarray(q, dtype=np.float64)
        self.friction = 1.0
        self.restitution = 0.0
        self.source = source
        self.hull = hull
        self.density = None

    def com_body(self):
        """Centroid of the shape in the body frame."""
        if self.type == CONVEX:
            return self.p + _qmat(self.q) @ self.hull.com
        return self.p

    def volume(self):
        if self.type == CONVEX:
            return self.hull.volume
        if self.type == BOX:
            return 8.0 * self.size[0] * self.size[1] * self.size[2]
        if self.type == SPHERE:
            return 4.0 / 3.0 * math.pi * self.size[0] ** 3
        r, hh = self.size[0], self.size[1]
        return math.pi * r * r * 2.0 * hh + 4.0 / 3.0 * math.pi * r ** 3

    def inertia_unit_mass(self):
        """Rotational inertia about the shape centroid, shape frame, per unit mass."""
        if self.type == CONVEX:
            return self.hull.inertia / self.hull.volume
        if self.type == BOX:
            a, b, c = (2 * s for s in self.size)
            return np.diag([(b * b + c * c) / 12.0, (a * a + c * c) / 12.0, (a * a + b * b) / 12.0])
        if self.type == SPHERE:
            r = self.size[0]
            return np.eye(3) * 0.4 * r * r
        # capsule along x: cylinder (length 2hh) + two hemispheres
        r, hh = self.size[0], self.size[1]
        L = 2.0 * hh
        vc = math.pi * r * r * L
        vs = 4.0 / 3.0 * math.pi * r ** 3
        mc, ms = vc / (vc + vs), vs / (vc + vs)
        ix = mc * 0.5 * r * r + ms * 0.4 * r * r
        iy = mc * (L * L / 12.0 + 0.25 * r * r) + ms * (0.4 * r * r + L * L / 4.0 + 3.0 * L * r / 8.0)
        return np.diag([ix, iy, iy])


class Body:
    def __init__(self, name):
        self.name = name
        self.mass = None          # from <inertial>
        self.com = np.zeros(3)
        self.inertia = None       # 3x3 about COM, link frame
        self.has_inertial = False
        self.has_visual = False
        self.shapes = []


class Joint:
    def __init__(self, name, jtype, parent, child):
        self.name = name
        self.type = jtype
        self.parent = parent      # body index (after ordering)
        self.child = child
        self.p = np.zeros(3)
        self.q = np.array([0, 0, 0, 1.0])
        self.axis = np.array([1.0, 0, 0])
        self.has_limits = False
        self.lower = 0.0
        self.upper = 0.0
        self.effort = 0.0
        self.velocity = 0.0
        self.damping = 0.0
        self.friction = 0.0
        self.armature = None      # per-joint armature (MJCF), else AssetOptions.armature
        # hinges applied before this one on the same body (an MJCF body with
        # several joints, assets/mjcf/nv_humanoid.xml:53-54): each its own DOF,
        # about its axis in the body frame as rotated by the hinges before it;
        # they share this joint's origin (p, q)
        self.pre = []

    @property
    def has_dof(self):
        return self.ndof > 0

    @property
    def own_ndof(self):
        """DOFs of the joint itself: 1 revolute / prismatic, 3 spherical (rotations
        about the joint frame's x, y, z axes), 0 otherwise."""
        if self.type in (T.JOINT_REVOLUTE, T.JOINT_PRISMATIC):
            return 1
        return 3 if self.type == T.JOINT_BALL else 0

    @property
    def ndof(self):
        """DOFs between the body and its parent: the pre-hinges' and its own."""
        return len(self.pre) + self.own_ndof

    @property
    def chain(self):
        """The joints a body hangs by, in application (and DOF) order."""
        return self.pre + [self]


class MassProps:
    __slots__ = ("mass", "com", "inertia")

    def __init__(self, mass, com, inertia):
        self.mass = float(mass)
        self.com = np.asarray(com, dtype=np.float64)
        self.inertia = np.asarray(inertia, dtype=np.float64)

    def principal(self):
        """(inv_mass, inv principal moments[3], principal frame quat xyzw)."""
        I = 0.5 * (self.inertia + self.inertia.T)
        w, V = np.linalg.eigh(I)
        if np.linalg.det(V) < 0:
            V[:, 2] = -V[:, 2]
        q = _mat_to_quat(V)
        invm = 1.0 / self.mass if self.mass > 0 else 0.0
        invI = np.array([1.0 / x if x > 1e-12 else 0.0 for x in w])
        return invm, invI, q


class Asset:
    """A loaded asset: bodies in tree order, one joint per non-root body."""

    def __init__(self, name, options):
        self.name = name
        self.options = options
        self.bodies = []
        self.joints = []          # joints[k] attaches bodies[k + 1] (tree order)
        self.mass_props = []
        self.dof_props = None
        self.shape_props = []

    # ---- derived structure
    @property
    def api_joints(self):
        """Joints as the joint API lists them (get_asset_joint_*): every joint of
        every body, a multi-joint MJCF body's hinges one by one."""
        return [c for j in self.joints for c in j.chain]

    @property
    def dof_joints(self):
        """The joint of every DOF, in DOF order (a spherical joint three times)."""
        return [c for j in self.joints for c in j.chain for _ in range(c.own_ndof)]

    @property
    def dof_names(self):
        """DOF names: the joint's name; a spherical joint's three DOFs get
        `<joint>_0/_1/_2` (x, y, z of its frame; naming unpinned by the reference)."""
        out = []
        for c in self.api_joints:
            if c.own_ndof == 1:
                out.append(c.name)
            else:
                out.extend("%s_%d" % (c.name, k) for k in range(c.own_ndof))
        return out

    @property
    def num_dofs(self):
        return sum(j.ndof for j in self.joints)

    def dof_of_body(self, b):
        """first local DOF driven by body b's joint, or -1."""
        if b == 0:
            return -1
        d = 0
        for k, j in enumerate(self.joints):
            if k + 1 == b:
                return d if j.has_dof else -1
            d += j.ndof
        return -1

    @property
    def is_articulation(self):
        return len(self.bodies) > 1 or self.options.fix_base_link

    def finalize(self):
        opts = self.options
        self.mass_props = [compute_mass_props(b, opts.density) for b in self.bodies]
        n = self.num_dofs
        props = np.zeros(n, dtype=T.DOF_PROPERTIES_DTYPE)
        for d, j in enumerate(self.dof_joints):
            props[d]["hasLimits"] = j.has_limits
            props[d]["lower"] = j.lower
            props[d]["upper"] = j.upper
            props[d]["driveMode"] = opts.default_dof_drive_mode
            props[d]["velocity"] = j.velocity
            props[d]["effort"] = j.effort
            props[d]["stiffness"] = 0.0
            props[d]["damping"] = j.damping
            props[d]["friction"] = j.friction
            props[d]["armature"] = opts.armature if j.armature is None else j.armature
        self.dof_props = props
        self.shape_props = []
        for b in self.bodies:
            for s in b.shapes:
                sp = T.RigidShapeProperties()
                sp.friction = s.friction
                sp.restitution = s.restitution
                self.shape_props.append(sp)
        return self


def compute_mass_props(body, density):
    """Mass, COM and inertia about the COM (link frame) of a body."""
    shapes = body.shapes
    vols = [s.volume() for s in shapes]
    vtot = sum(vols)
    if body.has_inertial and body.inertia is not None and body.mass is not None:
        return MassProps(body.mass, body.com, body.inertia)
    if vtot > 0:
        m_shape = density * vtot
        com = sum(s.com_body() * v for s, v in zip(shapes, vols)) / vtot
        I = np.zeros((3, 3))
        for s, v in zip(shapes, vols):
            ms = density * v
            R = _qmat(s.q)
            Ic = R @ (s.inertia_unit_mass() * ms) @ R.T
            d = s.com_body() - com
            I += Ic + ms * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        if body.mass is not None:             # mass given, inertia missing: scale the shape inertia
            scale = body.mass / m_shape
            com_out = body.com if body.has_inertial else com
            return MassProps(body.mass, com_out, I * scale)
        return MassProps(m_shape, com, I)
    mass = body.mass if body.mass is not None else 1.0
    return MassProps(mass, body.com, np.eye(3) * 0.01 * mass)


# ------------------------------------------------------------------ primitives
def _primitive_asset(name, shape, options):
    a = Asset(name, options)
    b = Body(name)
    b.shapes.append(shape)
    b.has_visual = True
    a.bodies.append(b)
    return a.finalize()


def create_box(width, height, depth, options):
    return _primitive_asset("box", Shape(BOX, (0.5 * width, 0.5 * height, 0.5 * depth)), options)


def create_sphere(radius, options):
    return _primitive_asset("sphere", Shape(SPHERE, (radius,)), options)


def create_capsule(radius, length, options):
    return _primitive_asset("capsule", Shape(CAPSULE, (radius, 0.5 * length)), options)


# ------------------------------------------------------------------ meshes
def _mesh_vertices(path):
    ext = os.path.splitext(path)[1].lower()
    if ext == ".obj":
        vs = []
        with open(path, "r", errors="ignore") as f:
            for line in f:
                if line.startswith("v "):
                    parts = line.split()
                    vs.append([float(parts[1]), float(parts[2]), float(parts[3])])
        return np.array(vs, dtype=np.float64).reshape(-1, 3)
    if ext == ".stl":
        with open(path, "rb") as f:
            data = f.read()
        if data[:5].lower() == b"solid" and b"facet" in data[:400]:
            vs = [[float(t) for t in ln.split()[1:4]] for ln in data.decode(errors="ignore").splitlines()
                  if ln.strip().startswith("vertex")]
            return np.array(vs, dtype=np.float64).reshape(-1, 3)
        n = int(np.frombuffer(data[80:84], dtype="<u4")[0])
        rec = np.frombuffer(data[84:84 + 50 * n], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)),
                                                                   ("a", "<u2")]))
        return rec["v"].reshape(-1, 3).astype(np.float64)
    if ext == ".dae":
        return _collada_vertices(path)
    return np.zeros((0, 3))


def _collada_vertices(path):
    """Vertex positions of a COLLADA (.dae) file in metres: every <geometry>
    mesh's POSITION source, placed by the <visual_scene> nodes that instance it
    (<matrix> / <translate> / <rotate> / <scale>, composed down the node tree;
    a geometry no node instances is taken as is), times <asset><unit meter>.
    A Y_UP file is turned to Z_UP (y -> z), as URDF meshes are z-up. Only the
    vertices matter: the importer reduces a collision mesh to its convex hull."""
    import xml.etree.ElementTree as ET
    root = ET.parse(path).getroot()

    def tag(el):
        return el.tag.rsplit("}", 1)[-1]

    def kids(el, name):
        return [c for c in el if tag(c) == name]

    def floats(el):
        return np.array([float(t) for t in (el.text or "").split()], dtype=np.float64)

    unit, up = 1.0, "Z_UP"
    for a in kids(root, "asset"):
        for u in kids(a, "unit"):
            unit = float(u.get("meter", "1"))
        for ua in kids(a, "up_axis"):
            up = (ua.text or "Z_UP").strip()
    geoms = {}
    for lib in kids(root, "library_geometries"):
        for g in kids(lib, "geometry"):
            for mesh in kids(g, "mesh"):
                srcs = {}
                for src in kids(mesh, "source"):
                    for fa in kids(src, "float_array"):
                        srcs[src.get("id")] = floats(fa)
                pos = None
                for vx in kids(mesh, "vertices"):
                    for inp in kids(vx, "input"):
                        if inp.get("semantic") == "POSITION":
                            pos = srcs.get(inp.get("source", "").lstrip("#"))
                if pos is not None and len(pos) >= 3:
                    geoms[g.get("id")] = pos[:len(pos) // 3 * 3].reshape(-1, 3)

    def node_matrix(node):
        M = np.eye(4)
        for c in node:
            t = tag(c)
            if t == "matrix":
                M = M @ floats(c).reshape(4, 4)
            elif t == "translate":
                T4 = np.eye(4)
                T4[:3, 3] = floats(c)[:3]
                M = M @ T4
            elif t == "scale":
                M = M @ np.diag(list(floats(c)[:3]) + [1.0])
            elif t == "rotate":
                ax, ang = floats(c)[:3], math.radians(floats(c)[3])
                n = np.linalg.norm(ax)
                if n > 0:
                    x, y, z = ax / n
                    cth, sth = math.cos(ang), math.sin(ang)
                    R = np.array([[cth + x * x * (1 - cth), x * y * (1 - cth) - z * sth, x * z * (1 - cth) + y * sth],
                                  [y * x * (1 - cth) + z * sth, cth + y * y * (1 - cth), y * z * (1 - cth) - x * sth],
                                  [z * x * (1 - cth) - y * sth, z * y * (1 - cth) + x * sth, cth + z * z * (1 - cth)]])
                    R4 = np.eye(4)
                    R4[:3, :3] = R
                    M = M @ R4
        return M

    out, used = [], set()

    def visit(node, M):
        M = M @ node_matrix(node)
        for ig in kids(node, "instance_geometry"):
            gid = ig.get("url", "").lstrip("#")
            if gid in geoms:
                v = geoms[gid]
                out.append(v @ M[:3, :3].T + M[:3, 3])
                used.add(gid)
        for c in kids(node, "node"):
            visit(c, M)

    for lib in kids(root, "library_visual_scenes"):
        for vs in kids(lib, "visual_scene"):
            for nd in kids(vs, "node"):
                visit(nd, np.eye(4))
    for gid, v in geoms.items():
        if gid not in used:
            out.append(v)
    if not out:
        return np.zeros((0, 3))
    v = np.concatenate(out, 0) * unit
    if up == "Y_UP":
        v = np.stack([v[:, 0], -v[:, 2], v[:, 1]], 1)
    return v


_HULL_CACHE = {}


def mesh_shape(verts, p, q, source):
    """A collision mesh (vertices in the geometry frame p, q) as a convex-hull
    shape whose origin is the hull's box centre; None for a degenerate mesh."""
    caps = HULL_CAPS.get(os.path.basename(str(source).split(":")[-1]), (HULL_MAX_VERTS, None))
    key = (np.asarray(verts, dtype=np.float64).tobytes(), caps)
    hull = _HULL_CACHE.get(key)
    if hull is None:
        try:
            hull = make_hull(verts, caps[0], caps[1])
        except Exception:                 # flat / degenerate cloud (scipy QhullError)
            return None
        c = 0.5 * (hull.verts.min(0) + hull.verts.max(0))
        hull = Hull(hull.verts - c, np.concatenate([hull.planes[:, :3], hull.planes[:, 3:] -
                                                    hull.planes[:, :3] @ c[:, None]], 1),
                    hull.volume, hull.com - c, hull.inertia, hull.edge_list)
        hull.box_centre = c
        _HULL_CACHE[key] = hull
    brad = float(np.sqrt((hull.verts ** 2).sum(1).max()))
    return Shape(CONVEX, (brad,), np.asarray(p) + _qmat(q) @ hull.box_centre, q, source, hull)


_DECOMP_CACHE = {}


def _decomposed_shapes(path, scale, p, q, params, base):
    """AssetOptions.vhacd_enabled: the mesh as several convex hulls
    (_decomp.decompose with the VhacdParams' hull budget, voxel resolution,
    concavity and minimum piece volume), or [] when the file has no triangles
    (the caller then takes the single hull)."""
    from . import _decomp
    key = (os.path.abspath(path), os.path.getmtime(path), tuple(np.asarray(scale, float)),
           int(params.max_convex_hulls), int(params.resolution), float(params.concavity),
           float(params.min_volume_per_ch))
    pts = _DECOMP_CACHE.get(key)
    if pts is None:
        tm = _decomp.mesh_triangles(path)
        if tm is None or len(tm[1]) == 0:
            return []
        v, f = tm
        pts = _decomp.decompose(v * scale, f, max_convex_hulls=int(params.max_convex_hulls),
                                resolution=int(params.resolution), concavity=float(params.concavity),
                                min_volume_per_ch=float(params.min_volume_per_ch))
        _DECOMP_CACHE[key] = pts
    out = []
    for k, pc in enumerate(pts):
        sh = mesh_shape(pc, p, q, "vhacd:%s#%d" % (base, k)) if len(pc) >= 4 else None
        if sh is not None:
            out.append(sh)
    return out


def _resolve(filename, urdf_dir, asset_root):
    if filename.startswith("package://"):
        rest = filename[len("package://"):]
        d = urdf_dir
        for _ in range(6):
            cand = os.path.join(d, rest)
            if os.path.exists(cand):
                return cand
            parent = os.path.dirname(d)
            cand = os.path.join(parent, rest)
            if os.path.exists(cand):
                return cand
            if parent == d:
                break
            d = parent
        return os.path.join(asset_root, rest)
    if filename.startswith("file://"):
        filename = filename[len("file://"):]
    return filename if os.path.isabs(filename) else os.path.join(urdf_dir, filename)


def _floats(s, n, default):
    if s is None:
        return list(default)
    v = [float(t) for t in s.split()]
    return v if len(v) == n else list(default)


def _origin(el):
    o = el.find("origin") if el is not None else None
    if o is None:
        return np.zeros(3), np.array([0, 0, 0, 1.0])
    xyz = _floats(o.get("xyz"), 3, (0, 0, 0))
    rpy = _floats(o.get("rpy"), 3, (0, 0, 0))
    return np.array(xyz, dtype=np.float64), _quat_from_rpy(*rpy)


def _geometry_shapes(col, urdf_dir, asset_root, options, warnings):
    geo = col.find("geometry")
    if geo is None:
        return []
    p, q = _origin(col)
    out = []
    for g in geo:
        if g.tag == "box":
            sx, sy, sz = _floats(g.get("size"), 3, (1, 1, 1))
            out.append(Shape(BOX, (0.5 * sx, 0.5 * sy, 0.5 * sz), p, q, "box"))
        elif g.tag == "sphere":
            out.append(Shape(SPHERE, (float(g.get("radius", 1.0)),), p, q, "sphere"))
        elif g.tag == "cylinder":
            r, l = float(g.get("radius", 1.0)), float(g.get("length", 1.0))
            if options.replace_cylinder_with_capsule:
                # URDF cylinders run along z, capsules along x
                qc = _qmul(q, _quat_from_rpy(0.0, -0.5 * math.pi, 0.0))
                out.append(Shape(CAPSULE, (r, max(0.5 * l - r, 0.0)), p, qc, "cylinder->capsule"))
            else:
                out.append(Shape(BOX, (r, r, 0.5 * l), p, q, "cylinder->box"))
        elif g.tag == "mesh":
            fn = g.get("filename", "")
            scale = _floats(g.get("scale"), 3, (1, 1, 1))
            path = _resolve(fn, urdf_dir, asset_root)
            base = os.path.basename(fn)
            if os.path.exists(path):
                if getattr(options, "vhacd_enabled", False):
                    pieces = _decomposed_shapes(path, np.array(scale), p, q, options.vhacd_params, base)
                    if pieces:
                        out.extend(pieces)
                        continue
                vs = _mesh_vertices(path) * np.array(scale)
                sh = mesh_shape(vs, p, q, "mesh-hull:" + base) if len(vs) >= 4 else None
                if sh is not None:
                    out.append(sh)
                else:
                    warnings.append("mesh %s has no volume" % fn)
            elif base in MESH_PROXIES:
                ex = MESH_PROXIES[base]
                out.append(Shape(BOX, (0.5 * ex[0], 0.5 * ex[1], 0.5 * ex[2]), None, None, "proxy:" + base))
            else:
                warnings.append("mesh %s not found; shape skipped" % fn)
    return out


_URDF_JOINT = {"revolute": T.JOINT_REVOLUTE, "continuous": T.JOINT_REVOLUTE, "prismatic": T.JOINT_PRISMATIC,
               "fixed": T.JOINT_FIXED, "floating": T.JOINT_FLOATING, "planar": T.JOINT_PLANAR,
               "spherical": T.JOINT_BALL}


def load_urdf(asset_root, filename, options):
    path = filename if os.path.isabs(filename) else os.path.join(asset_root, filename)
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    root = ET.parse(path).getroot()
    urdf_dir = os.path.dirname(os.path.abspath(path))
    warnings = []
    links = {}
    order = []
    for le in root.findall("link"):
        b = Body(le.get("name"))
        ine = le.find("inertial")
        if ine is not None:
            b.has_inertial = True
            p, q = _origin(ine)
            b.com = p
            m = ine.find("mass")
            if m is not None:
                b.mass = float(m.get("value", 0.0))
            it = ine.find("inertia")
            if it is not None:
                g = lambda k: float(it.get(k, 0.0))  # noqa: E731
                I = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")],
                              [g("ixz"), g("iyz"), g("izz")]])
                R = _qmat(q)
                b.inertia = R @ I @ R.T
        b.has_visual = le.find("visual") is not None
        for col in le.findall("collision"):
            b.shapes.extend(_geometry_shapes(col, urdf_dir, asset_root, options, warnings))
        links[b.name] = b
        order.append(b.name)

    joints = []
    for je in root.findall("joint"):
        jt = _URDF_JOINT.get(je.get("type", "fixed"), T.JOINT_FIXED)
        parent = je.find("parent").get("link")
        child = je.find("child").get("link")
        j = Joint(je.get("name"), jt, parent, child)
        j.p, j.q = _origin(je)
        ax = je.find("axis")
        if ax is not None:
            a = np.array(_floats(ax.get("xyz"), 3, (1, 0, 0)))
            n = np.linalg.norm(a)
            j.axis = a / n if n > 0 else np.array([1.0, 0, 0])
        lim = je.find("limit")
        if lim is not None:
            j.effort = float(lim.get("effort", 0.0))
            j.velocity = float(lim.get("velocity", 0.0))
            if je.get("type") in ("revolute", "prismatic"):
                j.has_limits = True
                j.lower = float(lim.get("lower", 0.0))
                j.upper = float(lim.get("upper", 0.0))
        dyn = je.find("dynamics")
        if dyn is not None:
            j.damping = float(dyn.get("damping", 0.0))
            j.friction = float(dyn.get("friction", 0.0))
        joints.append(j)

    # merge empty links hanging on fixed joints (and all fixed joints if collapse_fixed_joints)
    changed = True
    while changed:
        changed = False
        for j in joints:
            if j.type != T.JOINT_FIXED:
                continue
            c = links[j.child]
            empty = not c.has_inertial and not c.shapes and not c.has_visual
            if not (empty or options.collapse_fixed_joints):
                continue
            par = links[j.parent]
            R = _qmat(j.q)
            for s in c.shapes:
                s.p = j.p + R @ s.p
                s.q = _qmul(j.q, s.q)
                par.shapes.append(s)
            if c.has_inertial and c.mass:
                mp_p = compute_mass_props(par, options.density)
                mp_c = compute_mass_props(c, options.density)
                cc = j.p + R @ mp_c.com
                Ic = R @ mp_c.inertia @ R.T
                M = mp_p.mass + mp_c.mass
                com = (mp_p.com * mp_p.mass + cc * mp_c.mass) / M
                I = np.zeros((3, 3))
                for (mm, cm, Im) in ((mp_p.mass, mp_p.com, mp_p.inertia), (mp_c.mass, cc, Ic)):
                    d = cm - com
                    I += Im + mm * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
                par.mass, par.com, par.inertia, par.has_inertial = M, com, I, True
            for k in joints:
                if k.parent == c.name:
                    k.p = j.p + R @ k.p
                    k.q = _qmul(j.q, k.q)
                    k.parent = j.parent
            joints.remove(j)
            order.remove(c.name)
            del links[c.name]
            changed = True
            break

    children = {n: [] for n in order}
    is_child = set()
    for j in joints:
        children[j.parent].append(j)
        is_child.add(j.child)
    roots = [n for n in order if n not in is_child]
    if len(roots) != 1:
        raise ValueError("URDF %s: expected one root link, found %s" % (path, roots))

    asset = Asset(root.get("name", os.path.basename(path)), options)
    index = {}

    def visit(name, via):
        index[name] = len(asset.bodies)
        asset.bodies.append(links[name])
        if via is not None:
            asset.joints.append(via)
        for j in children[name]:
            visit(j.child, j)

    visit(roots[0], None)
    for j in asset.joints:
        j.parent = index[j.parent]
        j.child = index[j.child]
    asset.warnings = warnings
    asset.path = path
    return asset.finalize()


# ------------------------------------------------------------------ MJCF
def _mj_floats(s, default=None):
    if s is None:
        return None if default is None else list(default)
    return [float(t) for t in s.split()]


def _mj_quat(el, angle_deg, default=None):
    """Orientation of an MJCF element as xyzw: quat (MJCF order w x y z), axisangle,
    euler (xyz, the MJCF default eulerseq) or zaxis; identity if none."""
    q = _mj_floats(el.get("quat"))
    if q is not None:
        v = np.array([q[1], q[2], q[3], q[0]])
        return v / np.linalg.norm(v)
    aa = _mj_floats(el.get("axisangle"))
    k = math.pi / 180.0 if angle_deg else 1.0
    if aa is not None:
        ax = np.array(aa[:3]) / np.linalg.norm(aa[:3])
        h = 0.5 * aa[3] * k
        return np.array([*(ax * math.sin(h)), math.cos(h)])
    eu = _mj_floats(el.get("euler"))
    if eu is not None:
        q = np.array([0, 0, 0, 1.0])
        for i, a in enumerate(eu):                  # intrinsic x, y, z
            ax = np.zeros(3)
            ax[i] = 1.0
            h = 0.5 * a * k
            q = _qmul(q, np.array([*(ax * math.sin(h)), math.cos(h)]))
        return q
    za = _mj_floats(el.get("zaxis"))
    if za is not None:
        z = np.array(za) / np.linalg.norm(za)
        return _quat_between(np.array([0, 0, 1.0]), z)
    return np.array([0, 0, 0, 1.0]) if default is None else default


def _quat_between(a, b):
    """Shortest-arc rotation taking unit vector a to unit vector b (xyzw)."""
    c = float(np.dot(a, b))
    if c < -0.999999:
        ax = np.cross(a, [1.0, 0, 0])
        if np.linalg.norm(ax) < 1e-6:
            ax = np.cross(a, [0, 1.0, 0])
        ax /= np.linalg.norm(ax)
        return np.array([*ax, 0.0])
    v = np.cross(a, b)
    q = np.array([v[0], v[1], v[2], 1.0 + c])
    return q / np.linalg.norm(q)


def _mj_expand_includes(el, base_dir, depth=0):
    """MJCF <include file="..."/> (open_ai_assets/hand/shadow_hand.xml:8-15): the
    included file's top-level children (its root is a <mujoco> element) replace
    the include element in place, recursively, paths relative to the including
    file."""
    if depth > 16:
        raise ValueError("MJCF: <include> nested deeper than 16 levels")
    out = []
    for child in list(el):
        if child.tag == "include":
            path = os.path.join(base_dir, child.get("file", ""))
            inc = ET.parse(path).getroot()
            _mj_expand_includes(inc, os.path.dirname(path), depth + 1)
            out.extend(list(inc))
        else:
            _mj_expand_includes(child, base_dir, depth)
            out.append(child)
    el[:] = out


class _MjDefaults:
    """<default> attribute sets: the top level and named classes (one level of
    nesting inherits from its parent class)."""

    def __init__(self, root):
        self.cls = {}
        d = root.find("default")
        if d is not None:
            self._read(d, "main", {})

    def _read(self, el, name, inherit):
        cur = {k: dict(v) for k, v in inherit.items()}
        for child in el:
            if child.tag == "default":
                continue
            cur.setdefault(child.tag, {}).update(child.attrib)
        self.cls[name] = cur
        for child in el.findall("default"):
            self._read(child, child.get("class", name), cur)

    def attrs(self, el, cls):
        base = dict(self.cls.get(cls, self.cls.get("main", {})).get(el.tag, {}))
        base.update(el.attrib)
        return base


def _mj_geom_shape(g, angle_deg, warnings):
    """One MJCF geom as a Shape (body frame), or None (planes, meshes)."""
    t = g.get("type", "sphere")
    size = _mj_floats(g.get("size"), (0.0,))
    fromto = _mj_floats(g.get("fromto"))
    p = np.array(_mj_floats(g.get("pos"), (0, 0, 0)), dtype=np.float64)
    q = _mj_quat(_Attr(g), angle_deg)
    if t in ("capsule", "cylinder"):
        if t == "cylinder":
            warnings.append("MJCF cylinder geom %s represented as a capsule" % g.get("name"))
        r = size[0]
        if fromto is not None:
            a, b = np.array(fromto[:3]), np.array(fromto[3:6])
            d = b - a
            ln = float(np.linalg.norm(d))
            p = 0.5 * (a + b)
            q = _quat_between(np.array([1.0, 0, 0]), d / ln) if ln > 0 else np.array([0, 0, 0, 1.0])
            hh = 0.5 * ln
        else:
            hh = size[1] if len(size) > 1 else 0.0
            q = _qmul(q, _quat_between(np.array([1.0, 0, 0]), np.array([0, 0, 1.0])))   # MJCF axis: local z
        return Shape(CAPSULE, (r, hh), p, q, source="mjcf:" + t)
    if t == "sphere":
        return Shape(SPHERE, (size[0],), p, q, source="mjcf:sphere")
    if t == "box":
        if fromto is not None:
            warnings.append("MJCF box %s: fromto ignored" % g.get("name"))
        return Shape(BOX, tuple(size[:3]), p, q, source="mjcf:box")
    if t != "plane":
        warnings.append("MJCF geom type %s (%s) skipped" % (t, g.get("name")))
    return None


class _Attr:
    """An element view over merged (default + own) attributes."""

    def __init__(self, attrs):
        self._a = attrs if isinstance(attrs, dict) else dict(attrs.attrib) if hasattr(attrs, "attrib") else attrs

    def get(self, k, d=None):
        return self._a.get(k, d)


def load_mjcf(asset_root, filename, options):
    """MuJoCo MJCF import (assets/mjcf/nv_ant.xml, examples/apply_forces.py:67):
    the body tree under <worldbody>, hinge / slide / ball joints (several hinges
    per body as a chain, nv_humanoid.xml:53-54; angles in degrees unless
    <compiler angle="radian">), a <freejoint> / free joint on the
    root (a floating base unless AssetOptions.fix_base_link), sphere / capsule /
    box geoms (fromto capsules; cylinders as capsules), mass properties from the
    geoms at their density (default 1000) unless the body has an <inertial>,
    geom friction (sliding coefficient), joint range / damping / armature, and
    motor actuators' gear x ctrlrange as the DOF effort limit. World geoms (the
    floor plane) are not part of the asset. A hinge whose anchor is off the body
    origin moves the child frame to the anchor (geoms and children re-expressed)."""
    path = filename if os.path.isabs(filename) else os.path.join(asset_root, filename)
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    root = ET.parse(path).getroot()
    _mj_expand_includes(root, os.path.dirname(path))
    comp = root.find("compiler")
    angle_deg = comp is None or comp.get("angle", "degree") != "radian"
    k_ang = math.pi / 180.0 if angle_deg else 1.0
    defaults = _MjDefaults(root)
    warnings = []
    # elements that would change the dynamics but are not modelled: said, not dropped silently
    for tag, what in (("tendon", "tendons"), ("equality", "equality constraints")):
        el = root.find(tag)
        if el is not None and len(el):
            warnings.append("MJCF %s: %d %s not modelled" % (os.path.basename(path), len(el), what))
    wb = root.find("worldbody")
    if wb is None:
        raise ValueError("MJCF %s: no <worldbody>" % path)
    tops = wb.findall("body")
    if len(tops) != 1:
        raise ValueError("MJCF %s: expected one top-level body, found %d" % (path, len(tops)))
    asset = Asset(root.get("model", os.path.basename(path)), options)
    joint_of_name = {}

    def geom_shapes(bel, cls, shift):
        out = []
        for g in bel.findall("geom"):
            ga = defaults.attrs(g, g.get("class", cls))
            sh = _mj_geom_shape(_Attr(ga), angle_deg, warnings)
            if sh is None:
                continue
            sh.p = sh.p - shift
            fr = _mj_floats(ga.get("friction"))
            if fr:
                sh.friction = fr[0]
            sh.density = float(ga.get("density", 1000.0))
            out.append(sh)
        return out

    def visit(bel, parent_idx, parent_shift, cls):
        cls = bel.get("childclass", cls)
        idx = len(asset.bodies)
        body = Body(bel.get("name", "body%d" % idx))
        bp = np.array(_mj_floats(bel.get("pos"), (0, 0, 0)), dtype=np.float64) - parent_shift
        bq = _mj_quat(bel, angle_deg)
        joints = [j for j in bel if j.tag in ("joint", "freejoint")]
        free = [j for j in joints if j.tag == "freejoint" or
                defaults.attrs(j, j.get("class", cls)).get("type", "hinge") == "free"]
        hinge = [j for j in joints if j not in free]
        if parent_idx is None and hinge:
            raise ValueError("MJCF %s: joints on the root body other than a free joint" % path)
        if parent_idx is not None and free:
            raise ValueError("MJCF %s: free joint below the root" % path)
        shift = np.zeros(3)
        if parent_idx is not None:
            # one joint per hinge / slide / ball element, in declaration order; a
            # body with several (nv_humanoid.xml:53-54, three hips at :61-63) hangs
            # by all of them: the last is the body's joint, the ones before it its
            # pre-hinges (each about its axis in the body frame as turned by the
            # ones before, MuJoCo's order), sharing one anchor
            chain = []
            anchors = []
            for hj in (hinge or [None]):
                j = Joint(hj.get("name") if hj is not None else body.name + "_fixed", T.JOINT_FIXED, parent_idx, idx)
                j.p, j.q = bp, bq
                anchor = np.zeros(3)
                if hj is not None:
                    ja = defaults.attrs(hj, hj.get("class", cls))
                    typ = ja.get("type", "hinge")
                    if typ not in ("hinge", "slide", "ball"):
                        raise ValueError("MJCF %s: joint type %s unsupported" % (path, typ))
                    if len(hinge) > 1 and typ != "hinge":
                        raise ValueError("MJCF %s: body %s: several joints, not all hinges (%s)" % (path, body.name, typ))
                    j.type = {"hinge": T.JOINT_REVOLUTE, "slide": T.JOINT_PRISMATIC, "ball": T.JOINT_BALL}[typ]
                    ax = np.array(_mj_floats(ja.get("axis"), (0, 0, 1)), dtype=np.float64)
                    j.axis = ax / np.linalg.norm(ax)
                    anchor = np.array(_mj_floats(ja.get("pos"), (0, 0, 0)), dtype=np.float64)
                    rng = _mj_floats(ja.get("range"))
                    limited = ja.get("limited", "auto")
                    if rng is not None and limited in ("true", "auto") and typ != "ball":   # a cone limit: not modelled
                        sc = k_ang if typ == "hinge" else 1.0
                        j.has_limits, j.lower, j.upper = True, rng[0] * sc, rng[1] * sc
                    j.damping = float(ja.get("damping", 0.0))
                    j.friction = float(ja.get("frictionloss", 0.0))
                    j.velocity = MJCF_MAX_JOINT_VELOCITY
                    if ja.get("armature") is not None:
                        j.armature = float(ja.get("armature"))
                    joint_of_name[j.name] = j
                chain.append(j)
                anchors.append(anchor)
            if any(np.any(a != anchors[0]) for a in anchors[1:]):
                raise ValueError("MJCF %s: body %s: its joints have different anchors (pos)" % (path, body.name))
            if np.any(anchors[0] != 0.0):
                shift = anchors[0]
                for j in chain:
                    j.p = bp + _qmat(bq) @ shift
            j = chain[-1]
            j.pre = chain[:-1]
            asset.joints.append(j)
        shapes = geom_shapes(bel, cls, shift)
        body.shapes = shapes
        body.has_visual = bool(shapes)
        ine = bel.find("inertial")
        if ine is not None:
            body.has_inertial = True
            body.mass = float(ine.get("mass", 0.0))
            body.com = np.array(_mj_floats(ine.get("pos"), (0, 0, 0)), dtype=np.float64) - shift
            R = _qmat(_mj_quat(ine, angle_deg))
            di = _mj_floats(ine.get("diaginertia"))
            fi = _mj_floats(ine.get("fullinertia"))
            if di is not None:
                body.inertia = R @ np.diag(di) @ R.T
            elif fi is not None:
                xx, yy, zz, xy, xz, yz = fi
                body.inertia = R @ np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]]) @ R.T
        elif shapes:
            # mass properties from the geoms, each at its own density
            vols = [s.volume() for s in shapes]
            ms = [s.density * v for s, v in zip(shapes, vols)]
            M = sum(ms)
            if M > 0:
                com = sum(s.com_body() * m for s, m in zip(shapes, ms)) / M
                I = np.zeros((3, 3))
                for s, m in zip(shapes, ms):
                    R = _qmat(s.q)
                    d = s.com_body() - com
                    I += R @ (s.inertia_unit_mass() * m) @ R.T + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
                body.has_inertial, body.mass, body.com, body.inertia = True, M, com, I
        asset.bodies.append(body)
        for child in bel.findall("body"):
            visit(child, idx, shift, cls)

    visit(tops[0], None, np.zeros(3), "main")
    act = root.find("actuator")
    if act is not None:
        for mo in act:
            if mo.tag not in ("motor", "general"):
                continue
            ma = defaults.attrs(mo, mo.get("class", "main"))     # <default><motor ctrlrange=...> applies
            j = joint_of_name.get(ma.get("joint"))
            cr = _mj_floats(ma.get("ctrlrange"))
            if j is None or cr is None or ma.get("ctrllimited", "true") == "false":
                continue
            gear = _mj_floats(ma.get("gear"), (1.0,))[0]
            j.effort = abs(gear) * max(abs(cr[0]), abs(cr[1]))
    asset.warnings = warnings
    asset.path = path
    asset.floating_root = True
    return asset.finalize()
