"""Sim / Env / actor bookkeeping, the packed model handed to libmigym, and the
persistent tensors of the tensor API.

Index maps (bit-exact contract):
  actor (DOMAIN_SIM)  = env-major, then actor creation order in the env
                        (test10_servo_vecenv.py:373 views (num_envs, 2, 13));
  rigid body          = env-major, actor order, body tree order
                        (examples/franka_cube_ik_osc.py:255,277);
  DOF                 = env-major, actor order, DOF tree order
                        (examples/franka_cube_ik_osc.py:323-326 views (num_envs, 9, 1)).
Tensor frame: global sim frame; env i's origin is its grid cell.
"""
import ctypes
import sys
import os

import numpy as np
import torch

from . import _native as N
from . import _types as T
from ._assets import _qmat, _qmul


def _raw_stream(device):
    return torch.cuda.current_stream(device).cuda_stream


if hasattr(torch._C, "_cuda_getCurrentRawStream"):
    _raw_stream = torch._C._cuda_getCurrentRawStream      # noqa: F811  (one C call, no Stream object)



_warned_multishape = [False]


def _warn_multishape_friction(A):
    """Friction is PhysX's patch friction (anchors, physx.friction_offset_threshold
    / friction_correlation_distance) for single-shape free bodies on the ground
    and for every coupled env; a free body of several
    shapes stepping alone on the ground keeps one friction row pair per contact
    point. Said once, on stderr — never silently."""
    if _warned_multishape[0]:
        return
    kind, tmpl, tbi = A["body_kind"], A["body_tmpl"], A["tmpl_body_i"]
    free = np.asarray(kind) == N.MG_BODY_FREE
    if free.any() and (np.asarray(tbi)[np.asarray(tmpl)[free], 1] > 1).any():
        _warned_multishape[0] = True
        print("*** migym: free bodies with several collision shapes keep per-point friction against the ground "
              "plane (patch friction: single-shape free bodies and coupled envs; DESIGN.md §3.2.1)",
              file=sys.stderr)

_warned_cross_env = [False]


def _scaled_hull_record(r, s):
    """An MG_HULL record (include/migym.h) scaled by s about the shape origin:
    vertices and plane offsets times s; normals and edges unchanged."""
    r = np.array(r, dtype=np.float32)
    nv, nf = int(r[0]), int(r[1])
    h = N.MG_HULL_HEADER
    r[h:h + 3 * nv] = (r[h:h + 3 * nv].astype(np.float64) * s).astype(np.float32)
    d = h + 3 * nv + 4 * np.arange(nf) + 3
    r[d] = (r[d].astype(np.float64) * s).astype(np.float32)
    return r


def _warn_cross_env_contacts(A):
    """Contacts are simulated within an env only (every kernel steps an env on
    its own): actors of different envs that share a collision
    group (or use group -1) with filters that let them touch — e.g.
    examples/1080_balls_of_solitude.py --all_collisions (group 0, filter 0) —
    would collide in Isaac Gym once they meet. Said once, on stderr."""
    if _warned_cross_env[0]:
        return
    ac = np.asarray(A["actor_coll"])
    if len(ac) == 0:
        return
    env, grp, filt = ac[:, 0], ac[:, 1], ac[:, 2]

    def touch(fs):        # some pair of filters (a pair may be one actor's twice) shares no bit
        fs = np.unique(fs)
        return any((int(a) & int(b)) == 0 for i, a in enumerate(fs) for b in fs[i:])

    # group -1 meets every group: its actors count with each group's. Sorted
    # once (O(n log n): 262,144 envs of one group each used to take minutes)
    m = grp == -1
    em, fm = np.unique(env[m]), np.unique(filt[m])
    hit = False
    if not (~m).any():
        hit = len(em) > 1 and touch(fm)
    else:
        g, e, f = grp[~m], env[~m], filt[~m]
        order = np.lexsort((e, g))
        g, e, f = g[order], e[order], f[order]
        ug, start = np.unique(g, return_index=True)
        bounds = list(start[1:]) + [len(g)]
        first_env, last_env = e[start], e[np.asarray(bounds) - 1]
        multi = first_env != last_env                 # the group itself spans envs
        if len(em) > 1:
            multi[:] = True
        elif len(em) == 1:
            multi |= (first_env != em[0]) | (last_env != em[0])
        for k in np.nonzero(multi)[0]:
            if touch(np.concatenate([f[start[k]:bounds[k]], fm])):
                hit = True
                break
    if hit:
        _warned_cross_env[0] = True
        print("*** migym: actors of different envs share a collision group and may touch; contacts are simulated "
              "within each env only (DESIGN.md §3.6, §6)", file=sys.stderr)


class Env:
    __slots__ = ("sim", "index", "lower", "upper", "per_row", "origin", "actors", "num_bodies", "num_dofs",
                 "cameras")

    def __init__(self, sim, index, lower, upper, per_row):
        self.sim = sim
        self.index = index
        self.lower = lower
        self.upper = upper
        self.per_row = max(int(per_row), 1)
        g = index + sim.env_offset           # grid cell of the global env index (sharded sims)
        col = g % self.per_row
        row = g // self.per_row
        dx = upper.x - lower.x
        if sim.params.up_axis == T.UP_AXIS_Z:
            self.origin = np.array([col * dx, row * (upper.y - lower.y), 0.0])
        else:
            self.origin = np.array([col * dx, 0.0, row * (upper.z - lower.z)])
        self.actors = []
        self.num_bodies = 0
        self.num_dofs = 0
        self.cameras = []

    def __repr__(self):
        return "Env(%d)" % self.index


class Actor:
    def __init__(self, env, asset, pose, name, group, filter_, seg):
        self.env = env
        self.asset = asset
        self.pose = T.Transform(pose.p, pose.r)
        self.name = name
        self.group = group
        self.filter = filter_
        self.segmentation_id = seg
        self.handle = len(env.actors)
        self.body_offset = env.num_bodies          # env-domain first body
        self.dof_offset = env.num_dofs             # env-domain first DOF
        self.global_index = -1
        self.global_body = -1
        self.global_dof = -1
        self.dof_props = asset.dof_props.copy()
        nd = asset.num_dofs
        self.dof_state = np.zeros((nd, 2), dtype=np.float32)
        self.dof_targets = np.zeros((nd, 3), dtype=np.float32)   # pos, vel, effort
        self.shape_props = asset.shape_props      # copy-on-write (set_actor_rigid_shape_properties)
        self.mass_props = asset.mass_props        # copy-on-write (set_actor_rigid_body_properties)
        self.body_colors = {}
        self.body_segs = {}
        self.body_textures = {}
        self.scale = 1.0
        # root (linear, angular) velocity set while the scene is still being
        # built (set_rigid_linear_velocity before prepare_sim,
        # examples/body_physics_props.py:128-130): the initial state's root row
        self.init_vel = None

    @property
    def num_bodies(self):
        return len(self.asset.bodies)

    @property
    def num_dofs(self):
        return self.asset.num_dofs


def _copy_shape_props(sp):
    c = T.RigidShapeProperties()
    c.__dict__.update(sp.__dict__)
    return c


class Viewer:
    """Headless viewer: a non-None handle whose window 'closes' after
    MIGYM_VIEWER_FRAMES draws (default 60), so the reference's
    `while not gym.query_viewer_has_closed(viewer)` loops terminate."""

    def __init__(self, sim, props):
        self.sim = sim
        self.props = props
        self.frames = 0
        self.max_frames = int(os.environ.get("MIGYM_VIEWER_FRAMES", "60"))
        self.cam_transform = T.Transform(T.Vec3(0, -5, 5), T.Quat())


class CameraSensor:
    def __init__(self, env, props, handle):
        self.env = env
        self.props = props
        self.handle = handle
        self.local = T.Transform()
        self.body = None          # env-domain body handle when attached
        self.follow = T.FOLLOW_TRANSFORM
        self.transform = T.Transform()   # env-frame transform when not attached
        self.images = {}                 # IMAGE_* -> persistent device tensor (get_camera_image_gpu_tensor)
        self.destroyed = False           # destroy_camera_sensor: no longer rendered (its handle stays taken)


class Sim:
    def __init__(self, compute_device, graphics_device, engine, params):
        self.compute_device = int(compute_device)
        self.graphics_device = graphics_device
        self.engine = engine
        self.params = params
        self.plane = None
        self.env_offset = 0        # global index of this sim's first env (sharding.shard_sim)
        self.envs = []
        self.assets = []
        self.num_actors = self.num_bodies = self.num_dofs = 0
        self._idx_dirty = False    # global actor / body / DOF indices need a recompute
        self.finalized = False
        self.native = None
        self.frame = 0
        self.time = 0.0
        self.use_gpu_pipeline = bool(params.use_gpu_pipeline)
        self.device = torch.device("cuda", self.compute_device) if self.use_gpu_pipeline else torch.device("cpu")
        self.tensors = {}
        self.jacobians = {}
        self.mass_matrices = {}
        # state epoch: bumped by simulate and every state setter; the mass matrix
        # computed alongside the Jacobian is reused while the epoch is unchanged
        self.epoch = 0
        # CPU pipeline: the host state staged by fetch_results(sim, True) and the
        # epoch it belongs to (gymapi.Gym._refresh serves refreshes from it)
        self.host_stage = None
        self.host_stage_offsets = {}
        self.host_stage_epoch = -1
        self.host_stage_parts = 0      # kinds refreshed so far: staged by the next waiting fetch
        self.host_staged = 0           # kinds the last waiting fetch staged
        self.held_src = []     # fused sets: (tensor, torch version at the set, setter), until the next simulate
        # step fusion (gym.set_step_fusion; opt-in, MIGYM_STEP_FUSION sets the default)
        self.fusion = int(os.environ.get("MIGYM_STEP_FUSION", "0") or 0) & 31
        self.rb_paired_version = None   # rb tensor version after a fused root refresh filled it
        self.root_out_version = None    # root tensor version after a simulate wrote it (STEP_OUT)
        self.dof_out_version = None     # DOF tensor version after a simulate wrote it (STEP_OUT)
        self.mm_cache = {}
        self._renderer = None
        self.cam_version = 0       # bumped by every camera change (render tables are rebuilt)
        self.render_version = 0    # bumped by body colour / segmentation changes
        self.textures = []          # create_texture_from_file / _buffer: the handle is the index
        self.light = None           # set_light_parameters (an _native.MgLight), None: the default light

    @property
    def renderer(self):
        if self._renderer is None:
            from ._render import Renderer
            self._renderer = Renderer(self)
        return self._renderer

    # ------------------------------------------------------------ params
    def mg_params(self):
        p = self.params
        px = p.physx
        mp = N.MgSimParams()
        mp.dt = float(p.dt)
        mp.substeps = int(p.substeps)
        mp.gravity[:] = [p.gravity.x, p.gravity.y, p.gravity.z]
        mp.up_axis = int(p.up_axis)
        mp.num_position_iterations = int(px.num_position_iterations)
        mp.num_velocity_iterations = int(px.num_velocity_iterations)
        mp.contact_offset = float(px.contact_offset)
        mp.rest_offset = float(px.rest_offset)
        mp.bounce_threshold_velocity = float(px.bounce_threshold_velocity)
        mp.max_depenetration_velocity = float(px.max_depenetration_velocity)
        mp.friction_offset_threshold = float(px.friction_offset_threshold)
        mp.friction_correlation_distance = float(px.friction_correlation_distance)
        if self.plane is not None:
            n = self.plane.normal.normalize()
            mp.has_ground = 1
            mp.ground_normal[:] = [n.x, n.y, n.z]
            mp.ground_distance = float(self.plane.distance)
            mp.ground_static_friction = float(self.plane.static_friction)
            mp.ground_dynamic_friction = float(self.plane.dynamic_friction)
            mp.ground_restitution = float(self.plane.restitution)
        return mp

    # ------------------------------------------------------------ layout
    @property
    def actors(self):
        for e in self.envs:
            for a in e.actors:
                yield a

    def note_actor_added(self, env, a):
        """Global indices of an actor appended to the last env follow from the
        running totals (the usual build order: O(1) per actor, so per-env index
        queries while building, examples/franka_cube_ik_osc.py:255, stay linear);
        an actor added to an earlier env shifts later ones: full recompute."""
        if not self._idx_dirty and env is self.envs[-1]:
            a.global_index, a.global_body, a.global_dof = self.num_actors, self.num_bodies, self.num_dofs
            self.num_actors += 1
            self.num_bodies += a.num_bodies
            self.num_dofs += a.num_dofs
        else:
            self._idx_dirty = True

    def _assign_indices(self):
        if not self._idx_dirty:
            return
        self._idx_dirty = False
        ai = bi = di = 0
        for e in self.envs:
            for a in e.actors:
                a.global_index = ai
                a.global_body = bi
                a.global_dof = di
                ai += 1
                bi += a.num_bodies
                di += a.num_dofs
        self.num_actors, self.num_bodies, self.num_dofs = ai, bi, di

    def actor_world_body_poses(self, a):
        """Initial world poses (p[3], q[4]) of an actor's bodies by forward kinematics."""
        asset = a.asset
        o = a.env.origin
        root_p = (o[0] + a.pose.p.x, o[1] + a.pose.p.y, o[2] + a.pose.p.z)
        r = a.pose.r
        nq = (r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w) ** 0.5
        root_q = (r.x / nq, r.y / nq, r.z / nq, r.w / nq)
        if not asset.joints:
            return [root_p], [root_q]
        root_p = np.array(root_p)
        root_q = np.array(root_q)
        ps = [root_p]
        qs = [root_q]
        for k, j in enumerate(asset.joints):
            b = k + 1
            d = asset.dof_of_body(b)
            qj = float(a.dof_state[d, 0]) if d >= 0 else 0.0
            qrel = j.q.copy()
            rr = j.p * a.scale
            for k, pj in enumerate(j.pre):      # pre-hinges of a multi-joint body, in order
                th = float(a.dof_state[d + k, 0])
                s, c = np.sin(0.5 * th), np.cos(0.5 * th)
                qrel = _qmul(qrel, np.array([pj.axis[0] * s, pj.axis[1] * s, pj.axis[2] * s, c]))
            d = d + len(j.pre) if d >= 0 else d
            qj = float(a.dof_state[d, 0]) if d >= 0 and j.own_ndof else 0.0
            if j.type == T.JOINT_REVOLUTE:
                s, c = np.sin(0.5 * qj), np.cos(0.5 * qj)
                qrel = _qmul(qrel, np.array([j.axis[0] * s, j.axis[1] * s, j.axis[2] * s, c]))
            elif j.type == T.JOINT_BALL:
                # exponential coordinates: the joint turns by exp(th), th the
                # rotation vector of its three DOFs (mg_spatial.h q_exp)
                th = np.array([float(a.dof_state[d + k, 0]) for k in range(3)])
                t = float(np.linalg.norm(th))
                if t > 0.0:
                    e = np.array([*(th / t * np.sin(0.5 * t)), np.cos(0.5 * t)])
                    qrel = _qmul(qrel, e)
            elif j.type == T.JOINT_PRISMATIC:
                rr = j.p * a.scale + _qmat(j.q) @ (j.axis * qj)
            pp, pq = ps[j.parent], qs[j.parent]
            qn = _qmul(pq, qrel)
            qs.append(qn / np.linalg.norm(qn))
            ps.append(pp + _qmat(pq) @ rr)
        return ps, qs

    def build_model(self):
        """Pack the scene into the arrays of mg_model (include/migym.h)."""
        self._assign_indices()
        nb, na, nd = self.num_bodies, self.num_actors, self.num_dofs
        st = np.zeros((nb, N.MG_STATE_N), dtype=np.float32)
        mass = np.zeros((nb, N.MG_MASS_N), dtype=np.float32)
        kind = np.zeros(nb, dtype=np.int32)
        btmpl = np.zeros(nb, dtype=np.int32)
        root = np.zeros(na, dtype=np.int32)
        adof = np.zeros(na + 1, dtype=np.int32)
        acoll = np.zeros((na, N.MG_ACOLL_N), dtype=np.int32)
        dof0 = np.zeros((nd, 2), dtype=np.float32)
        dprops = np.zeros((nd, N.MG_DOFPROP_N), dtype=np.float32)
        tbf, tbi, shapes = [], [], []
        hulls, hull_off = [], {}       # MG_HULL records, offset by id(hull)
        nhull = 0
        tb_key = {}
        artic, atmpl, lf, li = [], [], [], []
        atmpl_key = {}
        blocks = {}        # per (asset, mass props, shape props): mass rows, kinds, template ids
        for a in self.actors:
            asset = a.asset
            opts = asset.options
            nba = a.num_bodies
            g0 = a.global_body
            root[a.global_index] = g0
            acoll[a.global_index, :3] = [a.env.index, a.group, a.filter]
            adof[a.global_index + 1] = a.global_dof + a.num_dofs
            ps, qs = self.actor_world_body_poses(a)
            multi = nba > 1
            for b in range(nba):
                st[g0 + b, 0:3] = ps[b]
                st[g0 + b, 3:7] = qs[b]
            if a.init_vel is not None:
                st[g0, 7:13] = a.init_vel
            sc = a.scale                   # set_actor_scale: geometry and joint frames (mass props already scaled)
            bkey = (id(asset), id(a.mass_props), id(a.shape_props), sc)
            blk = blocks.get(bkey)
            if blk is None:
                bm = np.zeros((nba, N.MG_MASS_N), dtype=np.float32)
                bt = np.zeros(nba, dtype=np.int32)
                for b, body in enumerate(asset.bodies):
                    mp = a.mass_props[b]
                    invm, invI, iq = mp.principal()
                    bm[b, 0] = invm
                    bm[b, 1:4] = invI
                    bm[b, 4:8] = iq
                    bm[b, 8:11] = mp.com
                    bm[b, 11] = mp.mass
                    # template body: asset body + its shape materials + body options
                    sidx = sum(len(x.shapes) for x in asset.bodies[:b])
                    mats = tuple((a.shape_props[sidx + k].friction, a.shape_props[sidx + k].restitution)
                                 for k in range(len(body.shapes)))
                    key = (id(asset), b, mats, sc)
                    if key not in tb_key:
                        tb_key[key] = len(tbf)
                        tbf.append([opts.linear_damping, opts.angular_damping, opts.max_linear_velocity,
                                    opts.max_angular_velocity, 0.0 if opts.disable_gravity else 1.0, 0, 0, 0])
                        tbi.append([len(shapes), len(body.shapes), 0, 0])
                        for k, sh in enumerate(body.shapes):
                            rec = np.zeros(N.MG_SHAPE_STRIDE, dtype=np.float32)
                            rec[0] = sh.type
                            rec[1:1 + len(sh.size)] = np.asarray(sh.size, dtype=np.float64) * sc
                            if sh.type == N.MG_SHAPE_CONVEX:
                                hk = (id(sh.hull), sc)
                                if hk not in hull_off:
                                    r = sh.hull.record()
                                    if sc != 1.0:
                                        r = _scaled_hull_record(r, sc)
                                    hull_off[hk] = nhull
                                    hulls.append(r)
                                    nhull += len(r)
                                rec[2] = hull_off[hk]
                            rec[4:7] = np.asarray(sh.p, dtype=np.float64) * sc
                            rec[7:11] = sh.q
                            rec[11] = mats[k][0]
                            rec[12] = mats[k][1]
                            shapes.append(rec)
                    bt[b] = tb_key[key]
                if multi:
                    bk = N.MG_BODY_LINK
                elif opts.fix_base_link:
                    bk = N.MG_BODY_STATIC
                else:
                    bk = N.MG_BODY_FREE
                blk = blocks[bkey] = (bm, bt, bk)
            bm, bt, bk = blk
            mass[g0:g0 + nba] = bm
            btmpl[g0:g0 + nba] = bt
            kind[g0:g0 + nba] = bk
            for d in range(a.num_dofs):
                gd = a.global_dof + d
                dof0[gd] = a.dof_state[d]
                p = a.dof_props[d]
                dprops[gd, :10] = [p["driveMode"], p["stiffness"], p["damping"], p["effort"], p["velocity"],
                                   p["lower"], p["upper"], 1.0 if p["hasLimits"] else 0.0, p["armature"],
                                   p["friction"]]
            if multi:
                akey = (id(asset), sc)
                if akey not in atmpl_key:
                    atmpl_key[akey] = len(atmpl)
                    atmpl.append([len(lf), len(asset.bodies), asset.num_dofs, 1 if opts.fix_base_link else 0])
                    nl0 = len(lf)
                    link_of = []          # body -> its kernel link (local)
                    for b in range(len(asset.bodies)):
                        if b == 0:
                            lf.append(np.zeros(N.MG_LINK_F_N, dtype=np.float32))
                            li.append([-1, 0, -1, 0])
                            link_of.append(0)
                            continue
                        j = asset.joints[b - 1]
                        d = asset.dof_of_body(b)
                        parent = link_of[j.parent]
                        for k, pj in enumerate(j.pre):
                            # pre-hinges of a multi-joint body: virtual revolute
                            # links (body -1), the first at the joint origin
                            f = np.zeros(N.MG_LINK_F_N, dtype=np.float32)
                            f[3:7] = (0, 0, 0, 1)
                            if k == 0:
                                f[0:3] = j.p * sc
                                f[3:7] = j.q
                            f[7:10] = pj.axis
                            lf.append(f)
                            li.append([parent, T.JOINT_REVOLUTE, d + k, -1])
                            parent = len(lf) - 1 - nl0
                        if j.pre:
                            d = d + len(j.pre)
                        if j.type == T.JOINT_BALL:
                            # three revolute links about the joint frame's x, y, z:
                            # two virtual (body -1), then the child body
                            for k in range(3):
                                f = np.zeros(N.MG_LINK_F_N, dtype=np.float32)
                                f[3:7] = (0, 0, 0, 1)
                                if k == 0:
                                    f[0:3] = j.p * sc
                                    f[3:7] = j.q
                                f[7 + k] = 1.0
                                f[10] = k + 1     # place in the ball: the first link turns by exp(th)
                                lf.append(f)
                                li.append([parent, T.JOINT_REVOLUTE, d + k, b if k == 2 else -1])
                                parent = len(lf) - 1 - nl0
                        else:
                            f = np.zeros(N.MG_LINK_F_N, dtype=np.float32)
                            f[3:7] = (0, 0, 0, 1)
                            if not j.pre:
                                f[0:3] = j.p * sc
                                f[3:7] = j.q
                            f[7:10] = j.axis
                            li.append([parent, j.type if j.type in (T.JOINT_FIXED, T.JOINT_REVOLUTE,
                                                                    T.JOINT_PRISMATIC) else T.JOINT_FIXED, d, b])
                            lf.append(f)
                        link_of.append(len(lf) - 1 - nl0)
                    atmpl[-1][1] = len(lf) - nl0
                artic.append([a.global_body, a.global_dof, atmpl_key[akey], 0])
        self.model_arrays = dict(
            body_state0=st, body_mass=mass, body_kind=kind, body_tmpl=btmpl,
            tmpl_body_f=np.array(tbf, dtype=np.float32).reshape(-1, N.MG_TBODY_F_N),
            tmpl_body_i=np.array(tbi, dtype=np.int32).reshape(-1, N.MG_TBODY_I_N),
            shapes=np.array(shapes, dtype=np.float32).reshape(-1, N.MG_SHAPE_STRIDE),
            actor_root_body=root, actor_dof=adof, actor_coll=acoll, dof_state0=dof0, dof_props=dprops,
            artic_i=np.array(artic, dtype=np.int32).reshape(-1, N.MG_ARTIC_I_N),
            artic_tmpl_i=np.array(atmpl, dtype=np.int32).reshape(-1, N.MG_ATMPL_I_N),
            tmpl_link_f=np.array(lf, dtype=np.float32).reshape(-1, N.MG_LINK_F_N),
            tmpl_link_i=np.array(li, dtype=np.int32).reshape(-1, N.MG_LINK_I_N),
            hulls=np.concatenate(hulls).astype(np.float32) if hulls else np.zeros(0, np.float32),
        )
        return self.model_arrays

    def mg_model(self, arrays=None):
        """ctypes mg_model over the packed arrays (kept alive by self._model_keep)."""
        A = arrays if arrays is not None else self.model_arrays
        m = N.MgModel()
        m.num_envs = len(self.envs)
        m.num_actors = len(A["actor_root_body"])
        m.num_bodies = len(A["body_kind"])
        m.num_dofs = len(A["dof_state0"])
        m.num_tmpl_bodies = len(A["tmpl_body_f"])
        m.num_shapes = len(A["shapes"])
        m.num_artics = len(A["artic_i"])
        m.num_artic_tmpls = len(A["artic_tmpl_i"])
        m.num_tmpl_links = len(A["tmpl_link_f"])
        keep = {}
        m.num_hull_floats = len(A.get("hulls", ()))
        if m.num_hull_floats:
            arr = np.ascontiguousarray(A["hulls"], dtype=np.float32)
            keep["hulls"] = arr
            m.hulls = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        for name in ("body_state0", "body_mass", "tmpl_body_f", "shapes", "dof_state0", "dof_props", "tmpl_link_f"):
            arr = np.ascontiguousarray(A[name], dtype=np.float32)
            keep[name] = arr
            setattr(m, name, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        for name in ("body_kind", "body_tmpl", "tmpl_body_i", "actor_root_body", "actor_dof", "artic_i",
                     "artic_tmpl_i", "tmpl_link_i", "actor_coll"):
            arr = np.ascontiguousarray(A[name], dtype=np.int32)
            keep[name] = arr
            setattr(m, name, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        self._model_keep = keep
        return m

    # ------------------------------------------------------------ finalize
    def finalize(self):
        if self.finalized:
            return
        A = self.build_model()
        _warn_multishape_friction(A)
        _warn_cross_env_contacts(A)
        dev = self.device
        self.tensors["root"] = torch.from_numpy(A["body_state0"][A["actor_root_body"]].copy()).to(dev)
        self.tensors["rb"] = torch.from_numpy(A["body_state0"].copy()).to(dev)
        self.tensors["dof"] = torch.from_numpy(A["dof_state0"].copy()).to(dev)
        self.tensors["ncf"] = torch.zeros((self.num_bodies, 3), dtype=torch.float32, device=dev)
        if dev.type == "cpu" and N.device_count() > 0 and torch.cuda.is_available():
            # the CPU pipeline's host tensors (test10's mode) in page-locked memory:
            # every refresh is a D2H copy and every set an H2D copy, which then go
            # straight over PCIe instead of through the runtime's staging buffer
            for k in ("root", "rb", "dof", "ncf"):
                self.tensors[k] = self.tensors[k].pin_memory()
            # fetch_results(sim, True) stages the whole state here in one round
            # trip (mg_fetch_host_state); the refreshes copy from it
            sizes = [self.tensors[k].numel() for k in ("root", "rb", "dof", "ncf")]
            offs = np.cumsum([0] + sizes)
            self.host_stage_offsets = {k: int(offs[i]) for i, k in enumerate(("root", "rb", "dof", "ncf"))}
            self.host_stage = torch.empty(int(offs[-1]), dtype=torch.float32).pin_memory()
        if N.device_count() > 0:
            handle = N.lib.mg_create_sim(self.compute_device, ctypes.byref(self.mg_params()))
            if not handle:
                raise N.MigymError("mg_create_sim: " + N.last_error())
            self.native = handle
            N.check(N.lib.mg_upload_model(handle, ctypes.byref(self.mg_model())), "mg_upload_model")
            if self.host_stage is not None and os.environ.get("MIGYM_HOST_STAGE", "mapped") != "copy":
                # the sim's own device-mapped host stage (mg_host_stage): the
                # waiting fetch is then zero-copy (the step writes its rows into it);
                # MIGYM_HOST_STAGE=copy keeps a torch page-locked stage and a D2H copy
                nst = int(self.host_stage.numel())
                ptr = N.lib.mg_host_stage(handle, max(nst, 1))
                if ptr:
                    buf = (ctypes.c_float * max(nst, 1)).from_address(ptr)
                    self.host_stage = torch.from_numpy(np.ctypeslib.as_array(buf))[:nst]
            # the persistent root / rigid-body tensors: a root refresh serves both
            # (mg_bind_refresh_targets, MG_FUSE_REFRESH)
            root, rb = self.tensors["root"], self.tensors["rb"]
            if root.is_cuda and rb.is_cuda and root.numel() and rb.numel():
                N.check(N.lib.mg_bind_refresh_targets(handle, root.data_ptr(), rb.data_ptr()),
                        "mg_bind_refresh_targets")
            dof = self.tensors["dof"]
            if dof.is_cuda and dof.numel():   # written by the step itself under STEP_FUSION_STEP_OUT
                N.check(N.lib.mg_bind_dof_refresh_target(handle, dof.data_ptr()), "mg_bind_dof_refresh_target")
            N.lib.mg_set_fusion(handle, self.fusion)
            if self.light is not None:
                N.check(N.lib.mg_set_light(handle, ctypes.byref(self.light)), "mg_set_light")
            # actor DOF targets / props set before prepare
            self._push_dof_targets_all()
        self.finalized = True

    def _push_dof_targets_all(self):
        if self.num_dofs == 0:
            return
        tgt = np.zeros((self.num_dofs, 3), dtype=np.float32)
        for a in self.actors:
            tgt[a.global_dof:a.global_dof + a.num_dofs] = a.dof_targets
        for col, fn in ((0, N.lib.mg_set_dof_position_target), (1, N.lib.mg_set_dof_velocity_target),
                        (2, N.lib.mg_set_dof_actuation_force)):
            c = np.ascontiguousarray(tgt[:, col])
            N.check(fn(self.native, c.ctypes.data, 1, None, 0, self.stream()), "set dof targets")

    def require_native(self, what):
        self.finalize()
        if self.native is None:
            raise N.MigymError(
                "%s needs a HIP device: libmigym found %d GPUs (no CPU engine exists; run on an MI355X)"
                % (what, N.device_count()))
        return self.native

    def stream(self):
        """torch's current HIP stream on the sim's device (raw handle), so our
        kernels order with the caller's torch work on the state tensors."""
        if self.native is None:
            return None
        return _raw_stream(self.compute_device)

    def destroy(self):
        if self.native:
            self.host_stage = None          # the sim's own memory (mg_host_stage), freed with it
            self.host_stage_epoch = -1
            N.lib.mg_destroy_sim(self.native)
            self.native = None
