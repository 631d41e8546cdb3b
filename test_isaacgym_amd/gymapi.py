"""isaacgym.gymapi mirror over libmigym (MI355X).

`acquire_gym()` returns the Gym singleton whose methods the reference's scripts
call (the hot loop is test10_servo_vecenv.py:376-471 and
examples/franka_cube_ik_osc.py:336-415). The physics path — simulate, refresh_*,
set_* — is libmigym's HIP kernels; everything here is scene bookkeeping and
argument marshalling. Error behaviour follows Isaac Gym: creators return None,
setters return False, lookups return INVALID_HANDLE (-1).

Camera sensors are rendered on the GPU (_render.py, csrc/mg_render.hip: config
5). The viewer is headless: a handle whose window "closes" after
MIGYM_VIEWER_FRAMES draws, so the reference scripts' loops end (§8b last row).
"""
import ctypes
import math
import os
import sys
import time

import numpy as np
import torch

from . import _assets
from . import _native as N
from . import _render
from ._sim import Actor, CameraSensor, Env, Sim, Viewer
from ._types import *  # noqa: F401,F403
from ._types import (_DOF_TYPE_STRINGS, _JOINT_TYPE_STRINGS, DOF_PROPERTIES_DTYPE, DofState, Quat,
                     RigidBodyProperties, RigidBodyState, Transform, Vec3)
from . import _types as _T


class Tensor:
    """Non-owning tensor descriptor (gymapi.Tensor): what acquire_* returns and
    gymtorch.unwrap_tensor builds (examples/interop_torch.py:133-142)."""

    def __init__(self, torch_tensor):
        self._t = torch_tensor
        self.data_address = torch_tensor.data_ptr()
        self.shape = tuple(torch_tensor.shape)
        self.device = -1 if torch_tensor.device.type == "cpu" else int(torch_tensor.device.index or 0)
        self.dtype = _T.DTYPE_FLOAT32 if torch_tensor.dtype == torch.float32 else _T.DTYPE_UINT32
        self.own_data = False
        self.ndim = torch_tensor.dim()

    @property
    def is_host(self):
        return self.device < 0

    def __repr__(self):
        return "gymapi.Tensor(shape=%s, device=%d, data_address=0x%x)" % (self.shape, self.device, self.data_address)


def _as_tensor_arg(t, name):
    if isinstance(t, Tensor):
        tt = t._t
    elif isinstance(t, torch.Tensor):
        tt = t
    else:
        raise TypeError("%s: expected a gymapi.Tensor (gymtorch.unwrap_tensor)" % name)
    if not tt.is_contiguous():
        raise ValueError("%s: tensor must be contiguous" % name)
    return tt


# step fusion flags (gym.set_step_fusion; include/migym.h MG_FUSE_*)
STEP_FUSION_ROOT_SET = 1
STEP_FUSION_REFRESH = 2
STEP_FUSION_DOF_TARGETS = 4
STEP_FUSION_IN_CAPTURE = 8
STEP_FUSION_STEP_OUT = 16
STEP_FUSION_ALL = 31


_FUSED_KIND = {"mg_set_actor_root_state": "root", "mg_set_dof_position_target": "tgt0",
               "mg_set_dof_velocity_target": "tgt1", "mg_set_dof_actuation_force": "tgt2"}


def _check_held(sim, what, kinds=None):
    """Copy-at-set guard for opt-in step fusion. A fused set's source is read by
    the call that consumes the pending set — the next simulate, or for a root set
    any earlier reader of the state (the library flushes it as a scatter) — so it
    must still hold what it held at the set call: Isaac Gym reads it during
    set_*_tensor (SURVEY.md §8b Ownership). Rather than read newer data silently,
    raise. `kinds`: the pending sets this call consumes (None: all); consumed
    entries are dropped."""
    if not sim.held_src:
        return
    keep = []
    for t, ver, setter, kind in sim.held_src:
        if kinds is not None and kind not in kinds:
            keep.append((t, ver, setter, kind))
            continue
        if t._version != ver:
            # the pending sets are dropped on both sides: none is applied with data
            # newer than its set call, and a retry does not meet this one again
            sim.held_src = []
            if sim.native:
                N.lib.mg_discard_pending_sets(sim.native)
            raise N.MigymError(
                "%s: the tensor passed to %s was modified before the simulate that reads it; with step "
                "fusion on (gym.set_step_fusion) a full device set is read at the next simulate, not at the "
                "set call — write the source before the set, or turn fusion off (Isaac Gym copies at set "
                "time)" % (what, setter))
    sim.held_src = keep


# mg_fetch_host_state part bits of the state tensors
_STAGE_BIT = {"root": 1, "rb": 2, "dof": 4, "ncf": 8}


class Gym:
    def __init__(self):
        self._sims = []
        self._t0 = time.time()

    # ================================================================ sim
    def create_sim(self, compute_device=0, graphics_device=0, type=_T.SIM_PHYSX, params=None):
        """test10_servo_vecenv.py:185. Returns a Sim, or None (Isaac Gym style)."""
        if params is None:
            params = _T.SimParams()
        if type != _T.SIM_PHYSX:
            print("*** migym: only the PhysX-style rigid solver is available (SIM_FLEX requested)", file=sys.stderr)
            return None
        sim = Sim(compute_device, graphics_device, type, params)
        self._sims.append(sim)
        return sim

    def destroy_sim(self, sim):
        if sim is not None:
            sim.destroy()
            if sim in self._sims:
                self._sims.remove(sim)

    def get_sim_params(self, sim):
        return sim.params

    def set_sim_params(self, sim, params):
        sim.params = params
        if sim.native:
            N.check(N.lib.mg_set_sim_params(sim.native, ctypes.byref(sim.mg_params())), "mg_set_sim_params")

    def add_ground(self, sim, params):
        sim.plane = params
        if sim.native:
            N.check(N.lib.mg_set_sim_params(sim.native, ctypes.byref(sim.mg_params())), "mg_set_sim_params")

    def prepare_sim(self, sim):
        """examples/franka_cube_ik_osc.py:288. Uploads the scene to HBM."""
        sim.finalize()
        return True

    def simulate(self, sim):
        """One frame (test10_servo_vecenv.py:380): the fused HIP step kernels."""
        h = sim.require_native("gym.simulate")
        _check_held(sim, "simulate")
        N.check(N.lib.mg_simulate(h, sim.stream()), "mg_simulate")
        sim.held_src = []
        if sim.fusion & STEP_FUSION_STEP_OUT and "root" in sim.tensors:
            # the step kernels may have written the bound root / rigid-body / DOF
            # tensors (MG_FUSE_STEP_OUT): a write to them before their refresh forces a gather
            sim.root_out_version = sim.tensors["root"]._version
            sim.rb_paired_version = sim.tensors["rb"]._version
            sim.dof_out_version = sim.tensors["dof"]._version
        sim.epoch += 1
        sim.frame += 1
        sim.time += sim.params.dt

    def set_step_fusion(self, sim, flags):
        """migym extension (not in Isaac Gym): opt in to step fusion
        (include/migym.h mg_set_fusion; STEP_FUSION_* flags, 0 = off, the
        default). With it, a full device-resident set_actor_root_state_tensor /
        set_dof_*_target_tensor / set_dof_actuation_force_tensor is read by the
        next simulate instead of at the set call, a root-state refresh also
        refreshes the rigid-body tensor (STEP_FUSION_REFRESH), and on a sim of
        single-shape free bodies simulate writes both state tensors itself, the
        refreshes then launching nothing (STEP_FUSION_STEP_OUT). Isaac Gym copies the source at the set
        call (SURVEY.md §8b Ownership), so a source written between its set and
        the simulate that consumes it raises MigymError instead of being read
        (torch version counters); the environment variable MIGYM_STEP_FUSION sets
        the default for new sims. Returns the previous flags."""
        prev = sim.fusion
        sim.fusion = int(flags) & STEP_FUSION_ALL
        if sim.native:
            N.lib.mg_set_fusion(sim.native, sim.fusion)
        return prev

    def get_step_fusion(self, sim):
        return sim.fusion

    def fetch_results(self, sim, wait=True):
        """test10_servo_vecenv.py:381. In the CPU pipeline a waiting fetch also
        stages the state kinds refreshed so far (one device round trip), so the
        refreshes after it are host copies (include/migym.h mg_fetch_host_state)."""
        if sim.native:
            if wait and sim.host_stage is not None:
                # CPU pipeline: the state the refreshes will copy — the kinds
                # refreshed so far — staged in one device round trip
                # (mg_fetch_host_state) as the wait
                N.check(N.lib.mg_fetch_host_state(sim.native, sim.host_stage.data_ptr(), sim.host_stage_parts,
                                                  sim.stream()), "mg_fetch_host_state")
                sim.host_stage_epoch = sim.epoch
                sim.host_staged = sim.host_stage_parts
            else:
                N.check(N.lib.mg_fetch_results(sim.native, 1 if wait else 0), "mg_fetch_results")
        return True

    def get_sim_time(self, sim):
        return sim.time

    def get_frame_count(self, sim):
        return sim.frame

    def get_elapsed_time(self, sim):
        return time.time() - self._t0

    def get_sim_actor_count(self, sim):
        return sum(len(e.actors) for e in sim.envs)

    def get_sim_rigid_body_count(self, sim):
        return sum(e.num_bodies for e in sim.envs)

    def get_sim_dof_count(self, sim):
        return sum(e.num_dofs for e in sim.envs)

    def get_env_count(self, sim):
        return len(sim.envs)

    def get_env(self, sim, index):
        return sim.envs[index]

    # ================================================================ assets
    def load_asset(self, sim, rootpath, filename, options=None):
        """test10_servo_vecenv.py:230. None on failure (:232-234)."""
        options = options if options is not None else _T.AssetOptions()
        try:
            if filename.lower().endswith(".urdf"):
                asset = _assets.load_urdf(rootpath, filename, _copy_options(options))
            elif filename.lower().endswith(".xml") or filename.lower().endswith(".mjcf"):
                asset = _assets.load_mjcf(rootpath, filename, _copy_options(options))
            else:
                print("*** migym: unsupported asset format: %s" % filename, file=sys.stderr)
                return None
        except (OSError, ValueError) as e:
            print("*** migym: failed to load asset %s: %s" % (filename, e), file=sys.stderr)
            return None
        for w in getattr(asset, "warnings", []):
            print("migym: %s" % w, file=sys.stderr)
        sim.assets.append(asset)
        return asset

    load_urdf = load_asset

    def create_box(self, sim, width, height, depth, options=None):
        a = _assets.create_box(width, height, depth, _copy_options(options or _T.AssetOptions()))
        sim.assets.append(a)
        return a

    def create_sphere(self, sim, radius, options=None):
        a = _assets.create_sphere(radius, _copy_options(options or _T.AssetOptions()))
        sim.assets.append(a)
        return a

    def create_capsule(self, sim, radius, length, options=None):
        a = _assets.create_capsule(radius, length, _copy_options(options or _T.AssetOptions()))
        sim.assets.append(a)
        return a

    def get_asset_rigid_body_count(self, asset):
        return len(asset.bodies)

    def get_asset_rigid_body_name(self, asset, i):
        return asset.bodies[i].name if 0 <= i < len(asset.bodies) else None

    def get_asset_rigid_body_names(self, asset):
        return [b.name for b in asset.bodies]

    def get_asset_rigid_body_dict(self, asset):
        return {b.name: i for i, b in enumerate(asset.bodies)}

    def find_asset_rigid_body_index(self, asset, name):
        return self.get_asset_rigid_body_dict(asset).get(name, _T.INVALID_HANDLE)

    def get_asset_joint_count(self, asset):
        return len(asset.api_joints)

    def get_asset_joint_name(self, asset, i):
        return asset.api_joints[i].name

    def get_asset_joint_names(self, asset):
        return [j.name for j in asset.api_joints]

    def get_asset_joint_dict(self, asset):
        return {j.name: i for i, j in enumerate(asset.api_joints)}

    def get_asset_joint_type(self, asset, i):
        return asset.api_joints[i].type

    def find_asset_joint_index(self, asset, name):
        return self.get_asset_joint_dict(asset).get(name, _T.INVALID_HANDLE)

    def get_asset_dof_count(self, asset):
        return asset.num_dofs

    def get_asset_dof_name(self, asset, i):
        return asset.dof_names[i]

    def get_asset_dof_names(self, asset):
        return asset.dof_names

    def get_asset_dof_dict(self, asset):
        return {n: i for i, n in enumerate(asset.dof_names)}

    def find_asset_dof_index(self, asset, name):
        return self.get_asset_dof_dict(asset).get(name, _T.INVALID_HANDLE)

    def get_asset_dof_type(self, asset, i):
        j = asset.dof_joints[i]
        return _T.DOF_ROTATION if j.type in (_T.JOINT_REVOLUTE, _T.JOINT_BALL) else _T.DOF_TRANSLATION

    def get_asset_dof_properties(self, asset):
        return asset.dof_props.copy()

    def get_asset_rigid_shape_count(self, asset):
        return sum(len(b.shapes) for b in asset.bodies)

    def get_asset_rigid_shape_properties(self, asset):
        return list(asset.shape_props)

    def set_asset_rigid_shape_properties(self, asset, props):
        asset.shape_props = list(props)
        return True

    def get_asset_rigid_body_shape_indices(self, asset):
        out, s = [], 0
        for b in asset.bodies:
            out.append((s, len(b.shapes)))
            s += len(b.shapes)
        return out

    def get_joint_type_string(self, jtype):
        return _JOINT_TYPE_STRINGS.get(jtype, "Invalid")

    def get_dof_type_string(self, dtype):
        return _DOF_TYPE_STRINGS.get(dtype, "Invalid")

    # ================================================================ envs / actors
    def create_env(self, sim, lower, upper, num_per_row):
        """test10_servo_vecenv.py:301."""
        if sim.finalized:
            print("*** migym: cannot create envs after prepare_sim / first tensor access", file=sys.stderr)
            return None
        env = Env(sim, len(sim.envs), lower, upper, num_per_row)
        sim.envs.append(env)
        return env

    def create_actor(self, env, asset, pose, name=None, group=-1, filter=0, segmentationId=0):
        """test10_servo_vecenv.py:317,323. Returns the env-local actor handle, -1 on failure."""
        if env.sim.finalized:
            print("*** migym: cannot create actors after prepare_sim / first tensor access", file=sys.stderr)
            return _T.INVALID_HANDLE
        if asset is None:
            return _T.INVALID_HANDLE
        a = Actor(env, asset, pose, name if name is not None else asset.name, group, filter, segmentationId)
        env.actors.append(a)
        env.num_bodies += a.num_bodies
        env.num_dofs += a.num_dofs
        env.sim.note_actor_added(env, a)
        return a.handle

    def _actor(self, env, handle):
        if handle is None or not (0 <= handle < len(env.actors)):
            raise IndexError("invalid actor handle %r" % (handle,))
        return env.actors[handle]

    def get_actor_count(self, env):
        return len(env.actors)

    def get_actor_handle(self, env, index):
        return index if 0 <= index < len(env.actors) else _T.INVALID_HANDLE

    def find_actor_handle(self, env, name):
        for a in env.actors:
            if a.name == name:
                return a.handle
        return _T.INVALID_HANDLE

    def get_actor_name(self, env, handle):
        return self._actor(env, handle).name

    def get_actor_index(self, env, handle, domain):
        a = self._actor(env, handle)
        if domain == _T.DOMAIN_SIM:
            env.sim._assign_indices()
            return a.global_index
        return a.handle

    def get_actor_rigid_body_count(self, env, handle):
        return self._actor(env, handle).num_bodies

    def get_actor_rigid_body_names(self, env, handle):
        return [b.name for b in self._actor(env, handle).asset.bodies]

    def get_actor_rigid_body_dict(self, env, handle):
        return {b.name: i for i, b in enumerate(self._actor(env, handle).asset.bodies)}

    def get_actor_rigid_body_handle(self, env, handle, index):
        a = self._actor(env, handle)
        return a.body_offset + index if 0 <= index < a.num_bodies else _T.INVALID_HANDLE

    def find_actor_rigid_body_handle(self, env, handle, name):
        a = self._actor(env, handle)
        for i, b in enumerate(a.asset.bodies):
            if b.name == name:
                return a.body_offset + i
        return _T.INVALID_HANDLE

    def get_actor_rigid_body_index(self, env, handle, index, domain):
        """examples/franka_cube_ik_osc.py:255."""
        a = self._actor(env, handle)
        if not 0 <= index < a.num_bodies:
            return _T.INVALID_HANDLE
        if domain == _T.DOMAIN_ACTOR:
            return index
        if domain == _T.DOMAIN_ENV:
            return a.body_offset + index
        env.sim._assign_indices()
        return a.global_body + index

    def find_actor_rigid_body_index(self, env, handle, name, domain):
        """examples/franka_cube_ik_osc.py:277."""
        d = self.get_actor_rigid_body_dict(env, handle)
        if name not in d:
            return _T.INVALID_HANDLE
        return self.get_actor_rigid_body_index(env, handle, d[name], domain)

    def get_rigid_handle(self, env, actor_name, body_name):
        h = self.find_actor_handle(env, actor_name)
        return _T.INVALID_HANDLE if h < 0 else self.find_actor_rigid_body_handle(env, h, body_name)

    def get_actor_joint_count(self, env, handle):
        return len(self._actor(env, handle).asset.api_joints)

    def get_actor_joint_names(self, env, handle):
        return [j.name for j in self._actor(env, handle).asset.api_joints]

    def get_actor_joint_dict(self, env, handle):
        return {j.name: i for i, j in enumerate(self._actor(env, handle).asset.api_joints)}

    def get_actor_joint_handle(self, env, handle, index):
        return index

    def get_actor_dof_count(self, env, handle):
        return self._actor(env, handle).num_dofs

    def get_actor_dof_names(self, env, handle):
        return self._actor(env, handle).asset.dof_names

    def get_actor_dof_dict(self, env, handle):
        return {n: i for i, n in enumerate(self._actor(env, handle).asset.dof_names)}

    def get_actor_dof_handle(self, env, handle, index):
        a = self._actor(env, handle)
        return a.dof_offset + index if 0 <= index < a.num_dofs else _T.INVALID_HANDLE

    def find_actor_dof_handle(self, env, handle, name):
        """test12_add_joint.py.py:100: a missing name gives INVALID_HANDLE, not an error."""
        d = self.get_actor_dof_dict(env, handle)
        return self._actor(env, handle).dof_offset + d[name] if name in d else _T.INVALID_HANDLE

    def get_actor_dof_index(self, env, handle, index, domain):
        a = self._actor(env, handle)
        if domain == _T.DOMAIN_ACTOR:
            return index
        if domain == _T.DOMAIN_ENV:
            return a.dof_offset + index
        env.sim._assign_indices()
        return a.global_dof + index

    def find_actor_dof_index(self, env, handle, name, domain):
        d = self.get_actor_dof_dict(env, handle)
        return self.get_actor_dof_index(env, handle, d[name], domain) if name in d else _T.INVALID_HANDLE

    def get_dof_frame(self, env, dof_handle):
        """examples/joint_monkey.py:255-259: the world origin and axis of a DOF's
        joint at the current state (forward kinematics of the packed links from
        the actor's root pose and DOF positions; a ball joint's or pre-hinge's
        virtual links included)."""
        a, d = self._dof_owner(env, dof_handle)
        sim = env.sim
        sim.finalize()
        A = sim.model_arrays
        rb, ds = self._host_state(sim)
        q = ds[a.global_dof:a.global_dof + a.num_dofs, 0].astype(np.float64)
        root = rb[a.global_body].astype(np.float64)
        k = [i for i, r in enumerate(A["artic_i"]) if r[0] == a.global_body][0]
        ti = A["artic_tmpl_i"][A["artic_i"][k][2]]
        lf = A["tmpl_link_f"][ti[0]:ti[0] + ti[1]].astype(np.float64)
        li = A["tmpl_link_i"][ti[0]:ti[0] + ti[1]]
        from ._assets import _qmat, _qmul
        ps, qs = [root[0:3]], [root[3:7] / np.linalg.norm(root[3:7])]
        for l in range(1, len(li)):
            p, jt, dj = int(li[l, 0]), int(li[l, 1]), int(li[l, 2])
            po, qo, ax = lf[l, 0:3], lf[l, 3:7], lf[l, 7:10]
            org = ps[p] + _qmat(qs[p]) @ po
            qj = _qmul(qs[p], qo)                       # the joint frame (before its own motion)
            if dj == d:
                axis = _qmat(qj) @ ax
                return _T.DofFrame(_T.Vec3(*org), _T.Vec3(*axis))
            qrel, rr = qo, po
            ball = int(round(lf[l, 10]))
            if ball == 1:
                th = q[dj:dj + 3]
                t = np.linalg.norm(th)
                if t > 0:
                    qrel = _qmul(qo, np.array([*(th / t * np.sin(0.5 * t)), np.cos(0.5 * t)]))
            elif ball == 0 and jt == _T.JOINT_REVOLUTE and dj >= 0:
                qrel = _qmul(qo, np.array([*(ax * np.sin(0.5 * q[dj])), np.cos(0.5 * q[dj])]))
            elif jt == _T.JOINT_PRISMATIC and dj >= 0:
                rr = po + _qmat(qo) @ (ax * q[dj])
            ps.append(ps[p] + _qmat(qs[p]) @ rr)
            qn = _qmul(qs[p], qrel)
            qs.append(qn / np.linalg.norm(qn))
        raise IndexError("DOF %d has no joint" % d)

    def _dof_owner(self, env, dof_handle):
        for a in env.actors:
            if a.dof_offset <= dof_handle < a.dof_offset + a.num_dofs:
                return a, dof_handle - a.dof_offset
        raise IndexError("invalid DOF handle %r" % (dof_handle,))

    # ---- DOF properties and targets (non-tensor API)
    def get_actor_dof_properties(self, env, handle):
        return self._actor(env, handle).dof_props.copy()

    def set_actor_dof_properties(self, env, handle, props):
        a = self._actor(env, handle)
        props = np.asarray(props)
        for f in DOF_PROPERTIES_DTYPE.names:
            if props.dtype.names and f in props.dtype.names:
                a.dof_props[f] = props[f]
        sim = env.sim
        if sim.finalized and sim.native:
            self._push_dof_props(sim)
        return True

    def _push_dof_props(self, sim):
        dp = np.zeros((sim.num_dofs, N.MG_DOFPROP_N), dtype=np.float32)
        for a in sim.actors:
            for d in range(a.num_dofs):
                p = a.dof_props[d]
                dp[a.global_dof + d, :10] = [p["driveMode"], p["stiffness"], p["damping"], p["effort"], p["velocity"],
                                             p["lower"], p["upper"], 1.0 if p["hasLimits"] else 0.0, p["armature"],
                                             p["friction"]]
        N.check(N.lib.mg_set_dof_props(sim.native, dp.ctypes.data), "mg_set_dof_props")

    def _set_actor_dof_column(self, env, handle, values, col):
        a = self._actor(env, handle)
        vals = np.asarray(values, dtype=np.float32).reshape(-1)
        a.dof_targets[:len(vals), col] = vals[:a.num_dofs]
        sim = env.sim
        if sim.finalized and sim.native and a.num_dofs:
            full = np.zeros(sim.num_dofs, dtype=np.float32)
            full[a.global_dof:a.global_dof + a.num_dofs] = a.dof_targets[:, col]
            idx = np.array([a.global_index], dtype=np.int32)
            fn = (N.lib.mg_set_dof_position_target, N.lib.mg_set_dof_velocity_target,
                  N.lib.mg_set_dof_actuation_force)[col]
            N.check(fn(sim.native, full.ctypes.data, 1, idx.ctypes.data, 1, sim.stream()), "set dof column")
        return True

    def set_actor_dof_position_targets(self, env, handle, targets):
        return self._set_actor_dof_column(env, handle, targets, 0)

    def set_actor_dof_velocity_targets(self, env, handle, targets):
        return self._set_actor_dof_column(env, handle, targets, 1)

    def get_actor_dof_position_targets(self, env, handle):
        return self._actor(env, handle).dof_targets[:, 0].copy()

    def get_actor_dof_velocity_targets(self, env, handle):
        return self._actor(env, handle).dof_targets[:, 1].copy()

    def set_dof_target_position(self, env, dof_handle, target):
        a, d = self._dof_owner(env, dof_handle)
        vals = a.dof_targets[:, 0].copy()
        vals[d] = target
        return self._set_actor_dof_column(env, a.handle, vals, 0)

    def set_dof_target_velocity(self, env, dof_handle, target):
        a, d = self._dof_owner(env, dof_handle)
        vals = a.dof_targets[:, 1].copy()
        vals[d] = target
        return self._set_actor_dof_column(env, a.handle, vals, 1)

    def apply_dof_effort(self, env, dof_handle, effort):
        a, d = self._dof_owner(env, dof_handle)
        vals = a.dof_targets[:, 2].copy()
        vals[d] = effort
        return self._set_actor_dof_column(env, a.handle, vals, 2)

    def apply_actor_dof_efforts(self, env, handle, efforts):
        return self._set_actor_dof_column(env, handle, efforts, 2)

    # ---- DOF / body states (non-tensor API; slow path)
    def _host_state(self, sim):
        """Current (body_state[nb,13], dof_state[nd,2]) on the host."""
        sim.finalize()
        _check_held(sim, "a host state read", ("root",))
        if sim.native is None:
            A = sim.model_arrays
            return A["body_state0"].copy(), A["dof_state0"].copy()
        rb = np.zeros((sim.num_bodies, 13), dtype=np.float32)
        N.check(N.lib.mg_refresh_rigid_body_state(sim.native, rb.ctypes.data, 1, sim.stream()), "refresh")
        ds = np.zeros((max(sim.num_dofs, 1), 2), dtype=np.float32)
        if sim.num_dofs:
            N.check(N.lib.mg_refresh_dof_state(sim.native, ds.ctypes.data, 1, sim.stream()), "refresh")
        return rb, ds[:sim.num_dofs]

    def _host_dof_state(self, sim):
        """Current DOF state (nd, 2) on the host (no rigid-body download)."""
        ds = np.zeros((max(sim.num_dofs, 1), 2), dtype=np.float32)
        if sim.num_dofs:
            N.check(N.lib.mg_refresh_dof_state(sim.native, ds.ctypes.data, 1, sim.stream()), "refresh")
        return ds[:sim.num_dofs]

    def get_actor_dof_states(self, env, handle, flags=_T.STATE_ALL):
        a = self._actor(env, handle)
        out = np.zeros(a.num_dofs, dtype=DofState.dtype)
        if not env.sim.finalized:
            out["pos"], out["vel"] = a.dof_state[:, 0], a.dof_state[:, 1]
            return out
        ds = self._host_dof_state(env.sim) if env.sim.native else self._host_state(env.sim)[1]
        sl = ds[a.global_dof:a.global_dof + a.num_dofs]
        out["pos"], out["vel"] = sl[:, 0], sl[:, 1]
        return out

    def set_actor_dof_states(self, env, handle, states, flags=_T.STATE_ALL):
        a = self._actor(env, handle)
        st = np.asarray(states)
        if flags & _T.STATE_POS:
            a.dof_state[:, 0] = st["pos"][:a.num_dofs]
        if flags & _T.STATE_VEL:
            a.dof_state[:, 1] = st["vel"][:a.num_dofs]
        sim = env.sim
        if sim.finalized and sim.native and a.num_dofs:
            # start from the actor's current device state, so the column that
            # `flags` does not select keeps its simulated value (Isaac Gym leaves it
            # untouched: examples/joint_monkey.py:251 sets STATE_POS every frame);
            # both columns selected: nothing to merge, no download
            if (flags & _T.STATE_ALL) == _T.STATE_ALL:
                cur = a.dof_state.copy()
            else:
                cur = self._host_dof_state(sim)[a.global_dof:a.global_dof + a.num_dofs].copy()
            if flags & _T.STATE_POS:
                cur[:, 0] = a.dof_state[:, 0]
            if flags & _T.STATE_VEL:
                cur[:, 1] = a.dof_state[:, 1]
            a.dof_state[:] = cur
            full = np.zeros((sim.num_dofs, 2), dtype=np.float32)
            full[a.global_dof:a.global_dof + a.num_dofs] = cur
            idx = np.array([a.global_index], dtype=np.int32)
            sim.epoch += 1
            N.check(N.lib.mg_set_dof_state(sim.native, full.ctypes.data, 1, idx.ctypes.data, 1, sim.stream()),
                    "mg_set_dof_state")
        elif sim.finalized and a.num_dofs:
            # no device (scene-building host): the packed initial state is the state
            sim.model_arrays["dof_state0"][a.global_dof:a.global_dof + a.num_dofs] = a.dof_state
        return True

    def get_dof_position(self, env, dof_handle):
        a, d = self._dof_owner(env, dof_handle)
        return float(self.get_actor_dof_states(env, a.handle)["pos"][d])

    def get_dof_velocity(self, env, dof_handle):
        a, d = self._dof_owner(env, dof_handle)
        return float(self.get_actor_dof_states(env, a.handle)["vel"][d])

    def _rb_struct(self, rows):
        out = np.zeros(len(rows), dtype=RigidBodyState.dtype)
        for k, n in enumerate("xyz"):
            out["pose"]["p"][n] = rows[:, k]
            out["vel"]["linear"][n] = rows[:, 7 + k]
            out["vel"]["angular"][n] = rows[:, 10 + k]
        for k, n in enumerate("xyzw"):
            out["pose"]["r"][n] = rows[:, 3 + k]
        return out

    def _rb_rows(self, st):
        rows = np.zeros((len(st), 13), dtype=np.float32)
        for k, n in enumerate("xyz"):
            rows[:, k] = st["pose"]["p"][n]
            rows[:, 7 + k] = st["vel"]["linear"][n]
            rows[:, 10 + k] = st["vel"]["angular"][n]
        for k, n in enumerate("xyzw"):
            rows[:, 3 + k] = st["pose"]["r"][n]
        return rows

    def _pending_rows(self, actors):
        """Body-state rows of actors whose sim is still being built: the
        initial poses by forward kinematics (the state prepare_sim starts
        from), zero velocities but a root velocity set before it."""
        rows = []
        for a in actors:
            ps, qs = a.env.sim.actor_world_body_poses(a)
            r = np.zeros((a.num_bodies, 13), dtype=np.float32)
            r[:, 0:3] = np.asarray(ps, dtype=np.float64)
            r[:, 3:7] = np.asarray(qs, dtype=np.float64)
            if a.init_vel is not None:
                r[0, 7:13] = a.init_vel
            rows.append(r)
        return np.concatenate(rows, 0) if rows else np.zeros((0, 13), dtype=np.float32)

    def get_actor_rigid_body_states(self, env, handle, flags=_T.STATE_ALL):
        a = self._actor(env, handle)
        if not env.sim.finalized:           # during scene building: no state read finalizes the sim
            return self._rb_struct(self._pending_rows([a]))
        rb, _ = self._host_state(env.sim)
        return self._rb_struct(rb[a.global_body:a.global_body + a.num_bodies])

    def get_env_rigid_body_states(self, env, flags=_T.STATE_ALL):
        if not env.sim.finalized:
            return self._rb_struct(self._pending_rows(env.actors))
        rb, _ = self._host_state(env.sim)
        first = env.actors[0].global_body if env.actors else 0
        return self._rb_struct(rb[first:first + env.num_bodies])

    def get_sim_rigid_body_states(self, sim, flags=_T.STATE_ALL):
        if not sim.finalized:
            return self._rb_struct(self._pending_rows([a for e in sim.envs for a in e.actors]))
        rb, _ = self._host_state(sim)
        return self._rb_struct(rb)

    def _set_root_rows(self, sim, actors_rows):
        """Teleport actor roots: [(actor, row13)] through the indexed root setter.
        While the scene is being built (no prepare_sim, no tensor access yet) the
        row becomes the actor's creation pose and initial root velocity instead,
        so actors can still be added afterwards (examples/body_physics_props.py
        sets velocities between create_actor calls)."""
        if not sim.finalized:
            for a, row in actors_rows:
                o = a.env.origin
                a.pose = Transform(Vec3(float(row[0] - o[0]), float(row[1] - o[1]), float(row[2] - o[2])),
                                   Quat(float(row[3]), float(row[4]), float(row[5]), float(row[6])))
                a.init_vel = np.array(row[7:13], dtype=np.float32)
            return True
        sim.finalize()
        full = np.zeros((sim.num_actors, 13), dtype=np.float32)
        idx = np.zeros(len(actors_rows), dtype=np.int32)
        for k, (a, row) in enumerate(actors_rows):
            full[a.global_index] = row
            idx[k] = a.global_index
        if sim.native is None:
            A = sim.model_arrays
            for a, row in actors_rows:
                A["body_state0"][a.global_body] = row
            return True
        sim.epoch += 1
        N.check(N.lib.mg_set_actor_root_state(sim.native, full.ctypes.data, 1, idx.ctypes.data, len(idx),
                                              sim.stream()), "mg_set_actor_root_state")
        return True

    def set_actor_rigid_body_states(self, env, handle, states, flags=_T.STATE_ALL):
        a = self._actor(env, handle)
        cur = self.get_actor_rigid_body_states(env, handle)
        new = np.asarray(states)
        if flags & _T.STATE_POS:
            cur["pose"] = new["pose"][:len(cur)]
        if flags & _T.STATE_VEL:
            cur["vel"] = new["vel"][:len(cur)]
        return self._set_root_rows(env.sim, [(a, self._rb_rows(cur[:1])[0])])

    def set_sim_rigid_body_states(self, sim, states, flags=_T.STATE_ALL):
        cur = self.get_sim_rigid_body_states(sim)
        new = np.asarray(states)
        if flags & _T.STATE_POS:
            cur["pose"] = new["pose"]
        if flags & _T.STATE_VEL:
            cur["vel"] = new["vel"]
        rows = self._rb_rows(cur)
        if not sim.finalized:        # the pending rows' order: env by env, actor by actor
            acts = [a for e in sim.envs for a in e.actors]
            first = np.cumsum([0] + [a.num_bodies for a in acts])
            return self._set_root_rows(sim, [(a, rows[first[k]]) for k, a in enumerate(acts)])
        return self._set_root_rows(sim, [(a, rows[a.global_body]) for a in sim.actors])

    def set_rigid_linear_velocity(self, env, body_handle, vel):
        a = self._body_owner(env, body_handle)
        st = self.get_actor_rigid_body_states(env, a.handle)
        st["vel"]["linear"][0] = (vel.x, vel.y, vel.z)
        return self.set_actor_rigid_body_states(env, a.handle, st, _T.STATE_ALL)

    def set_rigid_angular_velocity(self, env, body_handle, vel):
        a = self._body_owner(env, body_handle)
        st = self.get_actor_rigid_body_states(env, a.handle)
        st["vel"]["angular"][0] = (vel.x, vel.y, vel.z)
        return self.set_actor_rigid_body_states(env, a.handle, st, _T.STATE_ALL)

    def set_rigid_transform(self, env, body_handle, transform):
        a = self._body_owner(env, body_handle)
        st = self.get_actor_rigid_body_states(env, a.handle)
        st["pose"]["p"][0] = (transform.p.x, transform.p.y, transform.p.z)
        st["pose"]["r"][0] = (transform.r.x, transform.r.y, transform.r.z, transform.r.w)
        return self.set_actor_rigid_body_states(env, a.handle, st, _T.STATE_ALL)

    def _body_owner(self, env, body_handle):
        for a in env.actors:
            if a.body_offset <= body_handle < a.body_offset + a.num_bodies:
                return a
        raise IndexError("invalid rigid body handle %r" % (body_handle,))

    def get_rigid_transform(self, env, body_handle):
        """examples/franka_cube_ik_osc.py:272."""
        a = self._body_owner(env, body_handle)
        env.sim._assign_indices()
        if env.sim.finalized:
            rb, _ = self._host_state(env.sim)
            r = rb[a.global_body + body_handle - a.body_offset]
            return Transform(Vec3(*r[0:3]), Quat(*r[3:7]))
        ps, qs = env.sim.actor_world_body_poses(a)
        k = body_handle - a.body_offset
        return Transform(Vec3(*ps[k]), Quat(*qs[k]))

    # ---- rigid body / shape properties
    def get_actor_rigid_body_properties(self, env, handle):
        a = self._actor(env, handle)
        out = []
        for mp in a.mass_props:
            p = RigidBodyProperties(mp.mass, Vec3(*mp.com))
            p.inertia = _T.Mat33(Vec3(*mp.inertia[0]), Vec3(*mp.inertia[1]), Vec3(*mp.inertia[2]))
            out.append(p)
        return out

    def set_actor_rigid_body_properties(self, env, handle, props, recomputeInertia=False):
        a = self._actor(env, handle)
        if env.sim.finalized:
            print("*** migym: rigid body properties are frozen after prepare_sim", file=sys.stderr)
            return False
        new = []
        for mp, p in zip(a.mass_props, props):
            I = mp.inertia
            if getattr(p, "inertia", None) is not None and not recomputeInertia:
                I = np.array([[p.inertia.x.x, p.inertia.x.y, p.inertia.x.z], [p.inertia.y.x, p.inertia.y.y,
                              p.inertia.y.z], [p.inertia.z.x, p.inertia.z.y, p.inertia.z.z]])
            if recomputeInertia and mp.mass > 0:
                I = mp.inertia * (p.mass / mp.mass)
            new.append(_assets.MassProps(p.mass, [p.com.x, p.com.y, p.com.z], I))
        a.mass_props = new          # a private list: the actor no longer shares the asset's
        return True

    def get_actor_rigid_shape_properties(self, env, handle):
        return [_copy_shape(sp) for sp in self._actor(env, handle).shape_props]

    def set_actor_rigid_shape_properties(self, env, handle, props):
        a = self._actor(env, handle)
        if env.sim.finalized:
            print("*** migym: shape properties are frozen after prepare_sim", file=sys.stderr)
            return False
        a.shape_props = [_copy_shape(sp) for sp in props]
        return True

    def set_rigid_body_color(self, env, handle, body_index, mesh_type, color):
        self._actor(env, handle).body_colors[body_index] = Vec3(color.x, color.y, color.z)
        env.sim.render_version += 1

    def get_rigid_body_color(self, env, handle, body_index, mesh_type):
        return self._actor(env, handle).body_colors.get(body_index, Vec3(1, 1, 1))

    def set_rigid_body_segmentation_id(self, env, handle, body_index, seg):
        self._actor(env, handle).body_segs[body_index] = int(seg)
        env.sim.render_version += 1

    # textures (examples/domain_randomization.py:91,179, graphics.py:100): handles
    # are kept per body, but the camera renderer draws a body in its colour
    # (set_rigid_body_color) — texture sampling is not modelled
    def create_texture_from_file(self, sim, filename):
        if not os.path.isfile(filename):
            print("*** migym: texture file %s not found" % filename, file=sys.stderr)
            return -1
        sim.textures.append(os.path.abspath(filename))
        return len(sim.textures) - 1

    def create_texture_from_buffer(self, sim, width, height, pixels):
        sim.textures.append((int(width), int(height)))
        return len(sim.textures) - 1

    def free_texture(self, sim, tex):
        return None

    def set_rigid_body_texture(self, env, handle, body_index, mesh_type, tex):
        self._actor(env, handle).body_textures[body_index] = int(tex)

    def get_rigid_body_texture(self, env, handle, body_index, mesh_type):
        return self._actor(env, handle).body_textures.get(body_index, -1)

    def set_actor_scale(self, env, handle, scale):
        """examples/actor_scaling.py:126. Scales the actor's collision geometry
        and joint frames by `scale` and its mass properties with them (mass by
        scale^3, inertia by scale^5, centres of mass by scale), as a body of the
        same density would. Before prepare_sim only: the packed model is frozen
        after it (returns False, said on stderr)."""
        a = self._actor(env, handle)
        scale = float(scale)
        if env.sim.finalized:
            print("*** migym: actor scale is frozen after prepare_sim", file=sys.stderr)
            return False
        if not scale > 0.0:
            return False
        r = scale / a.scale
        if r != 1.0:
            a.mass_props = [_assets.MassProps(mp.mass * r ** 3, mp.com * r, mp.inertia * r ** 5) for mp in a.mass_props]
            a.scale = scale
        return True

    def get_actor_scale(self, env, handle):
        return self._actor(env, handle).scale

    # ================================================================ tensor API
    def _acquire(self, sim, key):
        sim.finalize()
        return Tensor(sim.tensors[key])

    def acquire_actor_root_state_tensor(self, sim):
        """test10_servo_vecenv.py:372,400: the same storage on every call."""
        return self._acquire(sim, "root")

    def acquire_rigid_body_state_tensor(self, sim):
        return self._acquire(sim, "rb")

    def acquire_dof_state_tensor(self, sim):
        return self._acquire(sim, "dof")

    def acquire_net_contact_force_tensor(self, sim):
        return self._acquire(sim, "ncf")

    def _refresh(self, sim, key, fn, what):
        sim.finalize()
        t = sim.tensors[key]
        if t.numel() == 0:
            return True
        h = sim.require_native(what)
        if key in ("root", "rb"):
            _check_held(sim, what, ("root",))      # flushes a pending root set
        stale = ((key == "rb" and sim.rb_paired_version is not None and t._version != sim.rb_paired_version) or
                 (key == "root" and sim.root_out_version is not None and t._version != sim.root_out_version))
        if stale:
            # the user wrote the tensor after the paired root refresh or the step
            # (STEP_FUSION_STEP_OUT) filled it: re-gather it (rebinding clears the
            # served-without-launch marks)
            N.check(N.lib.mg_bind_refresh_targets(h, sim.tensors["root"].data_ptr(), sim.tensors["rb"].data_ptr()),
                    "mg_bind_refresh_targets")
        if key == "dof" and sim.dof_out_version is not None and t._version != sim.dof_out_version:
            N.check(N.lib.mg_bind_dof_refresh_target(h, t.data_ptr()), "mg_bind_dof_refresh_target")
        bit = _STAGE_BIT[key]
        if t.device.type == "cpu" and sim.host_stage_epoch == sim.epoch and sim.host_staged & bit:
            # CPU pipeline after fetch_results(sim, True): no simulate and no
            # state set since the staged copy — a host copy, no device round trip
            o = sim.host_stage_offsets[key]
            t.view(-1).copy_(sim.host_stage[o:o + t.numel()])
        else:
            N.check(fn(h, t.data_ptr(), 1 if t.device.type == "cpu" else 0, sim.stream()), what)
            if t.device.type == "cpu":
                sim.host_stage_parts |= bit      # stage this kind at the next fetch_results(sim, True)
        # the tensor now holds the sim state, whether this refresh launched a
        # gather or was served by the step / the paired gather: a later in-place
        # write makes the next refresh rebind and gather again, as Isaac Gym's
        # refresh overwrites it (write -> refresh -> write -> refresh)
        # (device tensors only: a host tensor of the CPU pipeline is bound to nothing)
        ver = t._version if t.is_cuda else None
        if key == "root":
            sim.root_out_version = ver
            if sim.fusion & STEP_FUSION_REFRESH:
                sim.rb_paired_version = sim.tensors["rb"]._version
        elif key == "dof":
            sim.dof_out_version = ver
        elif key == "rb":
            sim.rb_paired_version = ver
        return True

    def refresh_actor_root_state_tensor(self, sim):
        return self._refresh(sim, "root", N.lib.mg_refresh_actor_root_state, "refresh_actor_root_state_tensor")

    def refresh_rigid_body_state_tensor(self, sim):
        return self._refresh(sim, "rb", N.lib.mg_refresh_rigid_body_state, "refresh_rigid_body_state_tensor")

    def refresh_dof_state_tensor(self, sim):
        """test10_servo_vecenv.py:396: zero DOFs is an empty tensor, not an error."""
        return self._refresh(sim, "dof", N.lib.mg_refresh_dof_state, "refresh_dof_state_tensor")

    def refresh_net_contact_force_tensor(self, sim):
        return self._refresh(sim, "ncf", N.lib.mg_refresh_net_contact_force, "refresh_net_contact_force_tensor")

    def _set(self, sim, tensor, fn, ncols, nrows, what, index=None, count=None):
        sim.finalize()
        sim.epoch += 1
        t = _as_tensor_arg(tensor, what)
        kind = _FUSED_KIND.get(getattr(fn, "__name__", ""))
        if kind is not None:
            _check_held(sim, what, (kind,))        # a set of the same kind applies / replaces the pending one
        if t.dtype != torch.float32 or t.numel() != nrows * ncols:
            print("*** migym: %s: expected a float32 tensor of %d x %d" % (what, nrows, ncols), file=sys.stderr)
            return False
        if nrows == 0:
            return True
        host = 1 if t.device.type == "cpu" else 0
        if index is not None:
            it = _as_tensor_arg(index, what + " indices")
            if it.dtype != torch.int32:
                print("*** migym: %s: indices must be int32" % what, file=sys.stderr)
                return False
            it = it.reshape(-1)
            n = int(count) if count is not None else it.numel()
            if n < 0 or n > it.numel():
                print("*** migym: %s: count %d outside [0, %d] (index tensor size)" % (what, n, it.numel()),
                      file=sys.stderr)
                return False
            na = sim_num(sim, "actors")
            # index range check on the host (skipped while a graph is being captured:
            # the copy kernels skip out-of-range rows on the device as well)
            if n > 0 and not (it.is_cuda and torch.cuda.is_current_stream_capturing()):
                lo, hi = int(it[:n].min()), int(it[:n].max())
                if lo < 0 or hi >= na:
                    print("*** migym: %s: actor index %d outside [0, %d)" % (what, lo if lo < 0 else hi, na),
                          file=sys.stderr)
                    return False
            if (it.device.type == "cpu") != (t.device.type == "cpu"):
                it = it.to(t.device)
            it = it.contiguous()
            rc = fn(sim.require_native(what), t.data_ptr(), host, it.data_ptr(), n, sim.stream())
        else:
            h = sim.require_native(what)
            rc = fn(h, t.data_ptr(), host, None, 0, sim.stream())
            # a fused set (opt-in: STEP_FUSION_ROOT_SET / _DOF_TARGETS) whose read
            # the library deferred to the next simulate: keep its tensor alive
            # until then and remember its version, so a write to it before that
            # read raises (_check_held); a set the library copied at the call
            # (host source, a flag not set, a scene it cannot fuse) holds nothing
            if kind is not None and rc == N.MG_OK and N.lib.mg_last_set_deferred(h):
                sim.held_src.append((t, t._version, what, kind))
        if rc != N.MG_OK:
            print("*** migym: %s: %s" % (what, N.last_error()), file=sys.stderr)
            return False
        return True

    def set_actor_root_state_tensor(self, sim, tensor):
        """test10_servo_vecenv.py:456: teleports all actor roots; returns bool."""
        return self._set(sim, tensor, N.lib.mg_set_actor_root_state, 13, sim_num(sim, "actors"),
                         "set_actor_root_state_tensor")

    def set_actor_root_state_tensor_indexed(self, sim, tensor, indices, count):
        return self._set(sim, tensor, N.lib.mg_set_actor_root_state, 13, sim_num(sim, "actors"),
                         "set_actor_root_state_tensor_indexed", indices, count)

    def set_rigid_body_state_tensor(self, sim, tensor):
        sim.finalize()
        t = _as_tensor_arg(tensor, "set_rigid_body_state_tensor")
        _check_held(sim, "set_rigid_body_state_tensor", ("root",))
        if t.numel() != sim.num_bodies * 13:
            return False
        h = sim.require_native("set_rigid_body_state_tensor")
        sim.epoch += 1
        rc = N.lib.mg_set_rigid_body_state(h, t.data_ptr(), 1 if t.device.type == "cpu" else 0, sim.stream())
        return rc == N.MG_OK

    def set_dof_state_tensor(self, sim, tensor):
        return self._set(sim, tensor, N.lib.mg_set_dof_state, 2, sim_num(sim, "dofs"), "set_dof_state_tensor")

    def set_dof_state_tensor_indexed(self, sim, tensor, indices, count):
        return self._set(sim, tensor, N.lib.mg_set_dof_state, 2, sim_num(sim, "dofs"),
                         "set_dof_state_tensor_indexed", indices, count)

    def set_dof_position_target_tensor(self, sim, tensor):
        """examples/franka_cube_ik_osc.py:409."""
        return self._set(sim, tensor, N.lib.mg_set_dof_position_target, 1, sim_num(sim, "dofs"),
                         "set_dof_position_target_tensor")

    def set_dof_position_target_tensor_indexed(self, sim, tensor, indices, count):
        return self._set(sim, tensor, N.lib.mg_set_dof_position_target, 1, sim_num(sim, "dofs"),
                         "set_dof_position_target_tensor_indexed", indices, count)

    def set_dof_velocity_target_tensor(self, sim, tensor):
        return self._set(sim, tensor, N.lib.mg_set_dof_velocity_target, 1, sim_num(sim, "dofs"),
                         "set_dof_velocity_target_tensor")

    def set_dof_velocity_target_tensor_indexed(self, sim, tensor, indices, count):
        return self._set(sim, tensor, N.lib.mg_set_dof_velocity_target, 1, sim_num(sim, "dofs"),
                         "set_dof_velocity_target_tensor_indexed", indices, count)

    def set_dof_actuation_force_tensor(self, sim, tensor):
        """examples/franka_cube_ik_osc.py:410."""
        return self._set(sim, tensor, N.lib.mg_set_dof_actuation_force, 1, sim_num(sim, "dofs"),
                         "set_dof_actuation_force_tensor")

    def set_dof_actuation_force_tensor_indexed(self, sim, tensor, indices, count):
        return self._set(sim, tensor, N.lib.mg_set_dof_actuation_force, 1, sim_num(sim, "dofs"),
                         "set_dof_actuation_force_tensor_indexed", indices, count)

    def apply_rigid_body_force_tensors(self, sim, forceTensor=None, torqueTensor=None, space=_T.ENV_SPACE):
        sim.finalize()
        h = sim.require_native("apply_rigid_body_force_tensors")
        tensors = [_as_tensor_arg(x, "apply_rigid_body_force_tensors") if x is not None else None
                   for x in (forceTensor, torqueTensor)]
        given = [t for t in tensors if t is not None]
        if not given:
            return True
        if len({t.device for t in given}) > 1:
            print("*** migym: apply_rigid_body_force_tensors: force and torque tensors on different devices "
                  "(%s)" % ", ".join(str(t.device) for t in given), file=sys.stderr)
            return False
        if any(t.dtype != torch.float32 or t.numel() != sim.num_bodies * 3 for t in given):
            print("*** migym: apply_rigid_body_force_tensors: expected float32 tensors of %d x 3"
                  % sim.num_bodies, file=sys.stderr)
            return False
        tensors = [t.contiguous() if t is not None else None for t in tensors]
        host = 1 if given[0].device.type == "cpu" else 0
        ptr = [t.data_ptr() if t is not None else None for t in tensors]
        mg_space = 1 if space == _T.LOCAL_SPACE else 0
        rc = N.lib.mg_apply_rigid_body_force(h, ptr[0], ptr[1], mg_space, host, sim.stream())
        if rc != N.MG_OK:
            print("*** migym: apply_rigid_body_force_tensors: %s" % N.last_error(), file=sys.stderr)
            return False
        return True

    def apply_rigid_body_force_at_pos_tensors(self, sim, forceTensor, posTensor=None, space=_T.ENV_SPACE):
        """examples/apply_forces_at_pos.py:126: forces (num_bodies, 3) applied at
        points (num_bodies, 3) during the next simulate — the same as the force
        at the centre of mass plus the torque (p - c) x F. ENV_SPACE / GLOBAL_SPACE:
        points in the rigid-body tensor's frame (the example passes the refreshed
        body positions plus an offset); LOCAL_SPACE: force and point in the body
        frame. No points: forces at the centres of mass."""
        if posTensor is None:
            return self.apply_rigid_body_force_tensors(sim, forceTensor, None, space)
        sim.finalize()
        h = sim.require_native("apply_rigid_body_force_at_pos_tensors")
        F = _as_tensor_arg(forceTensor, "apply_rigid_body_force_at_pos_tensors")
        P = _as_tensor_arg(posTensor, "apply_rigid_body_force_at_pos_tensors")
        nb = sim.num_bodies
        if (F.dtype != torch.float32 or P.dtype != torch.float32 or F.numel() != nb * 3 or P.numel() != nb * 3
                or F.device != P.device):
            print("*** migym: apply_rigid_body_force_at_pos_tensors: expected float32 tensors of %d x 3 on one "
                  "device" % nb, file=sys.stderr)
            return False
        dev = F.device
        F = F.reshape(nb, 3)
        P = P.reshape(nb, 3)
        # the bodies' current state (a gather into a scratch tensor: the caller's
        # tensors are left alone) and their centres of mass in the body frame
        st = torch.empty((nb, 13), dtype=torch.float32, device=dev)
        N.check(N.lib.mg_refresh_rigid_body_state(h, st.data_ptr(), 1 if dev.type == "cpu" else 0, sim.stream()),
                "apply_rigid_body_force_at_pos_tensors")
        com = getattr(sim, "_com_local", None)
        if com is None or com.device != dev:
            com = torch.from_numpy(np.ascontiguousarray(sim.model_arrays["body_mass"][:, 8:11],
                                                        dtype=np.float32)).to(dev)
            sim._com_local = com
        x, q = st[:, 0:3], st[:, 3:7]

        def rot(v):           # q (x, y, z, w) applied to v
            u, w = q[:, 0:3], q[:, 3:4]
            t = 2.0 * torch.cross(u, v, dim=1)
            return v + w * t + torch.cross(u, t, dim=1)

        c = x + rot(com)
        if space == _T.LOCAL_SPACE:
            F = rot(F)
            P = x + rot(P)
        tau = torch.cross(P - c, F, dim=1)
        return self.apply_rigid_body_force_tensors(sim, F.contiguous(), tau.contiguous(), _T.ENV_SPACE)

    def _artic_template(self, sim, actor_name):
        """(template id, asset) of the articulated actors named actor_name; the
        tensors cover every instance of that template, in actor order."""
        sim.finalize()
        A = sim.model_arrays
        for a in sim.actors:
            if a.name == actor_name and len(a.asset.bodies) > 1:
                for row in A["artic_i"]:
                    if row[0] == a.global_body:
                        t = int(row[2])
                        named = sum(1 for b in sim.actors if b.name == actor_name and b.asset is a.asset)
                        if named != int((A["artic_i"][:, 2] == t).sum()):
                            raise ValueError("actors named %r must be exactly the instances of one asset" % actor_name)
                        return t, a.asset
        raise KeyError("no articulated actor named %r" % (actor_name,))

    def acquire_jacobian_tensor(self, sim, actor_name):
        """examples/franka_cube_ik_osc.py:305: (num_envs, links-1, 6, dofs) for a fixed base."""
        t, asset = self._artic_template(sim, actor_name)
        if actor_name not in sim.jacobians:
            n = sum(1 for a in sim.actors if a.name == actor_name)
            fixed = asset.options.fix_base_link
            nl = len(asset.bodies) - (1 if fixed else 0)
            nd = asset.num_dofs + (0 if fixed else 6)
            sim.jacobians[actor_name] = (t, torch.zeros((n, nl, 6, nd), dtype=torch.float32, device=sim.device))
        return Tensor(sim.jacobians[actor_name][1])

    def acquire_mass_matrix_tensor(self, sim, actor_name):
        """examples/franka_cube_ik_osc.py:315: (num_envs, dofs, dofs) for a fixed base."""
        t, asset = self._artic_template(sim, actor_name)
        if actor_name not in sim.mass_matrices:
            n = sum(1 for a in sim.actors if a.name == actor_name)
            nd = asset.num_dofs + (0 if asset.options.fix_base_link else 6)
            sim.mass_matrices[actor_name] = (t, torch.zeros((n, nd, nd), dtype=torch.float32, device=sim.device))
        return Tensor(sim.mass_matrices[actor_name][1])

    def refresh_jacobian_tensors(self, sim):
        """examples/franka_cube_ik_osc.py:345. When the actor's mass-matrix tensor is
        acquired too, one launch also computes it (same kinematics) into a cache that
        refresh_mass_matrix_tensors copies from while the state is unchanged."""
        h = sim.require_native("refresh_jacobian_tensors")
        for name, (t, ten) in sim.jacobians.items():
            host = 1 if ten.device.type == "cpu" else 0
            if name in sim.mass_matrices:
                mm = sim.mass_matrices[name][1]
                cache = sim.mm_cache.get(name)
                if cache is None or cache[1].shape != mm.shape or cache[1].device != mm.device:
                    cache = (None, torch.empty_like(mm))
                N.check(N.lib.mg_refresh_jacobian_mass_matrix(h, t, ten.data_ptr(), cache[1].data_ptr(), host,
                                                              sim.stream()), "refresh_jacobian_tensors(%s)" % name)
                sim.mm_cache[name] = (sim.epoch, cache[1])
            else:
                N.check(N.lib.mg_refresh_jacobian(h, t, ten.data_ptr(), host, sim.stream()),
                        "refresh_jacobian_tensors(%s)" % name)
        return True

    def refresh_mass_matrix_tensors(self, sim):
        """examples/franka_cube_ik_osc.py:346."""
        h = sim.require_native("refresh_mass_matrix_tensors")
        for name, (t, ten) in sim.mass_matrices.items():
            cache = sim.mm_cache.get(name)
            if cache is not None and cache[0] == sim.epoch:
                ten.copy_(cache[1])
                continue
            N.check(N.lib.mg_refresh_mass_matrix(h, t, ten.data_ptr(), 1 if ten.device.type == "cpu" else 0,
                                                 sim.stream()), "refresh_mass_matrix_tensors(%s)" % name)
        return True

    # ================================================================ viewer (headless)
    def create_viewer(self, sim, props):
        return Viewer(sim, props)

    def destroy_viewer(self, viewer):
        pass

    def query_viewer_has_closed(self, viewer):
        return viewer is None or viewer.frames >= viewer.max_frames

    def draw_viewer(self, viewer, sim, render_collision=False):
        if viewer is not None:
            viewer.frames += 1

    def step_graphics(self, sim):
        pass

    def sync_frame_time(self, sim):
        """Real-time throttle in Isaac Gym (test10_servo_vecenv.py:392): a no-op here."""

    def poll_viewer_events(self, viewer):
        pass

    def viewer_camera_look_at(self, viewer, env, pos, target):
        if viewer is not None:
            viewer.cam_transform = Transform(pos, Quat())

    def get_viewer_camera_transform(self, viewer, env):
        return viewer.cam_transform if viewer is not None else Transform()

    def get_viewer_size(self, viewer):
        return Vec3(_T.DEFAULT_VIEWER_WIDTH, _T.DEFAULT_VIEWER_HEIGHT, 0)

    def get_viewer_mouse_position(self, viewer):
        return Vec3(0.5, 0.5, 0)

    def subscribe_viewer_keyboard_event(self, viewer, key, action):
        pass

    def subscribe_viewer_mouse_event(self, viewer, button, action):
        pass

    def query_viewer_action_events(self, viewer):
        return []

    def add_lines(self, viewer, env, num_lines, vertices, colors):
        pass

    def clear_lines(self, viewer):
        pass

    def set_light_parameters(self, sim, light_index, intensity, ambient, direction):
        """examples/domain_randomization.py:186: the directional light of the
        camera renders (include/migym.h mg_set_light): per channel, a body is
        drawn as colour * (ambient + intensity * max(n . direction, 0)),
        direction pointing towards the light. One light (index 0) is modelled."""
        if light_index != 0:
            print("*** migym: set_light_parameters: only light 0 is modelled", file=sys.stderr)
            return
        L = N.MgLight()
        L.dir[:] = (direction.x, direction.y, direction.z)
        L.color[:] = (intensity.x, intensity.y, intensity.z)
        L.ambient[:] = (ambient.x, ambient.y, ambient.z)
        if not (direction.x ** 2 + direction.y ** 2 + direction.z ** 2) > 0.0:
            print("*** migym: set_light_parameters: zero direction", file=sys.stderr)
            return
        sim.light = L
        if sim.native:
            N.check(N.lib.mg_set_light(sim.native, ctypes.byref(L)), "mg_set_light")

    def draw_env_rigid_contacts(self, viewer, env, color, scale, flag):
        pass

    # ================================================================ cameras (device ray caster)
    def create_camera_sensor(self, env, props):
        """Per-env 0-based handles (test11's aliased list needs that)."""
        p = _T.CameraProperties()
        p.__dict__.update(props.__dict__)          # test11 mutates its props between cameras (:327-329)
        cam = CameraSensor(env, p, len(env.cameras))
        env.cameras.append(cam)
        env.sim.cam_version += 1
        return cam.handle

    def destroy_camera_sensor(self, sim, env, handle):
        """The camera is no longer rendered and its images can no longer be read
        (the other cameras keep their handles)."""
        cam = env.cameras[handle]
        cam.destroyed = True
        cam.images = {}
        sim.cam_version += 1

    def set_camera_location(self, handle, env, pos, target):
        """examples/interop_torch.py:111: env-frame position looking at target."""
        cam = env.cameras[handle]
        cam.body = None
        cam.transform = _render.look_at(pos, target, env.sim.params.up_axis)
        env.sim.cam_version += 1

    def set_camera_transform(self, handle, env, transform):
        cam = env.cameras[handle]
        cam.body = None
        cam.transform = Transform(transform.p, transform.r)
        env.sim.cam_version += 1

    def attach_camera_to_body(self, handle, env, body_handle, local_transform, follow_mode):
        """test11_servo_vecenv_camerazoom.py:333-336 (FOLLOW_TRANSFORM)."""
        cam = env.cameras[handle]
        cam.body = body_handle
        cam.local = Transform(local_transform.p, local_transform.r)
        cam.follow = follow_mode
        env.sim.cam_version += 1

    def get_camera_transform(self, sim, env, handle):
        cam = env.cameras[handle]
        if cam.body is None:
            o = env.origin
            return Transform(Vec3(o[0], o[1], o[2]), Quat()) * cam.transform
        b = self.get_rigid_transform(env, cam.body)
        if cam.follow == _T.FOLLOW_POSITION:
            return Transform(b.p + cam.local.p, cam.local.r)
        return b * cam.local

    def get_camera_view_matrix(self, sim, env, handle):
        t = self.get_camera_transform(sim, env, handle)
        inv = t.inverse()
        R = _assets._qmat(np.array([inv.r.x, inv.r.y, inv.r.z, inv.r.w]))
        m = np.eye(4, dtype=np.float32)
        m[:3, :3] = R.T
        m[3, :3] = [inv.p.x, inv.p.y, inv.p.z]
        return m

    def get_camera_proj_matrix(self, sim, env, handle):
        p = env.cameras[handle].props
        fx = 1.0 / math.tan(math.radians(p.horizontal_fov) * 0.5)
        fy = fx * p.width / p.height
        n = p.near_plane
        m = np.zeros((4, 4), dtype=np.float32)
        m[0, 0], m[1, 1] = fx, fy
        m[2, 2] = 0.0
        m[2, 3] = -1.0
        m[3, 2] = n
        return m

    def set_camera_proj_matrix(self, *args):
        pass

    def render_all_camera_sensors(self, sim):
        """test11_servo_vecenv_camerazoom.py:388: freezes the poses the cameras
        see and renders every camera that has a GPU image tensor (one launch)."""
        _check_held(sim, "render_all_camera_sensors", ("root",))
        return sim.renderer.render_all()

    def start_access_image_tensors(self, sim):
        pass

    def end_access_image_tensors(self, sim):
        pass

    def get_camera_image(self, sim, env, handle, image_type):
        """test11_servo_vecenv_camerazoom.py:459: host image of the last render
        (color (H, W*4) uint8, depth (H, W) float32, segmentation (H, W) int32)."""
        if env.cameras[handle].destroyed:
            raise ValueError("camera %d of env %d was destroyed" % (handle, env.index))
        if image_type not in _render.IMAGE_KINDS:
            p = env.cameras[handle].props
            return np.zeros((p.height, p.width), dtype=np.float32)
        return sim.renderer.image(env.cameras[handle], image_type)

    def get_camera_image_gpu_tensor(self, sim, env, handle, image_type):
        """examples/interop_torch.py:116: the camera's persistent device image,
        updated by every render_all_camera_sensors."""
        cam = env.cameras[handle]
        if image_type not in _render.IMAGE_KINDS:
            raise ValueError("image type %r is not rendered" % (image_type,))
        return Tensor(_render.image_tensor(sim, cam, image_type))

    def write_camera_image_to_file(self, sim, env, handle, image_type, filename):
        """examples/domain_randomization.py:192 (--save_images): the last render
        of the camera as a PNG — color as RGBA, depth as 16-bit millimetres of
        -depth (Isaac Gym's depth is negative along the view axis; 0 = no hit;
        clipped at 65.535 m),
        segmentation as 16-bit ids. False when the image cannot be written."""
        from PIL import Image
        img = self.get_camera_image(sim, env, handle, image_type)
        try:
            if image_type == _T.IMAGE_COLOR:
                h = img.shape[0]
                Image.fromarray(np.ascontiguousarray(img.reshape(h, -1, 4)), "RGBA").save(filename)
            elif image_type == _T.IMAGE_DEPTH:
                d = np.nan_to_num(-np.asarray(img, dtype=np.float64), posinf=0.0, neginf=0.0)
                Image.fromarray(np.clip(np.rint(d * 1000.0), 0, 65535).astype(np.uint16)).save(filename)
            else:
                Image.fromarray(np.clip(np.asarray(img), 0, 65535).astype(np.uint16)).save(filename)
        except OSError as e:
            print("*** migym: cannot write %s: %s" % (filename, e), file=sys.stderr)
            return False
        return True

    def write_viewer_image_to_file(self, viewer, filename):
        """The viewer is headless (no window, nothing drawn): no image to write."""
        return False


def sim_num(sim, what):
    sim.finalize()
    return {"actors": sim.num_actors, "bodies": sim.num_bodies, "dofs": sim.num_dofs}[what]


def _copy_shape(sp):
    c = _T.RigidShapeProperties()
    c.__dict__.update(sp.__dict__)
    return c


def _copy_options(o):
    c = _T.AssetOptions()
    c.__dict__.update(o.__dict__)
    return c


_GYM = None


def acquire_gym():
    """gymapi.acquire_gym() (test10_servo_vecenv.py:177): the singleton Gym."""
    global _GYM
    if _GYM is None:
        _GYM = Gym()
    return _GYM
