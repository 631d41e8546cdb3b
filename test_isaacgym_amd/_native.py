"""ctypes binding of libmigym.so, the C ABI declared in include/migym.h.

The product path has exactly one engine: the HIP kernels in this library. There
is no CPU or PyTorch fallback — if the library is missing, importing the package
raises, and on a host without a GPU ``mg_create_sim`` fails and
``gym.simulate`` raises (see gymapi.Gym.simulate).
"""
import ctypes
import os

import torch  # noqa: F401  -- load torch's HIP runtime first, so libmigym binds to the same one

_HERE = os.path.dirname(os.path.abspath(__file__))
# MIGYM_LIB selects another build of the same library (kernel A/B experiments:
# tools/kbench.py); the default is the in-tree libmigym.so.
LIB_PATH = os.environ.get("MIGYM_LIB") or os.path.join(_HERE, "libmigym.so")

MG_OK = 0
MG_STATE_N = 13
MG_MASS_N = 12
MG_TBODY_F_N = 8
MG_TBODY_I_N = 4
MG_SHAPE_STRIDE = 16
MG_DOFPROP_N = 12
MG_LINK_F_N = 16
MG_LINK_I_N = 4
MG_ARTIC_I_N = 4
MG_DEBUG_GROUP_N = 8       # include/migym.h mg_debug_artic_groups
MG_ATMPL_I_N = 4
MG_ACOLL_N = 4

MG_SHAPE_SPHERE, MG_SHAPE_BOX, MG_SHAPE_CAPSULE, MG_SHAPE_CONVEX = 0, 1, 2, 3
MG_HULL_HEADER, MG_HULL_MAX_VERTS, MG_HULL_MAX_FACES = 4, 255, 255   # include/migym.h
MG_BODY_FREE, MG_BODY_STATIC, MG_BODY_LINK = 0, 1, 2

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)


class MgSimParams(ctypes.Structure):
    _fields_ = [
        ("dt", ctypes.c_float),
        ("substeps", ctypes.c_int32),
        ("gravity", ctypes.c_float * 3),
        ("up_axis", ctypes.c_int32),
        ("num_position_iterations", ctypes.c_int32),
        ("num_velocity_iterations", ctypes.c_int32),
        ("contact_offset", ctypes.c_float),
        ("rest_offset", ctypes.c_float),
        ("bounce_threshold_velocity", ctypes.c_float),
        ("max_depenetration_velocity", ctypes.c_float),
        ("has_ground", ctypes.c_int32),
        ("ground_normal", ctypes.c_float * 3),
        ("ground_distance", ctypes.c_float),
        ("ground_static_friction", ctypes.c_float),
        ("ground_dynamic_friction", ctypes.c_float),
        ("ground_restitution", ctypes.c_float),
        ("friction_offset_threshold", ctypes.c_float),
        ("friction_correlation_distance", ctypes.c_float),
        ("reserved", ctypes.c_int32 * 6),
    ]


class MgModel(ctypes.Structure):
    _fields_ = [
        ("num_envs", ctypes.c_int32), ("num_actors", ctypes.c_int32),
        ("num_bodies", ctypes.c_int32), ("num_dofs", ctypes.c_int32),
        ("num_tmpl_bodies", ctypes.c_int32), ("num_shapes", ctypes.c_int32),
        ("num_artics", ctypes.c_int32), ("num_artic_tmpls", ctypes.c_int32),
        ("num_tmpl_links", ctypes.c_int32),
        ("num_hull_floats", ctypes.c_int32),
        ("reserved_i", ctypes.c_int32 * 6),
        ("body_state0", _f32p), ("body_mass", _f32p), ("body_kind", _i32p), ("body_tmpl", _i32p),
        ("tmpl_body_f", _f32p), ("tmpl_body_i", _i32p), ("shapes", _f32p),
        ("actor_root_body", _i32p), ("actor_dof", _i32p),
        ("dof_state0", _f32p), ("dof_props", _f32p),
        ("artic_i", _i32p), ("artic_tmpl_i", _i32p), ("tmpl_link_f", _f32p), ("tmpl_link_i", _i32p),
        ("actor_coll", _i32p),
        ("hulls", _f32p),
        ("reserved_p", ctypes.c_void_p * 1),
    ]


class MgCamera(ctypes.Structure):
    """mg_camera (include/migym.h): one camera sensor to render."""
    _fields_ = [
        ("env", ctypes.c_int32), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("body", ctypes.c_int32), ("follow", ctypes.c_int32),
        ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
        ("near_plane", ctypes.c_float), ("far_plane", ctypes.c_float),
        ("p", ctypes.c_float * 3), ("q", ctypes.c_float * 4),
        ("reserved", ctypes.c_int32),
        ("color", ctypes.c_void_p), ("depth", ctypes.c_void_p), ("seg", ctypes.c_void_p),
    ]


class MgLight(ctypes.Structure):
    """mg_light (include/migym.h): the renderer's directional light."""
    _fields_ = [("dir", ctypes.c_float * 3), ("color", ctypes.c_float * 3), ("ambient", ctypes.c_float * 3)]


MG_RENDER_MAX_SHAPES = 64


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libmigym.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no fallback engine." % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    sig = {
        "mg_abi_version": (i32, []),
        "mg_last_error": (ctypes.c_char_p, []),
        "mg_device_count": (i32, []),
        "mg_create_sim": (vp, [i32, ctypes.POINTER(MgSimParams)]),
        "mg_destroy_sim": (None, [vp]),
        "mg_set_sim_params": (i32, [vp, ctypes.POINTER(MgSimParams)]),
        "mg_upload_model": (i32, [vp, ctypes.POINTER(MgModel)]),
        "mg_simulate": (i32, [vp, vp]),
        "mg_fetch_results": (i32, [vp, i32]),
        "mg_refresh_actor_root_state": (i32, [vp, vp, i32, vp]),
        "mg_refresh_rigid_body_state": (i32, [vp, vp, i32, vp]),
        "mg_refresh_dof_state": (i32, [vp, vp, i32, vp]),
        "mg_refresh_net_contact_force": (i32, [vp, vp, i32, vp]),
        "mg_set_actor_root_state": (i32, [vp, vp, i32, vp, i32, vp]),
        "mg_set_rigid_body_state": (i32, [vp, vp, i32, vp]),
        "mg_set_dof_state": (i32, [vp, vp, i32, vp, i32, vp]),
        "mg_set_dof_position_target": (i32, [vp, vp, i32, vp, i32, vp]),
        "mg_set_dof_velocity_target": (i32, [vp, vp, i32, vp, i32, vp]),
        "mg_set_dof_actuation_force": (i32, [vp, vp, i32, vp, i32, vp]),
        "mg_set_dof_props": (i32, [vp, vp]),
        "mg_apply_rigid_body_force": (i32, [vp, vp, vp, i32, i32, vp]),
        "mg_refresh_jacobian": (i32, [vp, i32, vp, i32, vp]),
        "mg_refresh_mass_matrix": (i32, [vp, i32, vp, i32, vp]),
        "mg_refresh_jacobian_mass_matrix": (i32, [vp, i32, vp, vp, i32, vp]),
        "mg_set_kernel_timing": (i32, [vp, i32]),
        "mg_set_fusion": (i32, [vp, i32]),
        "mg_bind_refresh_targets": (i32, [vp, vp, vp]),
        "mg_bind_dof_refresh_target": (i32, [vp, vp]),
        "mg_step_out_supported": (i32, [vp]),
        "mg_last_set_deferred": (i32, [vp]),
        "mg_discard_pending_sets": (i32, [vp]),
        "mg_last_step_ms": (ctypes.c_float, [vp]),
        "mg_step_time_stats": (i32, [vp, i32, vp, vp, vp]),
        "mg_num_free_bodies": (i32, [vp]),
        "mg_num_articulations": (i32, [vp]),
        "mg_num_coupled_envs": (i32, [vp]),
        "mg_num_pile_envs": (i32, [vp]),
        "mg_fetch_host_state": (i32, [vp, vp, i32, vp]),
        "mg_host_stage": (vp, [vp, ctypes.c_int64]),
        "mg_debug_copy_env_ctab": (i32, [vp, i32, vp, i32]),
        "mg_debug_artic_groups": (i32, [vp, vp, i32]),
        "mg_step_untimed_launches": (i32, [vp, i32]),
        "mg_env_ctab_floats": (i32, []),
        "mg_env_carry_floats": (i32, []),
        "mg_set_render_bodies": (i32, [vp, vp, vp, vp]),
        "mg_snapshot_render_state": (i32, [vp, vp]),
        "mg_render_cameras": (i32, [vp, vp, i32, vp]),
        "mg_set_light": (i32, [vp, vp]),
        "mg_last_render_ms": (ctypes.c_float, [vp]),
        "mg_cube_pick_step": (i32, [vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mg_abi_version() != 1:
        raise ImportError("libmigym.so ABI version mismatch")
    return lib


lib = _load()

EXPORTED_SYMBOLS = (
    "mg_abi_version", "mg_last_error", "mg_device_count", "mg_create_sim", "mg_destroy_sim",
    "mg_set_sim_params", "mg_upload_model", "mg_simulate", "mg_fetch_results",
    "mg_refresh_actor_root_state", "mg_refresh_rigid_body_state", "mg_refresh_dof_state",
    "mg_refresh_net_contact_force", "mg_set_actor_root_state", "mg_set_rigid_body_state",
    "mg_set_dof_state", "mg_set_dof_position_target", "mg_set_dof_velocity_target",
    "mg_set_dof_actuation_force", "mg_set_dof_props", "mg_apply_rigid_body_force",
    "mg_refresh_jacobian", "mg_refresh_mass_matrix", "mg_set_kernel_timing", "mg_set_fusion", "mg_bind_refresh_targets",
    "mg_bind_dof_refresh_target", "mg_step_out_supported", "mg_last_set_deferred", "mg_discard_pending_sets", "mg_last_step_ms", "mg_step_time_stats", "mg_num_free_bodies",
    "mg_num_articulations",
    "mg_num_coupled_envs", "mg_num_pile_envs", "mg_fetch_host_state", "mg_host_stage", "mg_refresh_jacobian_mass_matrix",
    "mg_set_render_bodies", "mg_snapshot_render_state", "mg_render_cameras", "mg_set_light", "mg_last_render_ms",
    "mg_debug_copy_env_ctab", "mg_debug_artic_groups", "mg_step_untimed_launches", "mg_cube_pick_step", "mg_env_ctab_floats", "mg_env_carry_floats",
)


class MigymError(RuntimeError):
    pass


def last_error():
    msg = lib.mg_last_error()
    return msg.decode() if msg else ""


def check(rc, what):
    if rc != MG_OK:
        raise MigymError("%s failed (%d): %s" % (what, rc, last_error()))


def device_count():
    return int(lib.mg_device_count())
