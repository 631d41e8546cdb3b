"""TEST INFRASTRUCTURE ONLY — the CPU restatement of the engine step
(oracle/migym_oracle.c) as a parity checker. Imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product
package test_isaacgym_amd. Physics parity with PhysX is UNPINNED (the
reference engine is a closed binary absent from the reference tree); see the
header of migym_oracle.c and DESIGN.md §4.
"""
import ctypes
import os
import subprocess
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    lib.oracle_step.restype = ctypes.c_int
    lib.oracle_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int]
    lib.oracle_step_mt.restype = ctypes.c_int
    lib.oracle_step_mt.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


# Friction patches are simulation state kept from
# step to step, as the device keeps them: per env, the coupled step's pairs —
# FC_N = 128 pairs x (16 + 1) floats (migym_oracle_env.c OE_FC_N) — and per
# body, a free body's ground patch — BC_N = 16 floats (migym_oracle.c OR_GP_N).
FC_N = 128 * (16 + 1)
BC_N = 16
_caches = {}


class ContactCache:
    """The friction patches of one simulation (zeros: no patch yet)."""

    def __init__(self, model):
        self.env = np.zeros((max(int(model.num_envs), 1), FC_N), dtype=np.float32)
        self.body = np.zeros((max(int(model.num_bodies), 1), BC_N), dtype=np.float32)

    def fits(self, model):
        return self.env.shape[0] >= int(model.num_envs) and self.body.shape[0] >= int(model.num_bodies)


def contact_cache(model):
    """A fresh (no patch yet) friction-patch cache for `model`."""
    return ContactCache(model)


def _cache_for(state, model):
    """The cache that goes with a state array: the one a caller stepping the
    same `state` in place used on the previous step (the device keeps its
    patches inside the sim the same way)."""
    key = id(state)
    ent = _caches.get(key)
    if ent is not None and ent[0]() is state and ent[1].fits(model):
        return ent[1]
    c = contact_cache(model)
    _caches[key] = (weakref.ref(state, lambda _r, k=key: _caches.pop(k, None)), c)
    return c


def step(sim_params, model, state, dof, tgt=None, props=None, ext=None, cforce=None, body_range=None,
         contact_cache=None):
    """One gym.simulate() on the host, in place.

    sim_params: _native.MgSimParams; model: _native.MgModel (its arrays alive);
    state [nb,13] f32, dof [nd,2] f32 (updated in place); tgt [nd,3]; props [nd,12];
    ext [nb,6]; cforce [nb,3] (written); contact_cache: the friction patches
    (default: the ones kept with this `state` array). Returns cforce.
    """
    nb = state.shape[0]
    nd = dof.shape[0]
    assert state.dtype == np.float32 and state.flags.c_contiguous and state.shape[1] == 13
    assert dof.dtype == np.float32 and dof.flags.c_contiguous
    if tgt is None:
        tgt = np.zeros((max(nd, 1), 3), dtype=np.float32)
    if cforce is None:
        cforce = np.zeros((nb, 3), dtype=np.float32)
    b0, b1 = body_range if body_range is not None else (0, -1)
    # converted copies bound to locals so they outlive the call
    tgt_c = np.ascontiguousarray(tgt, dtype=np.float32)
    props_c = None if props is None else np.ascontiguousarray(props, dtype=np.float32)
    ext_c = None if ext is None else np.ascontiguousarray(ext, dtype=np.float32)
    assert cforce.dtype == np.float32 and cforce.flags.c_contiguous and cforce.shape == (nb, 3)
    fc = _cache_for(state, model) if contact_cache is None else contact_cache
    assert fc.fits(model)
    rc = lib().oracle_step(ctypes.addressof(sim_params), ctypes.addressof(model), _ptr(state), _ptr(dof),
                           _ptr(tgt_c), _ptr(props_c), _ptr(ext_c), _ptr(cforce), _ptr(fc.env), _ptr(fc.body),
                           int(b0), int(b1))
    if rc != 0:
        raise RuntimeError("oracle_step: unsupported model")
    return cforce


def step_threads(sim_params, model, state, dof, nthreads, tgt=None, props=None, ext=None, cforce=None,
                 contact_cache=None):
    """step() on `nthreads` host threads (oracle_step_mt, OpenMP): the same
    result; the CPU baseline of bench.py."""
    nb, nd = state.shape[0], dof.shape[0]
    assert state.dtype == np.float32 and state.flags.c_contiguous and state.shape[1] == 13
    assert dof.dtype == np.float32 and dof.flags.c_contiguous
    if tgt is None:
        tgt = np.zeros((max(nd, 1), 3), dtype=np.float32)
    if cforce is None:
        cforce = np.zeros((nb, 3), dtype=np.float32)
    tgt_c = np.ascontiguousarray(tgt, dtype=np.float32)
    props_c = None if props is None else np.ascontiguousarray(props, dtype=np.float32)
    ext_c = None if ext is None else np.ascontiguousarray(ext, dtype=np.float32)
    fc = _cache_for(state, model) if contact_cache is None else contact_cache
    assert fc.fits(model)
    rc = lib().oracle_step_mt(ctypes.addressof(sim_params), ctypes.addressof(model), _ptr(state), _ptr(dof),
                              _ptr(tgt_c), _ptr(props_c), _ptr(ext_c), _ptr(cforce), _ptr(fc.env), _ptr(fc.body),
                              int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle_step_mt: unsupported model")
    return cforce


def collide(a, b, margin, hull_a=None, hull_b=None):
    """Narrow phase of the coupled step (oracle_collide2): a, b = [type, c.xyz,
    q.xyzw, h.xyz] (convex: h = (bounding radius, 0, 0) and its hull record
    hull_a / hull_b); returns an (n, 7) array of [point on a, normal b->a, sep]."""
    L = lib()
    vp = ctypes.c_void_p
    L.oracle_collide2.restype = ctypes.c_int
    L.oracle_collide2.argtypes = [vp, vp, vp, vp, ctypes.c_float, vp]
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    ha = None if hull_a is None else np.ascontiguousarray(hull_a, dtype=np.float32)
    hb = None if hull_b is None else np.ascontiguousarray(hull_b, dtype=np.float32)
    out = np.zeros((4, 7), dtype=np.float32)
    n = L.oracle_collide2(a.ctypes.data, _ptr(ha), b.ctypes.data, _ptr(hb), float(margin), out.ctypes.data)
    return out[:n]


def obb_apart(a, b, margin, hull_a=None, hull_b=None):
    """The coupled step's OBB pair screen (oracle_obb_apart = mg_env.hip
    obb_apart) on two shapes in collide()'s format: True when it rejects them."""
    L = lib()
    vp = ctypes.c_void_p
    L.oracle_obb_apart.restype = ctypes.c_int
    L.oracle_obb_apart.argtypes = [vp, vp, vp, vp, ctypes.c_float]
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    ha = None if hull_a is None else np.ascontiguousarray(hull_a, dtype=np.float32)
    hb = None if hull_b is None else np.ascontiguousarray(hull_b, dtype=np.float32)
    return bool(L.oracle_obb_apart(a.ctypes.data, _ptr(ha), b.ctypes.data, _ptr(hb), float(margin)))


def render(sim_params, state, body_tmpl, tbi, shapes, env_body_first, color, seg, cam, hulls=None, light=None):
    """One camera on the host (oracle_render, migym_oracle_render.c): returns
    (rgba (H, W, 4) uint8, depth (H, W) f32, seg (H, W) int32). state is the
    rigid-body tensor [nb, 13] (global order); cam a _native.MgCamera (its
    device pointers are ignored); light an _native.MgLight (mg_set_light) or
    None for the default light."""
    L = lib()
    vp = ctypes.c_void_p
    L.oracle_render.restype = ctypes.c_int
    L.oracle_render.argtypes = [vp] * 14
    H, W = cam.height, cam.width
    rgba = np.zeros((H, W, 4), np.uint8)
    depth = np.zeros((H, W), np.float32)
    sg = np.zeros((H, W), np.int32)
    arrs = [np.ascontiguousarray(state, np.float32), np.ascontiguousarray(body_tmpl, np.int32),
            np.ascontiguousarray(tbi, np.int32), np.ascontiguousarray(shapes, np.float32),
            np.ascontiguousarray(env_body_first, np.int32), np.ascontiguousarray(color, np.float32),
            np.ascontiguousarray(seg, np.int32)]
    hl = np.ascontiguousarray(hulls if hulls is not None and len(hulls) else np.zeros(1), np.float32)
    ptrs = [a.ctypes.data for a in arrs]
    rc = L.oracle_render(ctypes.addressof(sim_params), ptrs[0], ptrs[1], ptrs[2], ptrs[3], hl.ctypes.data, ptrs[4],
                         ptrs[5], ptrs[6], ctypes.addressof(cam), rgba.ctypes.data, depth.ctypes.data, sg.ctypes.data,
                         ctypes.addressof(light) if light is not None else None)
    if rc != 0:
        raise RuntimeError("oracle_render: too many shapes in the camera's env")
    return rgba, depth, sg
