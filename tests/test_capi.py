"""The C-ABI library loads and exports every entry point include/migym.h
declares; on a host without a GPU it refuses to create a sim (no CPU engine)."""
import ctypes
import os
import re

from conftest import ROOT, has_gpu


def _header_functions():
    src = open(os.path.join(ROOT, "include", "migym.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mg_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported():
    from test_isaacgym_amd import _native as N
    names = _header_functions()
    assert len(names) >= 25
    lib = ctypes.CDLL(N.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(N.EXPORTED_SYMBOLS)


def test_abi_version_and_errors():
    from test_isaacgym_amd import _native as N
    assert N.lib.mg_abi_version() == 1
    # null handles are rejected with a message, never dereferenced
    assert N.lib.mg_simulate(None, None) < 0
    assert "upload" in N.last_error() or "sim" in N.last_error()
    assert N.lib.mg_refresh_actor_root_state(None, None, 0, None) < 0


def test_no_gpu_means_no_sim():
    from test_isaacgym_amd import _native as N
    if has_gpu():
        return
    params = N.MgSimParams()
    assert not N.lib.mg_create_sim(0, ctypes.byref(params))
    assert "HIP device" in N.last_error()
