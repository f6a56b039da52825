"""C-ABI boundary checks that need no GPU: the library loads, exports every function
include/shipsim.h declares, its #defines agree with the Python binding, and the host-side
default config equals the scenario of record restated in shipsim_abi.py."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from ast_sac_amd import shipsim_abi as abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "shipsim.h")


@pytest.fixture(scope="module")
def lib():
    from ast_sac_amd import shipsim
    if not os.path.exists(shipsim.LIB_PATH):
        import __graft_entry__ as ge
        ge.build_hip()
    return shipsim.load_library()


def _header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(shipsim_\w+)\s*\(", src, re.M)))


def _header_defines():
    out = {}
    for name, val in re.findall(r"#define\s+SHIPSIM_(\w+)\s+(\(?-?[0-9xu <()]+\)?)", open(HEADER).read()):
        v = val.replace("u", "").strip()
        try:
            out[name] = int(eval(v))  # noqa: S307  (literal integer expressions from our own header)
        except Exception:  # noqa: BLE001
            pass
    return out


def test_library_exports_every_declared_function(lib):
    from ast_sac_amd.shipsim import EXPORTED_SYMBOLS
    declared = _header_functions()
    assert len(declared) >= 13
    assert set(declared) == set(EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.shipsim_abi_version() == abi.ABI_VERSION
    info = lib.shipsim_build_info().decode()
    assert "gfx950" in info


def test_header_constants_match_binding():
    d = _header_defines()
    pairs = {"ABI_VERSION": abi.ABI_VERSION, "MAX_ROUTE": abi.MAX_ROUTE, "MAX_POLYS": abi.MAX_POLYS,
             "MAX_VERTS": abi.MAX_VERTS, "KIND_SINGLE": abi.KIND_SINGLE, "KIND_AST": abi.KIND_AST,
             "COLLAV_NONE": abi.COLLAV_NONE, "COLLAV_SIMPLE": abi.COLLAV_SIMPLE, "COLLAV_SBMPC": abi.COLLAV_SBMPC,
             "MACH_SIMPLIFIED": abi.MACH_SIMPLIFIED, "MACH_DETAILED": abi.MACH_DETAILED,
             "EV_COLLISION": abi.EV_COLLISION, "EV_SAMPLING_FAILURE": abi.EV_SAMPLING_FAILURE,
             "EV_TERMINAL": abi.EV_TERMINAL, "EV_TEST_STOP": abi.EV_TEST_STOP, "EV_OBS_STOP": abi.EV_OBS_STOP,
             "F_NEXT_WPT": abi.F_NEXT_WPT, "F_STOP": abi.F_STOP, "N_SHIP_FIELDS": abi.N_SHIP_FIELDS,
             "E_SAMPLING_COUNT": abi.E_SAMPLING_COUNT, "E_ROUTE_EAST": abi.E_ROUTE_EAST}
    for name in dir(abi):  # trajectory record layout and SBMPC batch layout, every column
        if name.startswith(("TS_", "TE_", "TRAJ_", "SBMPC_IN", "LT_", "DL_", "DECLOG_")) and name != "LT_DONE_MASK":
            pairs[name] = getattr(abi, name)
    assert "TS_TIME_LIST" in pairs and "TE_FLAG_IMMINENT" in pairs and "LT_OBS_NAV_FAILURE" in pairs
    for k, v in pairs.items():
        assert d[k] == v, k
    assert C.sizeof(abi.Config) > 0


@pytest.mark.parametrize("collav", ["none", "simple", "sbmpc"])
@pytest.mark.parametrize("mach", [abi.MACH_DETAILED, abi.MACH_SIMPLIFIED])
def test_default_config_equals_binding_restatement(lib, collav, mach):
    cfg = abi.Config()
    rc = lib.shipsim_default_config(abi.KIND_AST, mach, abi.COLLAV[collav], 4.0, C.byref(cfg))
    assert rc == 0
    ref = abi.ast_config(collav, time_step=4, machinery=mach)
    for name, _ in abi.Config._fields_:
        if name in ("ship", "lanes_per_env", "reserved"):
            continue
        a, b = getattr(cfg, name), getattr(ref, name)
        if hasattr(a, "__len__"):
            np.testing.assert_array_equal(np.array(a[:]), np.array(b[:]), err_msg=name)
        else:
            assert a == b, name
    for s in range(2):
        for name, _ in abi.ShipConfig._fields_:
            a, b = getattr(cfg.ship[s], name), getattr(ref.ship[s], name)
            if hasattr(a, "__len__"):
                np.testing.assert_array_equal(np.array(a[:]), np.array(b[:]), err_msg=f"ship{s}.{name}")
            else:
                assert a == b or (np.isinf(a) and np.isinf(b)), f"ship{s}.{name}"


def test_create_rejects_bad_config_without_touching_a_device(lib):
    cfg = abi.ast_config("none")
    cfg.abi_version = 99
    h = C.c_void_p()
    rc = lib.shipsim_create(C.byref(cfg), 4, 0, 0, None, C.byref(h))
    assert rc == -1  # SHIPSIM_EINVAL
    assert b"abi_version" in lib.shipsim_last_error(None)
    cfg = abi.ast_config("none")
    rc = lib.shipsim_create(C.byref(cfg), 0, 0, 0, None, C.byref(h))
    assert rc == -1


@pytest.mark.parametrize("k,collav,mach,msg", [(5, "none", abi.MACH_DETAILED, b"obstacle ships"),
                                               (2, "simple", abi.MACH_DETAILED, b"collav none / sbmpc"),
                                               (4, "sbmpc", abi.MACH_SIMPLIFIED, b"detailed machinery")])
def test_create_rejects_unsupported_obstacle_counts(lib, k, collav, mach, msg):
    """C5 K obstacle ships: 1..SHIPSIM_MAX_OBS, K > 1 with detailed machinery and collav none / sbmpc."""
    cfg = abi.ast_config(collav, machinery=mach)
    h = C.c_void_p()
    rc = lib.shipsim_create(C.byref(cfg), 4, k, 0, None, C.byref(h))
    assert rc == -1 and not h.value
    assert msg in lib.shipsim_last_error(None)
