"""The C-ABI library loads and exports every function include/rsamd.h declares (CPU only:
no compute call needs a GPU here)."""
import ctypes
import re

import pytest

from tsbb15_amd import _ffi


def _declared_functions():
    src = open(_ffi.HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rs_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_expected_surface():
    names = _declared_functions()
    for must in ("rs_fmatrix_stls", "rs_fmatrix_residuals", "rs_f8_plan_run", "rs_f8_ransac_np",
                 "rs_np_choice_tuples", "rs_py_shuffle_tuples", "rs_pnp_dlt", "rs_pnp_ransac",
                 "rs_comm_allgather"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_ffi.LIB_PATH)
    missing = [n for n in _declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_every_declared_symbol():
    assert set(_declared_functions()) <= set(_ffi._SIGS), \
        set(_declared_functions()) - set(_ffi._SIGS)


def test_struct_layouts():
    assert ctypes.sizeof(_ffi.F8Result) == 9 * 8 + 2 * 8 + 2 * 8 + 3 * 8
    assert ctypes.sizeof(_ffi.F8Candidate) == 4 * 8 + 9 * 8
    assert ctypes.sizeof(_ffi.PnpResult) == 12 * 8 + 2 * 8
    assert ctypes.sizeof(_ffi.GsInfo) == 2 * 8 + 4 * 4


def test_version_and_errors_without_gpu():
    lib = _ffi.lib()
    assert lib.rs_version() >= 100
    n = ctypes.c_int(-1)
    assert lib.rs_device_count(ctypes.byref(n)) == 0
    if n.value == 0:
        with pytest.raises(RuntimeError, match="no HIP device"):
            _ffi.Context(0)
