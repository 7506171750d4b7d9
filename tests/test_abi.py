"""The C-ABI library loads (no GPU needed) and exports every symbol the header declares."""
import ctypes
import os
import re

from conftest import REPO


def header_functions():
    src = open(os.path.join(REPO, "include", "pulsarutils_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(pu_[a-z0-9_]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = header_functions()
    for must in ("pu_plan_create", "pu_plan_search", "pu_plan_dedisperse", "pu_row_sums", "pu_renorm_apply",
                 "pu_shift_table", "pu_last_error", "pu_rebin_time", "pu_roll_rows"):
        assert must in names


def test_library_exports_all_header_symbols():
    from pulsarutils import _hip
    lib = _hip.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
        assert name in _hip.SIGNATURES, f"{name} not bound in _hip.SIGNATURES"
    assert lib.pu_version().decode().startswith("pulsarutils-hip")


def test_error_path_without_gpu():
    """Argument validation happens before any HIP call: usable on CPU."""
    from pulsarutils import _hip
    h = ctypes.c_void_p()
    rc = _hip.lib().pu_plan_create(ctypes.byref(h), 7, 0, 4, 16, None, 1)
    assert rc == -1
    assert "unsupported dtype" in _hip.lib().pu_last_error().decode()
