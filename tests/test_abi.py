"""The C-ABI library loads (no GPU needed) and exports every symbol the header declares."""
import ctypes
import os
import re

import pytest

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


def test_m0_consumers_checked_on_device_code():
    """the slot build leaves its M0 behind; no other M0 consumer of the subband
    kernels may read it (scripts/check_m0.py on the assembly the production compile keeps)."""
    import subprocess
    import sys
    asm = os.path.join(REPO, "radio-pulsar-utils_amd", "csrc", "dedisperse-hip-amdgcn-amd-amdhsa-gfx950.s")
    if not os.path.exists(asm):
        pytest.skip("device assembly not built here (make -C radio-pulsar-utils_amd/csrc)")
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "check_m0.py"), asm],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 reading" in r.stdout, r.stdout


def test_every_launch_stub_has_a_device_image():
    """A host object with a stale embedded code object links but aborts at launch ("Cannot
    find Symbol"): every launch stub in the shipped library has its kernel descriptor."""
    import subprocess
    import sys
    lib = os.path.join(REPO, "radio-pulsar-utils_amd", "pulsarutils", "_lib", "libpulsarutils_hip.so")
    if not os.path.exists(lib):
        pytest.skip("library not built here")
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "check_stubs.py"), lib],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 without a device image" in r.stdout, r.stdout


def test_plan_opts_validated_without_gpu():
    """pu_plan_create_ex checks its options before any HIP call."""
    from pulsarutils import _hip
    h = ctypes.c_void_p()
    sh = (ctypes.c_int64 * 4)()
    bad = _hip.PlanOpts(group=0, shape=5, lds_budget_kb=0, u8_dma=-1, dt_major=-1)
    rc = _hip.lib().pu_plan_create_ex(ctypes.byref(h), _hip.PU_F32, 0, 4, 16, ctypes.cast(sh, ctypes.c_void_p), 1,
                                      ctypes.byref(bad))
    assert rc == -1 and "shape" in _hip.lib().pu_last_error().decode()


def test_production_library_reads_no_tuning_environment():
    """the tuning knobs (PU_GROUP, PU_SUB_SHAPE, ...) exist only in the
    diagnostic build; the production library does not even contain their names, so a
    stray variable in a user's environment cannot change a kernel."""
    from pulsarutils import _hip
    blob = open(_hip._LIB_PATH, "rb").read()
    for knob in (b"PU_SUB_SHAPE", b"PU_GROUP", b"PU_LDS_BUDGET_KB", b"PU_U8_DMA", b"PU_DT_MAJOR", b"PU_CLEAN_BATCH",
                 b"PU_APPLY_BATCH", b"PU_MEDIAN_GRID", b"PU_COLSEG", b"PU_SUB_SKIP", b"PU_DMA_WAVES"):
        assert knob not in blob, knob


def test_one_hip_runtime_when_the_library_loads_first():
    """A process whose first pulsarutils call is host-only (shift_table) must still hold ONE
    HIP and HSA runtime: lib() imports torch before dlopen, so the library's
    libamdhip64.so.7 resolves to the copy PyTorch bundles (two runtimes made the library's
    hipMalloc fail with "no ROCm-capable device" on the MI355X box)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from pulsarutils import _hip\n"
            "_hip.shift_table(8, [1.0], 1400.0, 100.0, 1e-4)\n"
            "import torch\n"
            "maps = open('/proc/self/maps').read().splitlines()\n"
            "libs = {l.split()[-1] for l in maps if 'libamdhip64' in l or 'libhsa-runtime64' in l}\n"
            "print(len(libs))\n") % os.path.join(REPO, "radio-pulsar-utils_amd")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "2", out.stdout  # one libamdhip64 + one libhsa-runtime64
