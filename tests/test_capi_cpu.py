"""CPU: libxerus_amd.so builds for gfx950, loads, and exports every symbol include/xerus_amd.h declares."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "xerus_amd.h")).read()
    return sorted(set(re.findall(r"\b(xrs_[a-z0-9_]+)\s*\(", hdr)))


def test_header_and_binding_agree():
    from xerus_amd import capi

    assert sorted(capi.SIGNATURES) == _declared()


def test_library_exports_every_symbol():
    from xerus_amd import capi

    lib = capi.load()
    out = subprocess.run(["nm", "-D", "--defined-only", capi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (xrs_[a-z0-9_]+)", out))
    missing = [s for s in _declared() if s not in exported]
    assert not missing, missing
    assert lib.xrs_version().decode().startswith("xerus_amd")


def test_code_object_targets_gfx950():
    from xerus_amd import capi

    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", capi.LIB_PATH], capture_output=True, text=True)
    blob = open(capi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_errors_without_gpu_are_loud():
    """No compute call without a GPU: creating a handle must fail with a status, never fall back."""
    from xerus_amd import capi

    import ctypes

    lib = capi.load()
    h = ctypes.c_void_p()
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        has_gpu = hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        has_gpu = False
    if has_gpu:
        return
    st = lib.xrs_create(ctypes.byref(h), 0)
    assert st != 0
    assert lib.xrs_last_error()
