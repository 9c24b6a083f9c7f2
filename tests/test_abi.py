"""The C-ABI library builds for gfx950, loads, and exports every symbol include/gpx.h declares
(no compute calls here: this container has no GPU)."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

from portfoliooptgp_amd import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "gpx.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gpx_[a-z_]+)\s*\(", src)))


def test_header_declarations_match_binding():
    assert declared_functions() == sorted(N.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = N.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (gpx_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", N.LIB_PATH], capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_struct_layouts_match_header():
    assert ctypes.sizeof(N.GpxTerm) == 16
    assert ctypes.sizeof(N.GpxKernelSpec) == 16 + 16 * N.GPX_MAX_TERMS
    hdr = open(HEADER).read()
    assert f"#define GPX_THETA_STRIDE {N.GPX_THETA_STRIDE}" in hdr
    assert f"#define GPX_MAX_TERMS {N.GPX_MAX_TERMS}" in hdr
    for name, val in [("GPX_SE", 1), ("GPX_LINEAR", 8), ("GPX_RQ", 6), ("GPX_PERIODIC_SE", 7)]:
        assert re.search(rf"{name}\s*=\s*{val}\b", hdr)
        assert getattr(N, name) == val


def test_version_string():
    assert N.load_library().gpx_version().startswith(b"gpx ")


def test_no_device_fails_cleanly_without_compute():
    """gpx_create must return an error code (not crash) when no HIP device is visible."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from portfoliooptgp_amd import _native as N\nimport ctypes\n"
            "lib = N.load_library(); h = ctypes.c_void_p()\n"
            "print(lib.gpx_create(0, ctypes.byref(h)))\n") % REPO
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    if r.returncode != 0:
        pytest.skip(f"HIP runtime unavailable in this container: {r.stderr[-200:]}")
    assert r.stdout.strip().splitlines()[-1] in {str(N.GPX_HIP_ERROR), str(N.GPX_BAD_ARG)}
