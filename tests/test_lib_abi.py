"""CPU checks of the C ABI boundary: libdvie.so loads (against torch's HIP runtime),
exports every entry point include/dvie.h declares, and the ctypes mirrors of the
descriptor structs have the C sizes.  No compute is launched (no GPU here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "dvie.h")


def declared():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(dvie_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    names = declared()
    for n in ("dvie_conv2d_fwd", "dvie_conv2d_wgrad", "dvie_ew", "dvie_loss", "dvie_warp_fwd", "dvie_adamax",
              "dvie_run_ops"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from deep_video_interpolation_extrapolation_amd import _lib
    _lib.load()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (dvie_[a-z0-9_]+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    assert set(_lib.EXPORTS) <= exported


def test_abi_struct_sizes_match():
    from deep_video_interpolation_extrapolation_amd import _lib
    lib = _lib.load()  # raises on any mismatch
    assert lib.dvie_version().startswith(b"dvie")


def test_single_hip_runtime_in_process():
    from deep_video_interpolation_extrapolation_amd import _lib
    _lib.load()
    maps = [l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l]
    assert len(set(maps)) == 1, set(maps)


def test_argument_validation_without_gpu():
    """Invalid descriptors are rejected before any launch (status DVIE_EINVAL)."""
    import ctypes
    from deep_video_interpolation_extrapolation_amd import _lib as L
    lib = L.load()
    d = L.ConvDesc()
    d.x, d.w, d.y = 16, 16, 16
    d.dtype = L.BF16
    d.c, d.cout = 12, 8  # 12 is not a multiple of 8 bf16 lanes
    assert lib.dvie_conv2d_fwd(ctypes.byref(d), None) == L.DVIE_EINVAL
    assert b"multiple of 8" in lib.dvie_last_error()


def test_warp_workspace_query_without_gpu():
    """dvie_warp_ws_floats: no workspace for the dflow-only backward; otherwise the taps
    (2 floats per pixel) and the far bytes (one per pixel, 16-byte aligned)."""
    import ctypes
    from deep_video_interpolation_extrapolation_amd import _lib as L
    lib = L.load()
    d = L.WarpDesc()
    d.n, d.c, d.h, d.w = 2, 3, 5, 7
    assert lib.dvie_warp_ws_floats(ctypes.byref(d)) == 0
    d.dimg = 16
    px = 2 * 5 * 7
    assert lib.dvie_warp_ws_floats(ctypes.byref(d)) == (2 * px + 3) // 4 * 4 + (px + 15) // 16 * 4
