"""The C-ABI library builds for gfx950, loads without a GPU, and exports every entry point
that include/pipnet_amd.h declares (no compute calls here: no GPU in this container)."""
import ctypes
import os
import re

from count_pipnet_amd import _lib, build

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "pipnet_amd.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(pipnet_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "pipnet_linear_f32" in syms and "pipnet_count_gumbel_f32" in syms
    assert set(syms) == set(_lib.SIGNATURES), "ctypes binding and header disagree"


def test_library_loads_and_exports_all_symbols():
    build.build()
    lib = _lib.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert lib.pipnet_amd_abi_version() == 1
    assert lib.pipnet_amd_status_string(1).decode().startswith("invalid argument")


def test_argument_validation_without_gpu():
    """Bad shapes are rejected before any HIP call (status PIPNET_ERR_ARG, no launch)."""
    lib = _lib.load()
    # K not a multiple of 4
    assert lib.pipnet_linear_f32(None, 3, None, None, None, None, 0, None, 8, 8, 8, 3, 0, None) == 1
    # unsupported dwconv channel count (B=0 would return OK; use B=1 with bad C and NULL ptrs)
    assert lib.pipnet_dwconv7_ln_f32(None, 1, 7, 7, 100, None, None, None, None, None, None) == 1
    # empty batch is a no-op
    assert lib.pipnet_conv2x2_f32(ctypes.c_void_p(16), 0, 4, 4, 32, ctypes.c_void_p(16), None, 8, 2,
                                  ctypes.c_void_p(16), None) == 0
    # stride 3 is not a ConvNeXt downsample
    assert lib.pipnet_conv2x2_f32(ctypes.c_void_p(16), 1, 4, 4, 32, ctypes.c_void_p(16), None, 8, 3,
                                  ctypes.c_void_p(16), None) == 1
