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
    assert lib.pipnet_amd_abi_version() == 3
    assert lib.pipnet_amd_status_string(1).decode().startswith("invalid argument")


def test_library_digest_matches_sources(tmp_path, monkeypatch):
    """Build provenance is a content digest compiled into the library, not a file mtime:
    the loaded library's digest equals the tree's, and a changed source is seen as stale
    whatever the mtimes say."""
    build.build()
    lib = _lib.load()
    assert lib.pipnet_amd_source_digest().decode() == build.source_digest()
    assert not build.is_stale()
    hdr = tmp_path / "extra.h"
    hdr.write_text("/* changed */\n")
    monkeypatch.setattr(build, "_deps", lambda orig=build._deps: orig() + [str(hdr)])
    assert build.is_stale()
    monkeypatch.setattr(_lib, "_lib", None)
    try:
        _lib.load()
        raise AssertionError("a library built from other sources loaded")
    except _lib.PipnetLibraryError as e:
        assert "other sources" in str(e)
    monkeypatch.setenv("PIPNET_AMD_ALLOW_STALE", "1")
    assert _lib.load() is not None


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


def _nm_demangled():
    import shutil
    import subprocess
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    return subprocess.run([nm, "-C", build.LIB], capture_output=True, text=True, check=True).stdout


def _kernel_symbols():
    return set(re.findall(r"void (pipnet_\w+::\w+<.*>)\(", _nm_demangled()))     # greedy: nested Cfg<...>


def test_roofline_kernel_names_exist_in_library():
    """bench.py labels each GEMM launch with kernels.gemm_kernel_name / bf16_conv_kernel_name
    (the rocprof name it must agree with): every label the ConvNeXt / ResNet / head shapes
    produce names a kernel instantiated in the library, NPAD tiles included."""
    from count_pipnet_amd import kernels as K
    build.build()
    syms = _kernel_symbols()
    assert any("gemm_f32_tn_kernel" in s for s in syms)
    shapes = [(200704, 384, 96, _lib.EPI_BIAS_GELU, 0), (200704, 96, 384, _lib.EPI_RESID, 0),
              (50176, 768, 192, _lib.EPI_BIAS_GELU, 0), (50176, 192, 768, _lib.EPI_RESID, 0),
              (46656, 1536, 384, _lib.EPI_BIAS_GELU, 0), (46656, 384, 1536, _lib.EPI_RESID, 0),
              (43264, 3072, 768, _lib.EPI_BIAS_GELU, 0), (43264, 768, 3072, _lib.EPI_RESID, 0),
              (50176, 192, 384, _lib.EPI_BIAS, 1), (46656, 384, 768, _lib.EPI_BIAS, 1),
              (43264, 768, 1536, _lib.EPI_BIAS, 1), (43264, 768, 768, _lib.EPI_NONE, 0),
              (1024, 16, 192, _lib.EPI_NONE, 0), (46656, 384, 1536, _lib.EPI_RESID_ROWSCALE, 0)]
    for m, n, k, epi, aload in shapes:
        name = K.gemm_kernel_name(m, n, k, epi, aload)
        assert name in syms, (m, n, k, epi, aload, name)
    # the plan is the library's own (pipnet_linear_f32_plan), no Python mirror of gemm_variant
    assert [K.gemm_variant(*s[:4], s[4]) for s in shapes[:8]] == [1, 2, 2, 2, 3, 5, 3, 3]
    assert K.gemm_variant(300, 256, 512) == 2 and K.gemm_variant(43264, 768, 1536, _lib.EPI_BIAS, 1) == 3
    # the wide 192 x 384 tile: from 100 tiles (C2's two-stream sub-batches), dense / 2x2 gather only
    assert K.gemm_variant(23328, 384, 1536, _lib.EPI_RESID) == 5 and K.gemm_variant(19199, 384, 1536) == 2
    assert K.gemm_variant(46656, 384, 768, _lib.EPI_BIAS, 1) == 5
    assert K.gemm_variant(46656, 384, 768, _lib.EPI_BIAS, 2) == 2
    assert K.gemm_variant(46656, 384, 1536, _lib.EPI_GELU_BWD) == 2
    assert "gemm_f32_tnw_kernel" in K.gemm_kernel_name(46656, 384, 768, _lib.EPI_BIAS, 1)
    # split-bf16 ConvNeXt GEMMs (stage-1/2 fc1 / fc2 incl. the N = 96 padded-column tile) and
    # ResNet bf16 convs
    out = _nm_demangled()
    for c, m in [(96, 200704), (96, 20000), (96, 9000), (96, 4096), (192, 50176), (192, 16384), (192, 5000),
                 (192, 1024)]:                                 # fused narrow-stage MLP (csrc/mlp_f32.hip)
        assert K.cnblock_mlp_kernel_name(c, m) in out, (c, m)
    assert K.cnblock_mlp_kernel_name(192, 16384, hw=256) in out          # hidden split (C5 stage 2)
    # the labels are the library's plan (pipnet_cnblock_mlp_plan), not a Python mirror
    assert K.cnblock_mlp_kernel_name(96, 200704) == "cnblock_mlp_kernel<96, 32, 4, 1, 1>"      # C2 stage 1
    assert K.cnblock_mlp_kernel_name(96, 65536) == "cnblock_mlp_kernel<96, 32, 8, 1, 1>"       # C5 stage 1
    assert K.cnblock_mlp_kernel_name(192, 25088) == "cnblock_mlp_kernel<192, 16, 8, 1, 1>"     # C2 stage 2 (half)
    assert K.cnblock_mlp_kernel_name(192, 16384, hw=256) == "cnblock_mlp_kernel<192, 16, 8, 1, 2>"
    assert K.cnblock_mlp_kernel_name(192, 16384) == "cnblock_mlp_kernel<192, 16, 4, 1, 1>"
    assert "pipnet_bf16::conv_bf16_ppp_kernel<12, 8>" in out                  # dual 1x1 (downsample + conv1)
    assert "pipnet_bf16::stem_pool_bf16_kernel" in out                     # fused stem + max-pool
    for m, n, epi in [(200704, 96, _lib.EPI_F32_RESID), (200704, 384, _lib.EPI_S3_GELU),
                      (50176, 192, _lib.EPI_F32_RESID)]:                      # split-bf16 GEMMs
        name = K.bf16_conv_kernel_name(m, n, epi, 0, K.s3_conv_tile(m, n, kv=3 * 4 * n), s3=True)
        assert name in syms, (m, n, epi, name)


# The C3 ResNet-50 bf16 layer list at 64 images of 224^2 (resnet_hip.py's launches):
# (name, H_in, Cin, Cout, k, stride, pad, epilogue, expected tile)
C3_LAYERS = [
    ("l1.c1", 56, 64, 64, 1, 1, 0, _lib.EPI_BIAS_RELU, 6), ("l1.c2", 56, 64, 64, 3, 1, 1, _lib.EPI_BIAS_RELU, 11),
    ("l1.c3", 56, 64, 256, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 4), ("l1.ds", 56, 64, 256, 1, 1, 0, _lib.EPI_BIAS, 4),
    ("l1.c1b", 56, 256, 64, 1, 1, 0, _lib.EPI_BIAS_RELU, 6),
    ("l2.c1", 56, 256, 128, 1, 1, 0, _lib.EPI_BIAS_RELU, 4), ("l2.c2s", 56, 128, 128, 3, 2, 1, _lib.EPI_BIAS_RELU, 4),
    ("l2.c2", 28, 128, 128, 3, 1, 1, _lib.EPI_BIAS_RELU, 11),
    ("l2.c3", 28, 128, 512, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 9), ("l2.ds", 56, 256, 512, 1, 2, 0, _lib.EPI_BIAS, 5),
    ("l3.c1", 28, 512, 256, 1, 1, 0, _lib.EPI_BIAS_RELU, 9), ("l3.c2", 28, 256, 256, 3, 1, 1, _lib.EPI_BIAS_RELU, 8),
    ("l3.c3", 28, 256, 1024, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 9),
    ("l4.c1", 28, 1024, 512, 1, 1, 0, _lib.EPI_BIAS_RELU, 9), ("l4.c2", 28, 512, 512, 3, 1, 1, _lib.EPI_BIAS_RELU, 8),
    ("l4.c3", 28, 512, 2048, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 9),
]


def test_bf16_labels_come_from_the_library_plan():
    """The roofline / profiling label of every C3 conv is the library's own tile choice
    (pipnet_conv2d_nhwc_bf16_plan, no Python mirror), and names a kernel instantiated in the library."""
    from count_pipnet_amd import kernels as K
    build.build()
    out = _nm_demangled()
    for name, h, cin, cout, k, s, pad, epi, want in C3_LAYERS:
        t = K.bf16_conv_plan(64, h, h, cin, cout, k, k, s, pad, epi)
        assert t == want, (name, t, want)
        oh = (h + 2 * pad - k) // s + 1
        label = K.bf16_conv_kernel_name(64 * oh * oh, cout, epi, 0 if k == 1 and s == 1 else 2, t, kv=k * k * cin)
        assert label in out, (name, label)
    # a requested tile is validated, not chosen: tile 8 needs a 3x3 stride-1 halo shape
    import pytest
    with pytest.raises(RuntimeError):
        K.bf16_conv_plan(64, 56, 56, 256, 512, 1, 1, 2, 0, _lib.EPI_BIAS, 8)
