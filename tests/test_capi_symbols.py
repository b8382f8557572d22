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
    # split-bf16 ConvNeXt GEMMs (stage-1/2 fc1 / fc2 incl. the N = 96 padded-column tile) and
    # ResNet bf16 convs
    out = _nm_demangled()
    for c, m in [(96, 200704), (96, 20000), (96, 9000), (96, 4096), (192, 50176), (192, 16384), (192, 5000),
                 (192, 1024)]:                                 # fused narrow-stage MLP (csrc/mlp_f32.hip)
        assert K.cnblock_mlp_kernel_name(c, m) in out, (c, m)
    assert K.cnblock_mlp_kernel_name(192, 16384, hw=256) in out          # hidden split (C5 stage 2)
    assert "pipnet_bf16::conv_bf16_ppp_kernel<12, 8>" in out                  # dual 1x1 (downsample + conv1)
    assert "pipnet_bf16::stem_pool_bf16_kernel" in out                     # fused stem + max-pool
    for m, c in ((401408, 64), (100352, 128)):                               # small-N halo tile (11)
        assert K.bf16_conv_kernel_name(m, c, _lib.EPI_BIAS_RELU, 2, kv=9 * c, halo64_ok=True) in out
    for m, n, epi, s3 in [(200704, 96, _lib.EPI_F32_RESID, True), (200704, 384, _lib.EPI_S3_GELU, True),
                          (50176, 192, _lib.EPI_F32_RESID, True), (401408, 64, _lib.EPI_BIAS_RELU, False),
                          (100352, 128, _lib.EPI_BIAS_RELU, False)]:
        name = K.bf16_conv_kernel_name(m, n, epi, 0, s3=s3)
        assert name in syms, (m, n, epi, s3, name)
