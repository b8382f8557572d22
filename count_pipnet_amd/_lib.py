"""ctypes binding of the C-ABI in ``include/pipnet_amd.h`` (``libpipnet_amd.so``).

This is exactly the binding a maintainer would add to the reference:
the library takes raw device pointers, sizes and a hipStream_t, and returns a status
code that is raised here as ``RuntimeError`` (the reference raises Python exceptions,
SURVEY.md 8b).  There is no fallback: if the library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PIPNET_AMD_LIB") or os.path.join(_HERE, "libpipnet_amd.so")    # env: A/B builds (tools)

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
F32 = ctypes.c_float
F64 = ctypes.c_double

# name -> argtypes (restype is int status unless listed in _RESTYPE)
SIGNATURES = {
    "pipnet_amd_abi_version": [],
    "pipnet_amd_status_string": [I32],
    "pipnet_amd_source_digest": [],
    "pipnet_linear_f32": [P, I64, P, P, P, P, I64, P, I64, I32, I32, I32, I32, P],
    "pipnet_linear_rowscale_f32": [P, I64, P, P, P, P, I64, P, I64, I32, I32, I32, P, I32, P],
    "pipnet_linear_splitk_f32": [P, I64, P, P, P, P, I64, P, I64, I32, I32, I32, I32, I32, P, P],
    "pipnet_linear_pair_mul_f32": [P, I64, P, P, I64, I32, I32, I32, I32, P, P],
    "pipnet_matmul_f64acc_f32": [P, I64, P, I64, P, I64, I32, I32, I32, P],
    "pipnet_matmul2_f64acc_f32": [P, P, I64, P, I64, P, P, I64, I32, I32, I32, P],
    "pipnet_conv2x2_f32": [P, I32, I32, I32, I32, P, P, I32, I32, P, P],
    "pipnet_convnext_stem_f32": [P, I32, I32, I32, P, P, P, P, P, P],
    "pipnet_conv2d_nhwc_f32": [P, I32, I32, I32, I32, P, P, I32, I32, I32, I32, I32, P, I32, P, P],
    "pipnet_maxpool2d_nhwc_f32": [P, I32, I32, I32, I32, I32, I32, I32, P, P],
    "pipnet_nchw_to_nhwc_f32": [P, I32, I32, I32, I32, I32, P, P],
    "pipnet_conv2d_nhwc_bf16": [P, I32, I32, I32, I32, P, P, I32, I32, I32, I32, I32, P, I32, P, P],
    "pipnet_conv2d_nhwc_bf16_tile": [P, I32, I32, I32, I32, P, P, I32, I32, I32, I32, I32, P, I32, P, I32, P],
    "pipnet_conv2d_nhwc_bf16_plan": [I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32],
    "pipnet_linear_f32_plan": [I32, I32, I32, I32, I32],
    "pipnet_cnblock_mlp_plan": [I64, I32, I32],
    "pipnet_count_gumbel_soft_f32": [P, I32, I32, I32, F32, P, U64, U64, P, P, P],
    "pipnet_philox_exp1_f32": [U64, U64, I64, I32, P, P],
    "pipnet_nonneg_linear_dx_f32": [P, P, I32, I32, I32, P, P],
    "pipnet_bilinear_bwd_prep_f32": [P, P, P, I64, P, P, P],
    "pipnet_linear_inter_partials_floats": [I32],
    "pipnet_linear_inter_bwd_f32": [P, I64, I32, P, P, P, P, I32, P, P],
    "pipnet_count_ste_bwd_f32": [P, I64, I32, I32, I32, P, P, P],
    "pipnet_onehot_ste_bwd_f32": [P, I64, I32, P, I32, I32, P, P, P],
    "pipnet_count_head_bwd_f32": [P, P, I32, I32, I32, P, F32, F32, F32, F32, P, P, P],
    "pipnet_conv2d_nhwc_s3": [P, I32, I32, I32, I32, P, P, P, P, I32, I32, I32, I32, I32, I32, P, I32, P],
    "pipnet_dwconv7_ln_s3": [P, I32, I32, I32, I32, P, P, P, P, P, P],
    "pipnet_layernorm_s3": [P, I64, I32, P, P, P, P],
    "pipnet_maxpool2d_nhwc_bf16": [P, I32, I32, I32, I32, I32, I32, I32, P, P],
    "pipnet_nchw_to_nhwc_bf16": [P, I32, I32, I32, I32, I32, P, P],
    "pipnet_nchw_to_s2d_bf16": [P, I32, I32, I32, P, P],
    "pipnet_stem_pool_bf16": [P, I32, I32, I32, P, P, P, P],
    "pipnet_conv1x1_bf16_dual": [P, I64, I32, P, P, I32, P, I32, P, P],
    "pipnet_softmax_pool_bf16": [P, I32, I32, I32, I32, P, P, P],
    "pipnet_eval_batch_f32": [P, P, P, I32, I32, I32, P, P, F32, P, P, P, P, P, P, P],
    "pipnet_weight_sparsify_f32": [P, I64, F32, P],
    "pipnet_dwconv7_ln_f32": [P, I32, I32, I32, I32, P, P, P, P, P, P],
    "pipnet_layernorm_f32": [P, I64, I32, P, P, P, P],
    "pipnet_softmax_pool_f32": [P, I32, I32, I32, I32, P, P, P],
    "pipnet_softmax_pool_linear_part_floats": [I32, I32, I32],
    "pipnet_softmax_pool_linear_f32": [P, I32, I32, I32, P, P, P, P, I32, I32, F32, P, P, P, P, P],
    "pipnet_softmax_pool_linear_bf16": [P, I32, I32, I32, P, P, P, P, I32, I32, F32, P, P, P, P, P],
    "pipnet_nonneg_linear_f32": [P, I32, I32, P, P, I32, I32, F32, P, P, P],
    "pipnet_count_gumbel_f32": [P, I32, I32, I32, F32, P, U64, U64, P, P, P],
    "pipnet_count_gumbel_devseed_f32": [P, I32, I32, I32, F32, P, P, P, P],
    "pipnet_count_finish_f32": [P, P, I32, I32, I32, I32, P, P, P],
    "pipnet_count_encode_f32": [P, I32, I32, I32, I32, I32, P, P, P],
    "pipnet_resize_plan": [P, I32, I32, I32, P, P],
    "pipnet_resize_normalize_rgb8": [P, P, P, I32, I32, I32, I32, I32, P, P, P, P, P, P],
    "pipnet_train_align_partials": [],
    "pipnet_train_align_partial_f32": [P, I32, I32, I32, P, P],
    "pipnet_train_loss_f32": [P, I32, I32, P, P, P, I32, I32, P, I32, F32, F32, F32, F32, I32, P, P, P],
    "pipnet_nonneg_linear_bwd_f32": [P, P, I32, I32, P, I32, P, P, P],
    "pipnet_adamw_step_f32": [P, P, P, P, I64, F64, F64, F64, F64, F64, I64, I32, F32, F32, P],
    "pipnet_clamp_min_f32": [P, I64, F32, P],
    "pipnet_wgrad_workspace_bytes": [I32, I32, I32],
    "pipnet_wgrad_f32": [P, I64, P, I64, I32, I32, I32, P, I64, I32, P, P],
    "pipnet_wgrad_conv2x2_f32": [P, P, I32, I32, I32, I32, I32, I32, P, I32, P, P],
    "pipnet_wgrad_conv_f32": [P, P, I32, I32, I32, I32, I32, I32, I32, I32, I32, P, I32, P, P],
    "pipnet_colsum_workspace_bytes": [I32],
    "pipnet_colsum_f32": [P, I64, I32, I32, P, I32, P, P],
    "pipnet_train_partials_floats": [I32],
    "pipnet_gelu_fwd_f32": [P, P, I64, P],
    "pipnet_resid_scale_f32": [P, P, P, P, I32, I64, I32, P, P],
    "pipnet_ls_bwd_f32": [P, P, P, P, I32, I64, I32, P, P, P, I32, P, P],
    "pipnet_ln_bwd_f32": [P, P, P, I64, I32, P, P, P, I32, P, P],
    "pipnet_dwconv7_plain_f32": [P, I32, I32, I32, I32, P, P, I32, P, P],
    "pipnet_dwconv7_wgrad_f32": [P, P, I32, I32, I32, I32, P, P, I32, P, P],
    "pipnet_head_bwd_f32": [P, P, I32, I32, I32, P, P, I32, F32, F32, F32, P, P, P, P],
    "pipnet_cnblock_mlp_f32": [P, P, P, P, P, P, P, I64, I32, P],
    "pipnet_cnblock_mlp_hw_f32": [P, P, P, P, P, P, P, I64, I32, I32, P],
    "pipnet_bn_workspace_floats": [I32],
    "pipnet_bn_stats_f32": [P, I64, I32, F32, F32, P, P, P, P, P, P],
    "pipnet_bn_apply_f32": [P, I64, I32, P, P, P, P, P, I32, P, P],
    "pipnet_bn_backward_f32": [P, P, P, I64, I32, P, P, P, P, P, P, P, P, P],
    "pipnet_stride_scatter_f32": [P, I32, I32, I32, I32, I32, I32, I32, I32, P, P],
}
_RESTYPE_EXTRA = {"pipnet_wgrad_workspace_bytes": ctypes.c_int64, "pipnet_train_partials_floats": ctypes.c_int64,
                  "pipnet_bn_workspace_floats": ctypes.c_int64,
                  "pipnet_softmax_pool_linear_part_floats": ctypes.c_int64}
_RESTYPE = {"pipnet_amd_status_string": ctypes.c_char_p, "pipnet_amd_source_digest": ctypes.c_char_p,
            **_RESTYPE_EXTRA}

EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_RESID, EPI_MUL, EPI_BIAS_RELU, EPI_BIAS_RESID_RELU = 0, 1, 2, 3, 4, 5, 6
EPI_RESID_ROWSCALE = 7
EPI_GELU_BWD = 8
EPI_S3_GELU, EPI_F32_BIAS, EPI_F32_RESID = 9, 10, 11      # split-bf16 ("bf16x3") ConvNeXt path
EPI_DUAL_BIAS_RELU = 12        # pipnet_conv1x1_bf16_dual: downsample + conv1 of a first Bottleneck

ABI_VERSION = 3          # include/pipnet_amd.h PIPNET_AMD_ABI_VERSION

_lib = None


class PipnetLibraryError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise if it is absent or incomplete."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PipnetLibraryError(
            f"{LIB_PATH} is missing: the MI355X inference path has no fallback. "
            "Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `python count_pipnet_amd/build.py`.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)          # AttributeError = missing export = loud failure
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
    _check_provenance(lib)
    if lib.pipnet_amd_abi_version() != ABI_VERSION:
        raise PipnetLibraryError(f"{LIB_PATH} exports ABI version {lib.pipnet_amd_abi_version()}, "
                                 f"this binding expects {ABI_VERSION} (include/pipnet_amd.h)")
    _lib = lib
    return lib


def _check_provenance(lib) -> None:
    """The library must have been compiled from the sources of this tree (sha256 compiled
    in by build.py).  ``PIPNET_AMD_ALLOW_STALE=1`` is the explicit A/B escape hatch (e.g. an
    experimental build loaded through ``PIPNET_AMD_LIB``)."""
    from .build import source_digest
    built = lib.pipnet_amd_source_digest().decode()
    here = source_digest()
    if built != here and os.environ.get("PIPNET_AMD_ALLOW_STALE") != "1":
        raise PipnetLibraryError(
            f"{LIB_PATH} was built from other sources (digest {built[:16]}..., tree {here[:16]}...): "
            "rebuild with `python count_pipnet_amd/build.py` (or set PIPNET_AMD_ALLOW_STALE=1 for an A/B run)")


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().pipnet_amd_status_string(status).decode()
        raise RuntimeError(f"{what} failed: PIPNET status {status} ({msg})")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)
