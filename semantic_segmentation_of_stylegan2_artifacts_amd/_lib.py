"""ctypes binding of the C-ABI in ``include/msunet_hip.h`` (``libmsunet_hip.so``).

There is no CPU fallback: if the library is missing or fails to load, every op raises.
"""
import ctypes
import os

from . import switches

_HERE = os.path.dirname(os.path.abspath(__file__))
# MSU_LIB_OVERRIDE: an alternative build of the same library (kernel ablation builds made by
# tools/build_exp.sh); the product path never sets it
LIB_PATH = switches.get("MSU_LIB_OVERRIDE") or os.path.join(_HERE, "libmsunet_hip.so")

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float
D = ctypes.c_double
U64 = ctypes.c_ulonglong

# name -> (restype, argtypes); must match include/msunet_hip.h
SIGNATURES = {
    "msu_ln_part_blocks": (I, [L, I]),
    "msu_layernorm_fwd": (I, [I, I, P, P, P, L, P, P, P, P, P, P, L, I, I, I, I, F, P]),
    "msu_layernorm_bwd": (I, [I, I, P, P, P, P, P, P, P, P, P, L, P, I, P, P, L, I, I, I, I, I, P]),
    "msu_layernorm_bwd3": (I, [I, I, P, P, P, P, P, P, P, P, P, P, P, L, P, I, P, P, L, I, I, I, I, I, P]),
    "msu_reduce_rows": (I, [P, I, I, L, P, I, P]),
    "msu_tail_reduce_mode": (I, [I]),
    "msu_conv_mode": (I, [I]),
    "msu_head_fwd": (I, [I, P, P, P, P, P, P, P, L, I, F, P]),
    "msu_head_bwd": (I, [I, P, P, P, P, P, P, P, P, P, I, P, P, P, L, I, P]),
    "msu_head_bwd2": (I, [I, P, P, P, P, P, P, P, P, P, I, P, P, P, L, I, I, P]),
    "msu_win_count": (L, [I, I, I]),
    "msu_win_attn_fwd_workspace": (L, [I, I, I]),
    "msu_win_attn_keep_words": (L, [I, I, I, I, I]),
    "msu_win_attn_fwd": (I, [I, P, P, P, P, P, I, I, I, I, I, I, F, U64, P, P, P]),
    "msu_win_attn_bwd_workspace": (L, [I, I, I, I, I, I]),
    "msu_win_attn_bwd": (I, [I, P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, U64, P, P, P]),
    "msu_win_attn_bwd2": (I, [I, P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, U64, P, P, P, P]),
    "msu_win_attn_bwd_tail": (I, [I, P, P, P, I, I, I, I, I, P]),
    "msu_win_attn_bwd_tail2": (I, [I, P, P, P, I, I, I, I, I, I, P]),
    "msu_win_attn_qkv_supported": (I, [I, I]),
    "msu_win_attn_qkv_fwd": (I, [I, P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, U64, P, P]),
    "msu_win_attn_qkv_fwd2": (I, [I, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, U64, P, P]),
    "msu_mlp_fused_supported": (I, [I, I]),
    "msu_mlp_fused_fwd": (I, [I, P, P, P, P, P, P, P, L, I, I, P]),
    "msu_add_ln_mlp_fwd": (I, [I, P, P, P, L, P, P, F, P, P, P, P, P, P, L, I, I, P]),
    "msu_gelu_fwd": (I, [I, P, P, L, P]),
    "msu_gelu_bwd": (I, [I, P, P, P, L, P]),
    "msu_residual": (I, [I, P, P, P, P, L, L, P]),
    "msu_patchify": (I, [I, P, P, I, I, I, I, I, P]),
    "msu_dynloss_nblk": (I, [L]),
    "msu_dynloss_fwd": (I, [I, P, P, I, L, F, F, F, P, I, P, P, P]),
    "msu_dynloss_bwd": (I, [I, P, P, P, P, P, I, L, F, F, F, P, P]),
    "msu_dynloss_fwd2": (I, [I, P, P, I, L, F, F, F, P, I, P, P, P, P]),
    "msu_dynloss_fwd3": (I, [I, P, P, I, L, F, F, F, P, I, P, P, P, P, P]),
    "msu_dynloss_bwd2": (I, [I, P, P, P, P, P, I, L, F, F, F, P, P]),
    "msu_adamw": (I, [P, P, P, P, L, F, F, F, F, F, I, P, P, P]),
    "msu_nonfinite": (I, [P, L, P, P]),
    "msu_nonfinite2": (I, [P, L, P, L, P, P]),
    "msu_adamw_dev": (I, [P, P, P, P, L, P, D, D, D, D, P, P, P]),
    "msu_adamw_dev2": (I, [P, P, P, P, L, P, D, D, D, D, P, P, P, I, I, P]),
    "msu_step_advance": (I, [P, P, P]),
    "msu_cast": (I, [I, P, P, L, P]),
    "msu_colsum_batch": (I, [I, P, P, P, P, P, I, P]),
    "msu_conv3x3_weight": (I, [I, P, P, I, I, I, P]),
    "msu_transpose16_multi": (I, [P, P, P, I, I, P]),
    "msu_conv3x3_fwd": (I, [I, I, P, P, P, P, I, I, I, I, I, P]),
    "msu_conv3x3_fwd2": (I, [I, I, P, P, P, P, P, I, I, I, I, I, P]),
    "msu_conv3x3_dgrad": (I, [I, I, P, P, P, P, I, I, I, I, I, P]),
    "msu_conv3x3_wgrad_workspace": (L, [I, I, I, I, I]),
    "msu_conv3x3_wgrad": (I, [I, I, P, P, P, P, P, P, I, I, I, I, I, I, P]),
    "msu_conv3x3_wgrad2": (I, [I, I, P, P, P, P, P, I, I, I, I, I, I, I, P]),
    "msu_wgrad_splits": (I, [L, I, I]),
    "msu_wgrad_workspace": (L, [L, I, I]),
    "msu_linear_wgrad": (I, [I, P, P, P, P, P, L, I, I, I, P]),
    "msu_linear_wgrad_ld": (I, [I, P, P, P, L, P, P, L, I, I, I, P]),
    "msu_linear_bwd_supported": (I, [L, I, I]),
    "msu_linear_bwd_workspace": (L, [L, I, I]),
    "msu_linear_bwd": (I, [I, P, P, P, P, P, P, P, P, L, I, I, I, P]),
    "msu_tok_gemm_supported": (I, [L, I, I]),
    "msu_tok_gemm_supported_epi": (I, [L, I, I, I]),
    "msu_tok_gemm": (I, [I, P, P, I, P, P, P, P, P, L, I, I, I, P]),
    "msu_tok_gemm_plan": (I, [L, I, I, P]),
    "msu_nt_gemm_supported": (I, [L, I, I]),
    "msu_nt_gemm_plan": (I, [L, I]),
    "msu_nt_gemm_mode": (I, [I]),
    "msu_nt_gemm": (I, [I, P, P, P, P, P, P, L, I, I, I, P]),
    "msu_nt_gemm_kn": (I, [I, P, P, P, P, P, P, L, I, I, I, P]),
    "msu_nt_gemm_cat": (I, [I, P, P, I, P, P, P, L, I, I, P]),
    "msu_metrics_nblk": (I, [L]),
    "msu_seg_metrics": (I, [I, P, P, I, L, F, P, I, P, P]),
    "msu_augment_batch": (I, [P, P, P, P, P, P, I, I, I, P]),
}

_lib = None


class HipLibraryError(RuntimeError):
    pass


def lib():
    """Load (once) and return the HIP library; raise loudly when it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipLibraryError(
            f"{LIB_PATH} not found: build it with "
            "`python -m semantic_segmentation_of_stylegan2_artifacts_amd.build` (no CPU fallback)")
    h = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = args
    # the library-side A/B switches (the C code reads no environment; switches.py does)
    h.msu_nt_gemm_mode((1 if switches.on("MSU_NT_PP") else 0) | (16 if switches.on("MSU_NT_DYN") else 0))
    h.msu_tail_reduce_mode(1 if switches.on("MSU_TAIL") else 0)
    h.msu_conv_mode(1 if switches.on("MSU_CONV_DYN") else 0)
    _lib = h
    return _lib


def plan_nt(M, N):
    """(tile rows, tile columns, ping-pong kernel?) msu_nt_gemm uses for an M x N output."""
    v = lib().msu_nt_gemm_plan(M, N)
    return (v % 1000000) // 1000, v % 1000, v >= 1000000


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise HipLibraryError(f"{name} failed with code {rc}")
    return rc
