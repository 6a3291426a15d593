"""CPU: every 16-bit Linear GEMM of the benchmarked step routes to a hand-written kernel.

SURVEY 8(a) row 8 (torchvision's block: qkv / proj / mlp.0 / mlp.3, model_parts.py:143-151) and
the Linears around it (PatchMerging.reduction :87-95, PatchExpand.expand, concat_back_dim
:792-824, FinalPatchExpand_X4_V2.expand :458): forward and input-gradient GEMMs at the Swin-T /
Swin-S / Swin-B widths for 8 x 1024^2 (and 8 x 512^2) go to the token GEMM (csrc/gemm_tok.h) or
the persistent tiled NT GEMM (csrc/gemm_nt.hip), never to the library GEMM, unless the
MSU_GEMM_ROUTE=lib A/B switch asks for it.  The routing queries are host functions of the C-ABI
library (no GPU needed).
"""
import pytest

from semantic_segmentation_of_stylegan2_artifacts_amd import ops


def _shapes(C, B, img):
    """(M, N, K, epi) of every Linear forward and input gradient of the step."""
    out = []
    res = img // 4
    for s in range(4):
        c = C * 2 ** s
        M = B * (res // 2 ** s) ** 2
        for n, k in ((3 * c, c), (c, c), (c, 2 * c), (2 * c, c)):  # qkv, proj, concat, expand
            out += [(M, n, k, ops.TOK_PLAIN), (M, k, n, ops.TOK_PLAIN)]
        out += [(M, 4 * c, c, ops.TOK_GELU_DUAL), (M, c, 4 * c, ops.TOK_PLAIN),   # mlp.0 / mlp.3 fwd
                (M, 4 * c, c, ops.TOK_GELU_GRAD), (M, c, 4 * c, ops.TOK_PLAIN)]   # mlp.3 / mlp.0 dgrad
        if s < 3:  # PatchMerging reduction 4c -> 2c at the next stage's token count
            out += [(M // 4, 2 * c, 4 * c, ops.TOK_PLAIN), (M // 4, 4 * c, 2 * c, ops.TOK_PLAIN)]
    M0 = B * res * res
    out += [(M0, 16 * C, C, ops.TOK_GELU_DUAL), (M0, C, 16 * C, ops.TOK_PLAIN),  # x4 expand
            (M0, C, 48, ops.TOK_PLAIN)]  # patch embed (im2col K = 3 * 4 * 4)
    return out


@pytest.mark.parametrize("C,img", [(96, 1024), (96, 512), (128, 1024)])
def test_every_step_gemm_is_hand_written(C, img, monkeypatch):
    monkeypatch.setattr(ops, "_ROUTE_FORCE", "")
    monkeypatch.setattr(ops, "_tok_cache", {})
    lib = [(M, N, K, e) for M, N, K, e in _shapes(C, 8, img) if ops.gemm_route(M, N, K, e) == "lib"]
    assert not lib, lib


def test_lib_switch_still_reaches_the_library(monkeypatch):
    monkeypatch.setattr(ops, "_ROUTE_FORCE", "lib")
    monkeypatch.setattr(ops, "_tok_cache", {})
    assert ops.gemm_route(8 * 64 ** 2, 3 * 384, 384) == "lib"
