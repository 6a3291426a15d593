"""CPU: the C-ABI library builds/loads and exports every symbol include/msunet_hip.h declares,
with ctypes signatures that match the header (no compute calls: no GPU here)."""
import os
import re

import pytest

from semantic_segmentation_of_stylegan2_artifacts_amd import _lib

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "msunet_hip.h")


def _declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(int|long)\s+(msu_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.S):
        args = [a.strip() for a in m.group(3).split(",") if a.strip()]
        out[m.group(2)] = (m.group(1), args)
    return out


def _ctype_of(decl):
    d = decl.replace("const", "").strip()
    if "*" in d:
        return "P"
    t = d.rsplit(" ", 1)[0].strip()
    return {"int": "I", "long": "L", "float": "F", "double": "D", "unsigned long long": "U64"}[t]


def test_header_and_bindings_agree():
    decl = _declared()
    assert decl, "no declarations parsed"
    names = {v: k for k, v in vars(_lib).items() if k in ("P", "I", "L", "F", "D", "U64")}
    assert set(decl) == set(_lib.SIGNATURES), set(decl) ^ set(_lib.SIGNATURES)
    for name, (ret, args) in decl.items():
        res, argtypes = _lib.SIGNATURES[name]
        assert names[res] == {"int": "I", "long": "L"}[ret], name
        assert [names[a] for a in argtypes] == [_ctype_of(a) for a in args], name


def test_library_loads_and_exports_all_symbols():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmsunet_hip.so not built (run __graft_entry__.build())")
    h = _lib.lib()
    for name in _declared():
        assert hasattr(h, name), name


def test_missing_library_raises(monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libmsunet_hip.so")
    with pytest.raises(_lib.HipLibraryError):
        _lib.lib()


def test_ops_refuse_cpu_tensors():
    import torch
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    x = torch.zeros(4, 32)
    with pytest.raises(RuntimeError):
        ops.layer_norm(x, torch.ones(32), torch.zeros(32))


def test_torch_library_ops_registered():
    """The hot-path ops are torch.library custom ops (torch.ops.msunet.*) with schemas, fake
    kernels (shape propagation without a device) and autograd formulas."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    expected = {"layer_norm", "add_layer_norm", "merge_layer_norm", "d2s_layer_norm", "window_attention",
                "linear", "linear_cat", "mlp", "residual", "gelu", "head_norm_output", "refine_conv",
                "refine_conv_act", "linear_gelu", "patchify", "dynamic_loss"}
    assert expected <= set(ops.registered_ops())
    for name in expected:
        op = getattr(torch.ops.msunet, name).default
        assert str(op._schema).startswith(f"msunet::{name}(")
    with FakeTensorMode():
        qkv = torch.empty(2, 10, 12, 3 * 64, device="cuda", dtype=torch.float16)
        out, keep, _ = torch.ops.msunet.window_attention(qkv, torch.empty(192, device="cuda"),
                                                      torch.empty(169, 2, device="cuda"), 2, 3, 0.0, 0, None)
        assert out.shape == (2, 10, 12, 64) and out.dtype == torch.float16 and keep.numel() == 0
        # with dropout the forward also returns its keep bits (128 words per window x head)
        _, keep, _ = torch.ops.msunet.window_attention(qkv, torch.empty(192, device="cuda"),
                                                    torch.empty(169, 2, device="cuda"), 2, 3, 0.1, 0, None)
        assert keep.shape == (2 * 2 * 2 * 2 * 128,) and keep.dtype == torch.int32
        y, mean, rstd = torch.ops.msunet.layer_norm(torch.empty(5, 96, device="cuda"), torch.empty(96, device="cuda"),
                                                    torch.empty(96, device="cuda"), 1e-5)
        assert y.shape == (5, 96) and mean.shape == (5,)
    # a CPU tensor has no kernel (no silent CPU fallback)
    with pytest.raises(NotImplementedError):
        torch.ops.msunet.gelu(torch.zeros(8))


def test_python_workspace_sizes_match_the_library():
    """The fake kernels size the attention workspaces / keep bits and pick the mlp route from
    Python restatements (no library needed for shape propagation); they equal the library's
    own msu_win_attn_*_workspace / keep_words / msu_mlp_fused_supported."""
    import torch
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    L = _lib.lib()
    for dt, code in ((torch.bfloat16, 1), (torch.float16, 2), (torch.float32, 0)):
        for B, H, W, nh in ((1, 7, 7, 1), (2, 10, 12, 2), (8, 256, 256, 3), (8, 128, 128, 6), (8, 64, 64, 12),
                            (8, 32, 32, 24), (1, 56, 56, 3), (3, 15, 9, 4), (8, 16, 16, 32)):
            C = 32 * nh
            assert ops._attn_fwd_ws(dt, C, nh) == L.msu_win_attn_fwd_workspace(code, C, nh)
            assert ops._attn_bwd_ws(dt, B, H, W, C, nh) == L.msu_win_attn_bwd_workspace(code, B, H, W, C, nh)
            assert ops._attn_keep_words(dt, B, H, W, nh) == L.msu_win_attn_keep_words(code, B, H, W, nh)
    for C, Hd in ((96, 384), (192, 768), (96, 192), (384, 96), (384, 1536)):
        assert ((C, Hd) in ops.MLP_KERNEL_SHAPES) == bool(L.msu_mlp_fused_supported(C, Hd))
        if ops._mlp_fused_ok(C, Hd):
            assert (C, Hd) in ops.MLP_KERNEL_SHAPES


def test_mlp_fake_matches_the_route_contract():
    """msunet::mlp's fake kernel reports the outputs the real kernel returns -- with
    keep (training) on the fused route H is [..., Hd] and G is empty (the backward re-derives
    GELU(H)); on the GEMM-pair route (f32, other widths) G is [..., Hd] too; without keep both
    are empty."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    with FakeTensorMode():
        for dt, C, Hd, fused in ((torch.bfloat16, 96, 384, ops._MLP_TRAIN), (torch.float16, 96, 384, ops._MLP_TRAIN),
                                 (torch.bfloat16, 192, 768, ops._MLP_TRAIN and ops._MLP_S1),
                                 (torch.bfloat16, 384, 1536, False), (torch.float32, 96, 384, False)):
            x = torch.empty(4, 7, C, device="cuda", dtype=dt)
            w1, w2 = torch.empty(Hd, C, device="cuda"), torch.empty(C, Hd, device="cuda")
            b1, b2 = torch.empty(Hd, device="cuda"), torch.empty(C, device="cuda")
            y, h, g = torch.ops.msunet.mlp(x, w1, b1, w2, b2, True)
            assert y.shape == (4, 7, C) and h.shape == (4, 7, Hd)
            assert g.numel() == 0 if fused else g.shape == (4, 7, Hd)
            y, h, g = torch.ops.msunet.mlp(x, w1, b1, w2, b2, False)
            assert y.shape == (4, 7, C) and h.numel() == 0 and g.numel() == 0
        # the fused stage-0 attention unit's fake sizes its workspace without the library
        x = torch.empty(2, 14, 14, 96, device="cuda", dtype=torch.bfloat16)
        out = torch.ops.msunet.window_attention_qkv(
            x, torch.empty(288, 96, device="cuda"), torch.empty(288, device="cuda"), torch.empty(169, 3, device="cuda"),
            torch.empty(96, 96, device="cuda"), torch.empty(96, device="cuda"), 3, 3, 0.1, 0, None, True)
        assert out[0].shape == (2, 14, 14, 96) and out[2].shape == (2, 14, 14, 288)
        assert out[3].numel() == 2 * 2 * 2 * 3 * 128
        assert out[4].numel() == ops._attn_ws_numel(torch.bfloat16, 2, 14, 14, 96, 3)
