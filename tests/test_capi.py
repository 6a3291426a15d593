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
