"""GPU: the fused MLP (csrc/mlp_fused.hip) against plain fp32 PyTorch and against the token-GEMM
pair: the inference form (ops.mlp without autograd) and the training form (H stored, all
gradients through the one-pass backward).

Reference: fp32 of the same 16-bit operands with the kernel's two roundings (the pre-activation
and GELU(H) stored in 16 bits, as the unfused epilogues do), exact erf GELU.  Tolerance as the
token-GEMM tests: |y - ref| <= 1e-2 |ref| + 4e-3 max|ref| (one f32 -> 16-bit rounding of the
output, different summation order; A&S 7.1.26 erf |err| <= 1.5e-7).  Against the training path
(same roundings, bias added in f32 instead of as a hi / lo k-block): rel. L2 <= 2e-3.
Every case runs for both 16-bit formats.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    return ops


@pytest.fixture(params=[torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def low(request):
    return request.param


def _params(seed, low, C=96):
    g = torch.Generator().manual_seed(seed)
    Hd = 4 * C
    w1 = torch.nn.Parameter((torch.randn(Hd, C, generator=g) / C ** 0.5).to(DEV))
    b1 = torch.nn.Parameter((torch.randn(Hd, generator=g) * 0.1).to(DEV))
    w2 = torch.nn.Parameter((torch.randn(C, Hd, generator=g) / Hd ** 0.5).to(DEV))
    b2 = torch.nn.Parameter((torch.randn(C, generator=g) * 0.1).to(DEV))
    return w1, b1, w2, b2


def _ref(x, w1, b1, w2, b2, low):
    h = (x.float() @ w1.detach().to(low).float().t() + b1.detach()).to(low).float()
    g = F.gelu(h).to(low).float()
    return g @ w2.detach().to(low).float().t() + b2.detach()


# M: ragged tails (tile 32 / 256), one wave's worth, several tiles per wave, production (stage 0:
# 8 x 256^2 tokens; stage 1, C = 192: 8 x 128^2)
@pytest.mark.parametrize("M,C", [(1, 96), (33, 96), (1000, 96), (8192 + 17, 96), (524288, 96),
                                 (1, 192), (33, 192), (1000, 192), (8192 + 17, 192), (131072, 192)])
def test_mlp_infer_matches_fp32(M, C, low):
    ops = _ops()
    w1, b1, w2, b2 = _params(M, low, C)
    x = torch.randn(M, C, generator=torch.Generator().manual_seed(M + 1)).to(DEV, low)
    n0 = ops.mlp_infer_calls
    with torch.no_grad(), torch.autocast("cuda", dtype=low):
        y = ops.mlp(x, w1, b1, w2, b2)
    assert ops.mlp_infer_calls == n0 + 1, "the no-grad MLP did not take the fused kernel"
    assert y.dtype == low and y.shape == (M, C)
    ref = _ref(x, w1, b1, w2, b2, low)
    scale = ref.abs().max().item()
    err = (y.float() - ref).abs() - 1e-2 * ref.abs()
    assert err.max().item() <= 4e-3 * scale, f"M={M}: excess err {err.max().item():.3e} vs scale {scale:.3e}"


def test_mlp_infer_matches_training_path(low, monkeypatch):
    """The same block forward with autograd off (fused kernel) and on with the training MLP
    forced onto the token-GEMM pair (MSU_MLP_TRAIN=0: H / GELU(H) kept); the fused training form
    (H stored) against the same pair: y and the stored pre-activation H."""
    ops = _ops()
    w1, b1, w2, b2 = _params(7, low)
    x = torch.randn(4, 64, 64, 96, generator=torch.Generator().manual_seed(8)).to(DEV, low)
    monkeypatch.setattr(ops, "_MLP_TRAIN", False)
    t0 = ops.mlp_train_calls
    with torch.autocast("cuda", dtype=low):
        y_pair, h_pair, g_pair = torch.ops.msunet.mlp(x.clone().requires_grad_(True), w1, b1, w2, b2, True)
    assert ops.mlp_train_calls == t0 and g_pair.numel() == h_pair.numel(), "the pair arm took the fused kernel"
    n0 = ops.mlp_infer_calls
    with torch.no_grad(), torch.autocast("cuda", dtype=low):
        y_inf = ops.mlp(x, w1, b1, w2, b2).float()
    assert ops.mlp_infer_calls == n0 + 1
    rel = ((y_inf - y_pair.float()).norm() / y_pair.float().norm()).item()
    assert rel <= 2e-3, rel
    monkeypatch.setattr(ops, "_MLP_TRAIN", True)
    with torch.autocast("cuda", dtype=low):
        y_tr, h_tr, g_tr = torch.ops.msunet.mlp(x.clone().requires_grad_(True), w1, b1, w2, b2, True)
    assert ops.mlp_train_calls == t0 + 1 and g_tr.numel() == 0
    for name, a, b in (("y", y_tr, y_pair), ("H", h_tr, h_pair)):
        rel = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert rel <= 2e-3, (name, rel)


# M: ragged (one partial tile), several tiles + a ragged tail, production (stage 0: 8 x 256^2
# tokens, stage 1: 8 x 128^2)
@pytest.mark.parametrize("M,C", [(33, 96), (8209, 96), (524288, 96), (33, 192), (8209, 192), (131072, 192)])
def test_mlp_train_matches_fp32(M, C, low):
    """the training form of the fused MLP (stage 0: mlp_fused_kernel with H
    stored, mlp.3's one-pass backward re-deriving GELU(H) from H; stage 1: mlp_s1_kernel, mlp.3's
    weight gradient on GELU(H) derived on the side stream) under autograd against fp32 PyTorch on
    the same 16-bit operands: y and the stored H with the token-GEMM tolerance, dx / dW1 / db1 /
    dW2 / db2 within 3e-2 of the largest entry (16-bit H, GELU(H) and dH in between), as
    tests/test_gpu_tok_gemm.py::test_fused_mlp_matches_fp32."""
    ops = _ops()
    if not ops._MLP_TRAIN:
        pytest.skip("MSU_MLP_TRAIN=0")
    w1, b1, w2, b2 = _params(M + 3, low, C)
    Hd = 4 * C
    # trainer-style parameters (flat .grad, 16-bit shadows, direct accumulation): the backward
    # takes the production route -- at M >= the one-pass threshold mlp.3's pass re-derives
    # GELU(H) from H (msu_linear_bwd with X = null), then mlp.0's pass
    for p_ in (w1, b1, w2, b2):
        p_.grad = torch.zeros_like(p_)
        p_._msu_direct = True
        p_._msu_shadow = p_.detach().to(low)
        if p_.dim() == 2:
            p_._msu_shadow_t = p_.detach().t().contiguous().to(low)
        p_._msu_shadow_ver = p_._version
    g = torch.Generator().manual_seed(M + 4)
    x = torch.randn(M, C, generator=g).to(DEV, low)
    dy = torch.randn(M, C, generator=g).to(DEV, low)
    # fp32 reference on the 16-bit operands (inputs, weights, upstream gradient)
    xr = x.float().requires_grad_(True)
    pr = [t.detach().to(low).float().requires_grad_(True) if t.dim() == 2 else t.detach().clone().requires_grad_(True)
          for t in (w1, b1, w2, b2)]
    hr = F.linear(xr, pr[0], pr[1])
    yr = F.linear(F.gelu(hr), pr[2], pr[3])
    yr.backward(dy.float())
    xg = x.clone().requires_grad_(True)
    t0 = ops.mlp_train_calls
    with torch.autocast("cuda", dtype=low):
        y, h, gg = torch.ops.msunet.mlp(xg, w1, b1, w2, b2, True)
    assert ops.mlp_train_calls == t0 + 1, "the training MLP did not take the fused kernel"
    assert gg.numel() == 0 and h.shape == (M, Hd) and h.dtype == low
    l0 = ops.linbwd_calls
    y.backward(dy)
    torch.cuda.synchronize()
    if M >= ops._LINBWD_MIN_M and C == 96:
        assert ops.linbwd_calls == l0 + 2, "the backward did not take the one-pass route"
    for name, a, r in (("y", y, yr), ("H", h, hr)):
        r = r.detach()
        scale = r.abs().max().item()
        err = (a.float() - r).abs() - 1e-2 * r.abs()
        assert err.max().item() <= 4e-3 * scale, f"{name} M={M}: excess err {err.max().item():.3e} vs {scale:.3e}"
    for name, a, r in (("dx", xg.grad, xr.grad), ("dw1", w1.grad, pr[0].grad), ("db1", b1.grad, pr[1].grad),
                       ("dw2", w2.grad, pr[2].grad), ("db2", b2.grad, pr[3].grad)):
        err = (a.float() - r).abs().max().item()
        assert err <= 3e-2 * r.abs().max().item(), f"{name} M={M}: {err:.3e} vs {r.abs().max().item():.3e}"


def test_mlp_infer_other_widths_keep_token_gemm_pair():
    """Stage-2 widths (384 -> 1536) are not covered: the no-grad MLP keeps the GEMM pair."""
    ops = _ops()
    g = torch.Generator().manual_seed(5)
    w1 = torch.nn.Parameter((torch.randn(1536, 384, generator=g) / 384 ** 0.5).to(DEV))
    b1 = torch.nn.Parameter((torch.randn(1536, generator=g) * 0.1).to(DEV))
    w2 = torch.nn.Parameter((torch.randn(384, 1536, generator=g) / 1536 ** 0.5).to(DEV))
    b2 = torch.nn.Parameter((torch.randn(384, generator=g) * 0.1).to(DEV))
    x = torch.randn(4096, 384, generator=g).to(DEV, torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        fusable = ops.mlp_fusable(x, w1, w2)
    if not fusable:
        pytest.skip("stage-2 MLP not on the fused GEMM pair")
    n0 = ops.mlp_infer_calls
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.mlp(x, w1, b1, w2, b2)
    assert ops.mlp_infer_calls == n0
    ref = _ref(x, w1, b1, w2, b2, torch.bfloat16)
    scale = ref.abs().max().item()
    assert ((y.float() - ref).abs() - 1e-2 * ref.abs()).max().item() <= 4e-3 * scale


def test_dead_branches_take_fused_mlp():
    """The reference's discarded branches (layers_cent1[-1], layers_cent2[-1]: stage-0 Swin
    blocks run without autograd) go through the fused inference MLP."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config, ops
    from semantic_segmentation_of_stylegan2_artifacts_amd.network import MSUNet
    cfg = load_config(None, "swin_t", **{"DATA.IMG_SIZE": 1024, "DATA.BATCH_SIZE": 1})
    torch.manual_seed(0)
    model = MSUNet(cfg, img_size=1024, num_classes=1).to(DEV).train()
    x = torch.randn(1, 3, 1024, 1024, device=DEV)
    probe = torch.empty(65536, 96, device=DEV, dtype=torch.bfloat16)
    blk = model.ms_unet.layers[0].blocks[0]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        fusable = ops.mlp_fusable(probe, blk.mlp[0].weight, blk.mlp[3].weight)
    if blk.dropout > 0 or not fusable:
        pytest.skip("stage-0 MLP not on the fused path in this configuration")
    n0, l0 = ops.mlp_infer_calls, ops.add_ln_mlp_calls
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = model(x)
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all()
    fused = (ops.mlp_infer_calls - n0) + (ops.add_ln_mlp_calls - l0)
    assert fused == 4, fused  # 2 + 2 dead stage-0 blocks
    if ops._MLP_LN:
        assert ops.add_ln_mlp_calls - l0 == 4  # norm2 folded in


def test_linbwd_gelu_from_h_matches_explicit_gelu(low):
    """mlp.3's one-pass backward with X = null re-derives GELU(H) while staging: bitwise the same
    dX / dW / db as with the GELU(H) tensor the token-GEMM pair stored (same gelu_fast, same
    16-bit rounding)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    ops = _ops()
    L = _lib.lib()
    M, K, N = 4096 + 17, 384, 96
    g = torch.Generator().manual_seed(11)
    dy = torch.randn(M, N, generator=g).to(DEV, low)
    h = torch.randn(M, K, generator=g).to(DEV, low)
    wt = (torch.randn(K, N, generator=g) / K ** 0.5).to(DEV, low)
    with torch.no_grad(), torch.autocast("cuda", dtype=low):
        gx = ops.gelu(h)
    assert gx.dtype == low and gx.is_contiguous()
    s = torch.cuda.current_stream().cuda_stream
    out = []
    for X in (gx, None):
        dx = torch.empty(M, K, device=DEV, dtype=low)
        dw = torch.zeros(N, K, device=DEV)
        db = torch.zeros(N, device=DEV)
        ws = torch.empty(L.msu_linear_bwd_workspace(M, K, N), device=DEV)
        _lib.call("msu_linear_bwd", ops._dt(h), dy.data_ptr(), None if X is None else X.data_ptr(), wt.data_ptr(),
                  h.data_ptr(), dx.data_ptr(), dw.data_ptr(), db.data_ptr(), ws.data_ptr(), M, K, N, 1, s)
        out.append((dx, dw, db))
    torch.cuda.synchronize()
    for a, b, name in zip(out[0], out[1], ("dx", "dW", "db")):
        assert torch.equal(a, b), name
    ref_dw = dy.float().t() @ F.gelu(h.float()).to(low).float()
    assert ((out[1][1] - ref_dw).norm() / ref_dw.norm()).item() < 1e-2


@pytest.mark.parametrize("with_scale", [False, True])
def test_add_ln_mlp_matches_two_kernels(with_scale, low):
    """No-grad norm2 residual-add LayerNorm + MLP in one kernel vs msu_layernorm_fwd (add mode)
    followed by the fused MLP: s bitwise (the same fma and rounding), y within rel. L2 2e-3 (the
    row statistics summed in a different order)."""
    ops = _ops()
    w1, b1, w2, b2 = _params(21, low)
    g = torch.Generator().manual_seed(22)
    B, R = 2, 97  # M = 18818 tokens: a ragged last tile
    x = torch.randn(B, R, R, 96, generator=g).to(DEV, low)
    a = torch.randn(B, R, R, 96, generator=g).to(DEV, low)
    lw = torch.nn.Parameter((1 + 0.1 * torch.randn(96, generator=g)).to(DEV))
    lb = torch.nn.Parameter((0.1 * torch.randn(96, generator=g)).to(DEV))
    sc = torch.tensor([1.25, 0.0], device=DEV) if with_scale else None
    with torch.no_grad(), torch.autocast("cuda", dtype=low):
        l0 = ops.add_ln_mlp_calls
        r = ops.add_layer_norm_mlp(x, a, sc, lw, lb, 1e-5, w1, b1, w2, b2)
        assert r is not None and ops.add_ln_mlp_calls == l0 + 1
        s_ref, xn = ops.add_layer_norm(x, a, sc, lw, lb, 1e-5)
        y_ref = ops.mlp(xn, w1, b1, w2, b2)
    torch.cuda.synchronize()
    s, y = r
    assert torch.equal(s, s_ref)
    rel = ((y.float() - y_ref.float()).norm() / y_ref.float().norm()).item()
    assert rel <= 2e-3, rel


def test_add_ln_mlp_not_under_autograd():
    ops = _ops()
    w1, b1, w2, b2 = _params(23, torch.bfloat16)
    x = torch.randn(2, 64, 64, 96, device=DEV, dtype=torch.bfloat16)
    lw = torch.nn.Parameter(torch.ones(96, device=DEV))
    lb = torch.nn.Parameter(torch.zeros(96, device=DEV))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert ops.add_layer_norm_mlp(x, x, None, lw, lb, 1e-5, w1, b1, w2, b2) is None
