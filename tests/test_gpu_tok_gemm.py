"""GPU: the token GEMM (csrc/gemm_tok.h) and the fused MLP against plain fp32 PyTorch.

Reference: fp32 matmul of the same 16-bit-rounded operands, then the epilogue in fp32.
Tolerance: the kernel rounds its f32 accumulator to bf16 / f16 once (<= 2^-8 relative) and sums
in a different order, so |y - ref| <= 1e-2 * |ref| + 4e-3 * max|ref| (bf16 storage, 8 significant
bits; f16's 11 bits sit well inside); GELU uses the A&S 7.1.26 erf (|err| <= 1.5e-7).
Every test runs for both 16-bit formats (bf16 training mode, f16 = the reference's autocast).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    return ops


def _check(y, ref, what):
    y = y.float()
    scale = ref.abs().max().item()
    err = (y - ref).abs() - 1e-2 * ref.abs()
    assert err.max().item() <= 4e-3 * scale, f"{what}: excess err {err.max().item():.3e} vs scale {scale:.3e}"


@pytest.fixture(params=[torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def low(request):
    return request.param


def _inputs(M, N, K, seed, low=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(M, K, generator=g).to(DEV, low)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, low)
    b = torch.randn(N, generator=g).to(DEV)
    return a, w, b


# (M, N, K): Swin-T stage shapes at small M plus ragged M, multi-chunk N and multi-stage K
SHAPES = [(1000, 288, 96), (4096, 384, 96), (4096, 96, 384), (2048, 192, 768), (777, 96, 48),
          (4096, 576, 192), (1024, 1152, 384), (300, 128, 128), (512, 512, 128), (33, 96, 96),
          (2048, 1536, 96), (64, 768, 3072)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("bias", [False, True])
def test_tok_gemm_plain(M, N, K, bias, low):
    ops = _ops()
    if not ops.tok_supported(M, N, K):
        pytest.skip("shape not covered by the token GEMM plan")
    a, w, b = _inputs(M, N, K, M + N + K, low)
    y = ops.tok_gemm(a, w, b if bias else None)
    ref = a.float() @ w.float().t() + (b if bias else 0)
    _check(y, ref, f"plain {M}x{N}x{K}")


def test_tok_gemm_plan_covers_stage0():
    """Every stage-0 (the HBM-bound bulk) Swin-T 1024^2 bs8 Linear, forward and input
    gradient, has a plan; wider-K shapes of deeper stages may go to the library GEMM."""
    ops = _ops()
    T, C = 8 * 256 ** 2, 96
    need = [(T, 3 * C, C), (T, C, C), (T, 4 * C, C), (T, C, 4 * C), (T, C, 3 * C),
            (T // 4, 2 * C, 4 * C), (T // 4, 4 * C, 2 * C), (T, C, 2 * C), (T, 2 * C, C),
            (T, 96, 48), (T, 1536, 96)]
    missing = [s for s in need if not ops.tok_supported(*s)]
    assert not missing, missing


@pytest.mark.parametrize("M,C,K1", [(1000, 96, 96), (2048, 192, 192), (333, 128, 128)])
def test_tok_gemm_concat(M, C, K1, low):
    """torch.cat([x, skip], -1) -> Linear(2C, C) without the cat (model_parts.py:792-794)."""
    ops = _ops()
    if not ops.tok_supported(M, C, 2 * K1):
        pytest.skip("shape not covered by the token GEMM plan")
    a, w, b = _inputs(M, C, 2 * K1, 7, low)
    x, skip = a[:, :K1].contiguous(), a[:, K1:].contiguous()
    y = ops.tok_gemm(x, w, b, a2=skip)
    ref = a.float() @ w.float().t() + b
    _check(y, ref, "concat")


@pytest.mark.parametrize("M,N,K", [(1000, 384, 96), (4096, 768, 192), (555, 1536, 384)])
def test_tok_gemm_gelu_dual_and_grad(M, N, K, low):
    ops = _ops()
    if not ops.tok_supported(M, N, K):
        pytest.skip("shape not covered by the token GEMM plan")
    a, w, b = _inputs(M, N, K, 11, low)
    h, g = ops.tok_gemm(a, w, b, ops.TOK_GELU_DUAL)
    ref_h = a.float() @ w.float().t() + b
    _check(h, ref_h, "H")
    _check(g, F.gelu(h.float()), "GELU(H)")
    # epi 2: (dY . W2) * GELU'(H) with dY [M, K'] and W2^T [N, K']
    g2 = torch.Generator().manual_seed(5)
    dy = torch.randn(M, K, generator=g2).to(DEV, low)
    w2t = (torch.randn(N, K, generator=g2) / K ** 0.5).to(DEV, low)
    dh = ops.tok_gemm(dy, w2t, None, ops.TOK_GELU_GRAD, h=h)
    hf = h.float().requires_grad_(True)
    F.gelu(hf).backward(torch.ones_like(hf))
    ref = (dy.float() @ w2t.float().t()) * hf.grad
    _check(dh, ref, "dH")


@pytest.mark.parametrize("M,C", [(4096, 96), (1000, 96), (512, 128)])
def test_fused_mlp_matches_fp32(M, C, low):
    """ops.mlp (mlp.0 -> GELU -> mlp.3) forward and all gradients vs fp32 autograd."""
    ops = _ops()
    g = torch.Generator().manual_seed(M + C)
    x = torch.randn(M, C, generator=g)
    w1 = torch.randn(4 * C, C, generator=g) / C ** 0.5
    b1 = 0.1 * torch.randn(4 * C, generator=g)
    w2 = torch.randn(C, 4 * C, generator=g) / (4 * C) ** 0.5
    b2 = 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(M, C, generator=g)
    # fp32 reference on the 16-bit-rounded input
    xr = x.to(low).float().requires_grad_(True)
    pr = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
    yr = F.linear(F.gelu(F.linear(xr, pr[0], pr[1])), pr[2], pr[3])
    yr.backward(dy.to(low).float())
    xg = x.to(DEV, low).requires_grad_(True)
    pg = [t.to(DEV).requires_grad_(True) for t in (w1, b1, w2, b2)]
    with torch.autocast("cuda", dtype=low):
        assert ops.mlp_fusable(xg, pg[0], pg[2])
        y = ops.mlp(xg, *pg)
    y.backward(dy.to(DEV, low))
    _check(y, yr.to(DEV), "y")
    # gradients: bf16 intermediates (H, G, dH) -> 3e-2 of the largest entry
    for name, a, r in [("dx", xg.grad, xr.grad), ("dw1", pg[0].grad, pr[0].grad), ("db1", pg[1].grad, pr[1].grad),
                       ("dw2", pg[2].grad, pr[2].grad), ("db2", pg[3].grad, pr[3].grad)]:
        err = (a.float().cpu() - r).abs().max().item()
        assert err <= 3e-2 * r.abs().max().item(), f"{name}: {err:.3e} vs {r.abs().max().item():.3e}"


@pytest.mark.parametrize("route", ["default", "nt"])
@pytest.mark.parametrize("M,C", [(4096, 96), (1000, 96), (2048, 192), (1000, 384)])
def test_mlp_no_grad_keeps_nothing_and_equals_grad_path(M, C, route, monkeypatch, low):
    """Under no_grad (the reference's discarded branches) ops.mlp keeps neither H nor G.  At
    C = 96 / 192 it runs the fused inference MLP (csrc/mlp_fused.hip, mlp_s1.hip: same roundings of H and GELU(H),
    biases added in f32 rather than as a hi / lo k-block): within rel. L2 2e-3 of the grad path.
    Elsewhere the GELU store overwrites the pre-activation in one buffer and the output is
    bitwise the grad path's (same kernels, same rounding of H before GELU)."""
    ops = _ops()
    if route == "nt":
        monkeypatch.setattr(ops, "_ROUTE_FORCE", "nt")
        monkeypatch.setattr(ops, "_tok_cache", {})
    g = torch.Generator().manual_seed(M + 7 * C)
    x = torch.randn(M, C, generator=g).to(DEV, low)
    w1 = (torch.randn(4 * C, C, generator=g) / C ** 0.5).to(DEV)
    b1 = (0.1 * torch.randn(4 * C, generator=g)).to(DEV)
    w2 = (torch.randn(C, 4 * C, generator=g) / (4 * C) ** 0.5).to(DEV)
    b2 = (0.1 * torch.randn(C, generator=g)).to(DEV)
    n0 = ops.mlp_infer_calls
    with torch.autocast("cuda", dtype=low):
        with torch.no_grad():
            y0 = ops.mlp(x, w1, b1, w2, b2)
            _, h, gg = torch.ops.msunet.mlp(x, w1, b1, w2, b2, False)
        y1, h1, g1 = torch.ops.msunet.mlp(x, w1, b1, w2, b2, True)
    torch.cuda.synchronize()
    assert h.numel() == 0 and gg.numel() == 0 and h1.shape == (M, 4 * C)
    if (C, 4 * C) in ops.MLP_FUSED_SHAPES and ops._MLP_INFER:
        assert ops.mlp_infer_calls == n0 + 2
        rel = ((y0.float() - y1.float()).norm() / y1.float().norm()).item()
        assert rel <= 2e-3, rel
    else:
        assert ops.mlp_infer_calls == n0
        assert torch.equal(y0, y1)


@pytest.mark.parametrize("M,C", [(1024, 384), (2048, 192), (1000, 768)])
def test_fused_mlp_mixed_routing(M, C, monkeypatch, low):
    """Stage-1/2/3 widths with the NT GEMM routed in (MSU_GEMM_ROUTE=nt): the GELU-epilogue
    GEMMs on the tiled NT GEMM, the other two on whichever GEMM is routed -- same numerics bar
    as the all-token-GEMM MLP."""
    ops = _ops()
    monkeypatch.setattr(ops, "_ROUTE_FORCE", "nt")
    monkeypatch.setattr(ops, "_tok_cache", {})
    assert ops.gemm_route(M, 4 * C, C, ops.TOK_GELU_DUAL) == "nt"
    assert ops.gemm_route(M, 4 * C, C, ops.TOK_GELU_GRAD) == "nt"
    test_fused_mlp_matches_fp32(M, C, low)


def test_linear_uses_tok_gemm_and_matches(low):
    """ops.linear in bf16 routes through the token GEMM for covered shapes (fwd + dgrad)."""
    ops = _ops()
    M, N, K = 2048, 288, 96
    assert ops.tok_supported(M, N, K) and ops.tok_supported(M, K, N)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g)
    xr = x.to(low).float().requires_grad_(True)
    yr = F.linear(xr, w.to(low).float(), b)
    yr.backward(dy.to(low).float())
    xg = x.to(DEV, low).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    bg = b.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=low):
        y = ops.linear(xg, wg, bg)
    y.backward(dy.to(DEV, low))
    _check(y, yr.to(DEV), "y")
    _check(xg.grad, xr.grad.to(DEV), "dx")


@pytest.mark.parametrize("M,C", [(4096, 96), (1000, 192), (2048, 384), (32768, 384)])
def test_linear_cat_matches_cat_then_linear(M, C, low):
    """ops.linear_cat (skip fusion without the concatenated copy) == Linear(cat([x, skip])):
    forward and all gradients, bf16 (model_parts.py:792-794).  C = 96 / 192 take the token
    GEMM's split-A loads, C = 384 (concat_back_dim[1] at stage 2) the NT GEMM's."""
    ops = _ops()
    assert ops._cat_route(M, C, 2 * C, C) == ("nt" if C == 384 else "tok")
    g = torch.Generator().manual_seed(M + C)
    x = torch.randn(M, C, generator=g)
    sk = torch.randn(M, C, generator=g)
    w = torch.randn(C, 2 * C, generator=g) / (2 * C) ** 0.5
    b = torch.randn(C, generator=g)
    dy = torch.randn(M, C, generator=g)
    xr, sr = x.to(low).float().requires_grad_(True), sk.to(low).float().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.linear(torch.cat([xr, sr], -1), wr.to(low).float(), br)
    yr.backward(dy.to(low).float())
    xg = x.to(DEV, low).requires_grad_(True)
    sg = sk.to(DEV, low).requires_grad_(True)
    wg, bg = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=low):
        y = ops.linear_cat(xg, sg, wg, bg)
    y.backward(dy.to(DEV, low))
    _check(y, yr.to(DEV), "y")
    _check(xg.grad, xr.grad.to(DEV), "dx")
    _check(sg.grad, sr.grad.to(DEV), "dskip")
    for name, a, r in [("dw", wg.grad, wr.grad), ("db", bg.grad, br.grad)]:
        err = (a.float().cpu() - r).abs().max().item()
        assert err <= 2e-2 * r.abs().max().item(), f"{name}: {err:.3e}"


# ----------------------------------------------------------------------------- production M
# The benchmarked step (Swin-T, 8 x 1024^2) runs these GEMMs at M = 8 * 256^2 = 524288 stage-0
# tokens (131072 at stage 1).  Same fp32 reference and tolerance as above, at full size
# (the small-M tests alone do not pin the benchmarked path).
T0 = 8 * 256 ** 2
PROD = [(T0, 288, 96), (T0, 96, 96), (T0, 384, 96), (T0, 96, 384), (T0, 96, 288), (T0 // 4, 576, 192),
        (T0 // 4, 192, 576), (T0 // 4, 192, 384), (T0, 96, 48), (T0, 96, 192)]


@pytest.fixture(autouse=False)
def strict_fp32():
    prev = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False
    yield
    torch.backends.cuda.matmul.allow_tf32 = prev


@pytest.mark.parametrize("M,N,K", PROD)
def test_tok_gemm_production_M(M, N, K, strict_fp32):
    """Plain + bias epilogue at the benchmark's token counts (forward shapes and the input
    gradients' [M, N] x [N, K] shapes: qkv, proj, fc1, fc2, merge reduction, patch embed, skip)."""
    ops = _ops()
    assert ops.tok_supported(M, N, K), (M, N, K)
    a, w, b = _inputs(M, N, K, N + K, torch.bfloat16)
    y = ops.tok_gemm(a, w, b)
    ref = torch.addmm(b, a.float(), w.float().t())
    _check(y, ref, f"plain {M}x{N}x{K}")


def test_tok_gemm_gelu_epilogues_production_M(strict_fp32):
    """mlp.0's GELU dual epilogue (H, GELU(H)) and mlp.3's GELU' input-gradient epilogue at
    M = 524288 (stage-0 fc1 / fc2, model_parts.py:143-151 via torchvision's MLP)."""
    ops = _ops()
    M, N, K = T0, 384, 96
    a, w, b = _inputs(M, N, K, 31, torch.bfloat16)
    h, g = ops.tok_gemm(a, w, b, ops.TOK_GELU_DUAL)
    ref_h = torch.addmm(b, a.float(), w.float().t())
    _check(h, ref_h, "H")
    del ref_h
    _check(g, F.gelu(h.float()), "GELU(H)")
    g2 = torch.Generator().manual_seed(6)
    dy = torch.randn(M, K, generator=g2).to(DEV, torch.bfloat16)
    w2t = (torch.randn(N, K, generator=g2) / K ** 0.5).to(DEV, torch.bfloat16)
    dh = ops.tok_gemm(dy, w2t, None, ops.TOK_GELU_GRAD, h=h)
    hf = h.float()
    # d/dh GELU(h) = Phi(h) + h * phi(h)
    gp = 0.5 * (1 + torch.erf(hf / 2 ** 0.5)) + hf * torch.exp(-0.5 * hf * hf) / (2 * torch.pi) ** 0.5
    ref = (dy.float() @ w2t.float().t()) * gp
    _check(dh, ref, "dH")


def test_linear_cat_production_M(strict_fp32):
    """Skip fusion at stage 0 (concat_back_dim[3]: [x | skip] 2x96 -> 96 over 524288 tokens):
    forward, both input gradients, weight and bias gradients vs fp32 autograd."""
    test_linear_cat_matches_cat_then_linear(T0, 96, torch.bfloat16)


def test_fused_mlp_production_M(strict_fp32):
    """The stage-0 fused MLP (fc1 GELU dual -> fc2; backward: fc2 wgrad, GELU' dgrad, fc1 wgrad
    and dgrad) at M = 524288 and the stage-1 one at 131072 vs fp32 autograd."""
    test_fused_mlp_matches_fp32(T0, 96, torch.bfloat16)
    test_fused_mlp_matches_fp32(T0 // 4, 192, torch.bfloat16)


@pytest.mark.parametrize("M,C", [(4096, 96), (32768, 384)])
def test_linear_cat_direct_grad_accumulates(M, C):
    """Trainer-style parameters (flat .grad, _msu_direct): linear_cat's two weight-gradient halves
    accumulate straight into the column slices of weight.grad (msu_linear_wgrad_ld, row stride
    2C) and the bias gradient into bias.grad -- no temporaries, no torch adds; the result equals
    the preset .grad plus the fp32 gradient of Linear(cat([x, skip]))."""
    ops = _ops()
    low = torch.bfloat16
    g = torch.Generator().manual_seed(M + 3 * C)
    x = torch.randn(M, C, generator=g).to(DEV, low)
    sk = torch.randn(M, C, generator=g).to(DEV, low)
    w = (torch.randn(C, 2 * C, generator=g) / (2 * C) ** 0.5).to(DEV)
    b = torch.randn(C, generator=g).to(DEV)
    dy = torch.randn(M, C, generator=g).to(DEV, low)
    wp, bp = torch.nn.Parameter(w.clone()), torch.nn.Parameter(b.clone())
    w0 = torch.randn(C, 2 * C, generator=g).to(DEV)
    b0 = torch.randn(C, generator=g).to(DEV)
    wp.grad, bp.grad = w0.clone(), b0.clone()
    wp._msu_direct = bp._msu_direct = True
    with torch.autocast("cuda", dtype=low):
        y = ops.linear_cat(x, sk, wp, bp)
    y.backward(dy)
    ops.join_side_streams()
    torch.cuda.synchronize()
    ref_w = dy.float().t() @ torch.cat([x, sk], -1).float()
    ref_b = dy.float().sum(0)
    assert (wp.grad - w0 - ref_w).abs().max().item() <= 1e-4 * ref_w.abs().max().item()
    assert (bp.grad - b0 - ref_b).abs().max().item() <= 1e-4 * ref_b.abs().max().item() + 1e-3
