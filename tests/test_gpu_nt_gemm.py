"""GPU: the tiled NT GEMM (csrc/gemm_nt.hip) against plain fp32 PyTorch, and its routing.

Reference: fp32 matmul of the same 16-bit-rounded operands, then the epilogue in fp32 (same
bar as the token GEMM's tests: one rounding of the f32 accumulator to bf16 / f16 and another
summation order -> |y - ref| <= 1e-2 |ref| + 4e-3 max|ref|).  Shapes: the Swin-T stage 1-3
Linears (forward and input gradient) at small M, plus ragged M (not a multiple of the 128-row
tile), N not a multiple of the 128-column tile (N % 32 == 0) and single-K-step K = 64.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
SHAPES = [(4096, 1152, 384), (4096, 384, 1152), (1000, 384, 384), (2048, 768, 192), (777, 192, 768),
          (300, 2304, 768), (128, 768, 3072), (513, 96, 64), (64, 160, 128), (1, 32, 64)]
# shapes that take the 256 x 128 tile (8 waves, three-stage ring: >= one tile per CU), incl. a
# ragged M, an N that is not a multiple of 128 and two-K-step tiles (vmcnt(0) fallback)
BIG = [(32768, 1152, 384), (32768, 384, 1536), (131072, 192, 768), (32000 + 77, 416, 192), (65536, 640, 128),
       (32000 + 77, 384, 192)]
# shapes the tile model puts on the 256 x 192 tile (two-stage ring; round 4): N = 384 / 1152 at
# the stage-2 token count, incl. a ragged M (BIG's 32768 x 1152, 32768 x 384, 32077 x 384 too)
WIDE = [(32768, 384, 384), (32768, 1152, 384), (32000 + 77, 384, 192), (131072, 576, 192)]


def _ops():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    return ops


@pytest.fixture(params=[17, 16, 0, 8], ids=["pingpong", "persistent", "static", "a3w2"], autouse=True)
def nt_mode(request):
    """Every test runs with each NT kernel form: the ping-pong one (gemm_pp.h, MSU_NT_PP=1 where the
    shape tiles exactly), the persistent 2-barrier one with its per-XCD tile queue (bit 4, the
    default) and with the static schedule, and the persistent kernel's 256 x 192 tile on the A3W2
    ring (msu_nt_gemm_mode bit 3: A two K steps ahead)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    prev = _lib.lib().msu_nt_gemm_mode(request.param)
    yield request.param
    _lib.lib().msu_nt_gemm_mode(prev)


@pytest.fixture(params=[torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def low(request):
    return request.param


def _check(y, ref, what):
    y = y.float()
    scale = ref.abs().max().item()
    err = (y - ref).abs() - 1e-2 * ref.abs()
    assert err.max().item() <= 4e-3 * scale, f"{what}: excess err {err.max().item():.3e} vs scale {scale:.3e}"


def _inputs(M, N, K, seed, low):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(M, K, generator=g).to(DEV, low)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV, low)
    b = torch.randn(N, generator=g).to(DEV)
    return a, w, b


@pytest.mark.parametrize("M,N,K", SHAPES + BIG)
@pytest.mark.parametrize("bias", [False, True])
def test_nt_gemm_plain(M, N, K, bias, low):
    ops = _ops()
    assert ops.nt_supported(M, N, K)
    a, w, b = _inputs(M, N, K, M + N + K, low)
    y = ops.nt_gemm(a, w, b if bias else None)
    ref = F.linear(a.float(), w.float(), b if bias else None)
    assert y.dtype == low and y.shape == (M, N)
    _check(y, ref, "y")


@pytest.mark.parametrize("M,N,K", [(4096, 1536, 384), (777, 768, 192), (300, 3072, 768), (32768, 1536, 384),
                                   (32768, 1152, 384), (32000 + 77, 384, 384)])
def test_nt_gemm_gelu_epilogues(M, N, K, low):
    """EPI 1: (H, GELU(H)) of mlp.0; EPI 2: (dY . W2) * GELU'(H) -- mlp.3's input gradient
    through the activation (W2^T [N, K'] passed as the weight)."""
    ops = _ops()
    a, w, b = _inputs(M, N, K, 7 * M + N, low)
    h, g = ops.nt_gemm(a, w, b, ops.TOK_GELU_DUAL)
    href = F.linear(a.float(), w.float(), b)
    _check(h, href, "h")
    _check(g, F.gelu(h.float()), "gelu(h)")
    gen = torch.Generator().manual_seed(M)
    dy = torch.randn(M, K, generator=gen).to(DEV, low)
    w2t = (torch.randn(N, K, generator=gen) / K ** 0.5).to(DEV, low)  # [Hd, C] = W2^T
    dh = ops.nt_gemm(dy, w2t, None, ops.TOK_GELU_GRAD, h=h)
    hf = h.float().requires_grad_(True)
    F.gelu(hf).backward(torch.ones_like(hf))
    ref = F.linear(dy.float(), w2t.float()) * hf.grad
    _check(dh, ref, "dh")


@pytest.mark.parametrize("M,N,K", SHAPES + BIG)
def test_nt_gemm_kn_plain(M, N, K, low):
    """msu_nt_gemm_kn: Y = A . Wk with Wk [K, N] read in place (a Linear's input gradient dX = dY . W
    with its forward weight W); same bar as the [N, K] form."""
    ops = _ops()
    a, w, _ = _inputs(M, N, K, 3 * M + N + K, low)
    wk = w.t().contiguous()  # [K, N]
    y = ops.nt_gemm_kn(a, wk)
    assert y.dtype == low and y.shape == (M, N)
    _check(y, a.float() @ wk.float(), "y")


@pytest.mark.parametrize("M,N,K", [(4096, 1536, 384), (777, 768, 192), (300, 3072, 768), (32768, 1536, 384)])
def test_nt_gemm_kn_gelu_grad(M, N, K, low):
    """EPI 2 with the weight in place: dH = (dY . W2) * GELU'(H), W2 [K, N] = mlp.3's weight."""
    ops = _ops()
    gen = torch.Generator().manual_seed(M + 1)
    dy = torch.randn(M, K, generator=gen).to(DEV, low)
    w2 = (torch.randn(K, N, generator=gen) / K ** 0.5).to(DEV, low)
    h = torch.randn(M, N, generator=gen).to(DEV, low)
    dh = ops.nt_gemm_kn(dy, w2, ops.TOK_GELU_GRAD, h=h)
    hf = h.float().requires_grad_(True)
    F.gelu(hf).backward(torch.ones_like(hf))
    _check(dh, (dy.float() @ w2.float()) * hf.grad, "dh")


@pytest.mark.parametrize("M,N,K", WIDE)
def test_nt_gemm_wide_tile_is_chosen_and_exact(M, N, K, nt_mode):
    """The shapes the round-4 tile model sends to the 192-column tile (a launch with that tile is
    told apart by the whole-round tile count; msu_nt_gemm_plan reports the choice), bias epilogue;
    with the ping-pong kernel where it tiles exactly (N % 192, M % 256), the 2-barrier one else."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    ops = _ops()
    wm, bn, pp = _lib.plan_nt(M, N)
    assert bn == 192, (M, N, wm, bn)
    assert pp == (bool(nt_mode & 1) and M % 256 == 0), (M, N, pp)
    a, w, b = _inputs(M, N, K, 11 * M + N, torch.bfloat16)
    y = ops.nt_gemm(a, w, b)
    _check(y, F.linear(a.float(), w.float(), b), "y")


@pytest.mark.parametrize("M,N,K", [(8192, 768, 3072), (8192, 768, 768), (8192 - 5, 576, 256)])
def test_nt_gemm_underfilled_shape_takes_all_cus(M, N, K):
    """Stage-3 shapes whose 256-row tiles would leave CUs idle (tiles < CUs) go to 128-row
    tiles, one per CU (r04h: 59 vs 65-75 us at 8192 x 768 x 3072); the result is unchanged."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    ops = _ops()
    rows, cols, pp = _lib.plan_nt(M, N)
    assert rows == 128 and cols == 192 and not pp, (M, N, rows, cols, pp)
    a, w, b = _inputs(M, N, K, 5 * M + N, torch.bfloat16)
    y = ops.nt_gemm(a, w, b)
    _check(y, F.linear(a.float(), w.float(), b), "y")


# every stage 1-3 shape of the Swin-T 8 x 1024^2 step the ping-pong kernel takes (forward and input
# gradient, both tile widths), the three epilogues and the skip concatenation's split A
PP = [(131072, 576, 192), (131072, 192, 192), (131072, 768, 192), (131072, 192, 768), (131072, 384, 192),
      (32768, 1152, 384), (32768, 384, 384), (32768, 1536, 384), (32768, 384, 1536), (32768, 768, 384),
      (32768, 384, 768)]


@pytest.mark.parametrize("M,N,K", PP)
def test_nt_gemm_production_shapes(M, N, K, nt_mode, low):
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    ops = _ops()
    _, bn, pp = _lib.plan_nt(M, N)
    if nt_mode & 1:
        assert pp, (M, N)
    a, w, b = _inputs(M, N, K, 13 * M + N + K, low)
    y = ops.nt_gemm(a, w, b)
    _check(y, F.linear(a.float(), w.float(), b), "y")
    if N % 192 == 0 or N % 256 == 0:
        h, g = ops.nt_gemm(a, w, b, ops.TOK_GELU_DUAL)
        _check(h, F.linear(a.float(), w.float(), b), "h")
        _check(g, F.gelu(h.float()), "gelu(h)")
        hf = h.float().requires_grad_(True)
        F.gelu(hf).backward(torch.ones_like(hf))
        dh = ops.nt_gemm(a, w, None, ops.TOK_GELU_GRAD, h=h)
        _check(dh, F.linear(a.float(), w.float()) * hf.grad, "dh")
    if K % 128 == 0:  # [x | skip] . W^T with K1 = K / 2 (concat_back_dim)
        K1 = K // 2
        y2 = ops.nt_gemm_cat(a[:, :K1].contiguous(), a[:, K1:].contiguous(), w, b)
        _check(y2, F.linear(a.float(), w.float(), b), "cat")


def test_nt_gemm_pingpong_matches_persistent():
    """Both kernels on the same operands agree to rounding (different summation order only)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    ops = _ops()
    a, w, b = _inputs(32768, 1152, 384, 5, torch.bfloat16)
    prev = _lib.lib().msu_nt_gemm_mode(1)
    y1 = ops.nt_gemm(a, w, b)
    _lib.lib().msu_nt_gemm_mode(0)
    y0 = ops.nt_gemm(a, w, b)
    _lib.lib().msu_nt_gemm_mode(prev)
    d = (y1.float() - y0.float()).abs().max().item()
    assert d <= 2e-2 * y0.float().abs().max().item(), d


def test_nt_gemm_rejects_uncovered_shapes():
    ops = _ops()
    assert not ops.nt_supported(4096, 100, 384)  # N % 32
    assert not ops.nt_supported(4096, 384, 96)   # K % 64
    a = torch.zeros(64, 96, device=DEV, dtype=torch.bfloat16)
    w = torch.zeros(64, 96, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.nt_gemm(a, w)


@pytest.mark.parametrize("M,N,K", [(32768, 1152, 384), (8192, 768, 3072), (131072, 192, 384)])
def test_linear_routes_stage_shapes_to_nt_and_matches(M, N, K, monkeypatch):
    """ops.linear at stage 1-3 shapes (bf16 autocast) with the NT GEMM routed in
    (MSU_GEMM_ROUTE=nt): forward and input gradient on the NT GEMM (the input gradient reads the
    weight in place, msu_nt_gemm_kn), weight gradient on the HIP wgrad kernel; all against fp32
    autograd."""
    ops = _ops()
    monkeypatch.setattr(ops, "_ROUTE_FORCE", "nt")
    monkeypatch.setattr(ops, "_tok_cache", {})
    assert ops.gemm_route(M, N, K) == "nt" and ops.gemm_route(M, K, N) == "nt"
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g)
    xr = x.bfloat16().float().requires_grad_(True)
    wr = w.bfloat16().float()
    yr = F.linear(xr, wr, b)
    yr.backward(dy.bfloat16().float())
    xg = x.to(DEV, torch.bfloat16).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    bg = b.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.linear(xg, wg, bg)
    y.backward(dy.to(DEV, torch.bfloat16))
    _check(y, yr.detach().to(DEV), "y")
    _check(xg.grad, xr.grad.to(DEV), "dx")
    gw = wg.grad.float().cpu()
    wref = dy.bfloat16().float().t() @ xr.detach()
    assert ((gw - wref).norm() / wref.norm()).item() < 1e-2


@pytest.mark.parametrize("M,N,K", [(32768, 384, 384), (131072, 576, 192), (32000 + 77, 384, 192), (8192, 2304, 768)])
def test_tile_queue_equals_static(M, N, K, nt_mode):
    """The two-stage kernel's per-XCD tile queue against its static schedule: bit-identical
    outputs (plain, GELU dual, GELU' epilogues) over repeated launches (the slot resets itself)
    and on a second stream (its own slot).  Grids of 256 (or 512) workgroups over >= 2 tiles each."""
    if nt_mode != 16:
        pytest.skip("queue vs static: one run")
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    ops = _ops()
    a, w, b = _inputs(M, N, K, M + N, torch.bfloat16)
    h = torch.randn(M, N, generator=torch.Generator().manual_seed(5)).to(DEV, torch.bfloat16)

    def run():
        return (ops.nt_gemm(a, w, b, 0), ops.nt_gemm(a, w, b, 1), ops.nt_gemm(a, w, None, 2, h=h))

    L = _lib.lib()
    L.msu_nt_gemm_mode(0)
    ref = run()
    L.msu_nt_gemm_mode(16)
    outs = [run() for _ in range(3)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        outs.append(run())
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    def flat(o):
        return [o[0], *o[1], o[2]]  # y (plain), (H, GELU(H)) (dual), y (GELU')

    for o in outs:
        for u, r in zip(flat(o), flat(ref)):
            assert torch.equal(u, r)
