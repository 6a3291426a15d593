"""GPU: the one-pass stage-0 Linear backward (csrc/gemm_linbwd.hip, msu_linear_bwd) against fp32
PyTorch, and the ops path that uses it against the two-kernel path.

Reference: fp32 products of the same 16-bit-rounded operands.  dX is rounded to 16 bits once
(tolerance as tests/test_gpu_tok_gemm.py: |y - ref| <= 1e-2 |ref| + 4e-3 max|ref|; the GELU'
epilogue uses the A&S erf); dW / db are f32 sums over up to 524 288 tokens in another order
(relative 1e-4 of the largest entry).  M = 524288 is the bench's stage 0 (8 x 256^2 tokens), where
every workgroup walks many 64- / 32-token steps.  Shapes: the block Linears of stage 0 (K x N = in x out:
qkv 96 x 288, proj 96 x 96, mlp.0 96 x 384, mlp.3 384 x 96 with and without the GELU' epilogue)
at a ragged M and above the ops threshold; both 16-bit formats.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
CASES = [(96, 288, False), (96, 96, False), (96, 384, False), (384, 96, False), (384, 96, True)]


def _gelu_grad(h):
    return 0.5 * (1.0 + torch.erf(h / math.sqrt(2.0))) + h * torch.exp(-0.5 * h * h) / math.sqrt(2.0 * math.pi)


def _check(y, ref, what, rel=1e-2, frac=4e-3):
    y = y.float()
    scale = ref.abs().max().item()
    err = (y - ref).abs() - rel * ref.abs()
    assert err.max().item() <= frac * scale, f"{what}: excess err {err.max().item():.3e} vs scale {scale:.3e}"


@pytest.fixture(params=[torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def low(request):
    return request.param


@pytest.mark.parametrize("K,N,gg", CASES)
@pytest.mark.parametrize("M", [1000, 65549, 524288])
def test_linear_bwd_matches_fp32(K, N, gg, M, low):
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    L = _lib.lib()
    assert L.msu_linear_bwd_supported(M, K, N) == 1
    g = torch.Generator().manual_seed(K + N + M + int(gg))
    dy = torch.randn(M, N, generator=g).to(DEV, low)
    x = torch.randn(M, K, generator=g).to(DEV, low)
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV, low)
    h = torch.randn(M, K, generator=g).to(DEV, low) if gg else None
    wt = w.t().contiguous()
    dx = torch.empty(M, K, device=DEV, dtype=low)
    dw0 = torch.randn(N, K, generator=g).to(DEV)  # accumulate = 1 adds to these
    db0 = torch.randn(N, generator=g).to(DEV)
    dw, db = dw0.clone(), db0.clone()
    ws = torch.empty(L.msu_linear_bwd_workspace(M, K, N), device=DEV)
    dt = 1 if low == torch.bfloat16 else 2
    _lib.call("msu_linear_bwd", dt, dy.data_ptr(), x.data_ptr(), wt.data_ptr(), None if h is None else h.data_ptr(),
              dx.data_ptr(), dw.data_ptr(), db.data_ptr(), ws.data_ptr(), M, K, N, 1,
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref_dx = dy.float() @ w.float()
    if gg:
        ref_dx = ref_dx * _gelu_grad(h.float())
    _check(dx, ref_dx, f"dX {M}x{K}x{N}")
    ref_dw = dy.float().t() @ x.float()
    ref_db = dy.float().sum(0)
    tol_w = 1e-4 * ref_dw.abs().max().item()
    assert (dw - dw0 - ref_dw).abs().max().item() <= tol_w
    assert (db - db0 - ref_db).abs().max().item() <= 1e-4 * ref_db.abs().max().item() + 1e-3


def _direct_params(*shapes, dtype=torch.bfloat16, seed=0):
    """Parameters set up the way the Trainer does (flat .grad, 16-bit shadow and transposed
    shadow, direct accumulation)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for shp in shapes:
        p = torch.nn.Parameter((torch.randn(*shp, generator=g) / math.sqrt(shp[-1])).to(DEV))
        p.grad = torch.zeros_like(p)
        p._msu_direct = True
        p._msu_shadow = p.detach().to(dtype)
        if p.dim() == 2:
            p._msu_shadow_t = p.detach().t().contiguous().to(dtype)
        p._msu_shadow_ver = p._version
        out.append(p)
    return out


def _grads(params):
    return [p.grad.clone() for p in params]


@pytest.mark.parametrize("amp", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("which", ["linear_qkv", "linear_proj", "mlp"])
def test_ops_one_pass_backward_equals_two_kernel_path(which, amp):
    """ops.linear / ops.mlp with trainer-style parameters: the one-pass backward (default) and the
    two-kernel path (input-gradient GEMM + side-stream weight gradient) give the same dX to
    16-bit rounding and the same dW / db to f32 summation order.  The trainer's shadows are bf16:
    under fp16 autocast the one-pass backward takes a per-call W^T of the f16 weight (it used to
    be skipped silently); ops.linbwd_calls shows which path ran."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    M = 8 * 128 * 128  # stage 0 at 512^2
    g = torch.Generator().manual_seed(7)
    outs = []
    for fused in (True, False):
        prev = ops._LINBWD
        ops._LINBWD = fused
        try:
            calls0 = ops.linbwd_calls
            x = torch.randn(M, 96, generator=g.manual_seed(7)).to(DEV, amp).requires_grad_(True)
            with torch.autocast("cuda", dtype=amp):
                if which == "mlp":
                    params = _direct_params((384, 96), (384,), (96, 384), (96,), seed=3)
                    y = ops.mlp(x, *params)
                else:
                    n = 288 if which == "linear_qkv" else 96
                    params = _direct_params((n, 96), (n,), seed=3)
                    y = ops.linear(x, *params)
            dy = torch.randn(y.shape, generator=g.manual_seed(9)).to(DEV, y.dtype)
            y.backward(dy)
            ops.join_side_streams()
            torch.cuda.synchronize()
            ran = ops.linbwd_calls - calls0
            assert ran == ((2 if which == "mlp" else 1) if fused else 0), (which, amp, fused, ran)
            outs.append((x.grad.float(), _grads(params)))
        finally:
            ops._LINBWD = prev
    (dx1, g1), (dx2, g2) = outs
    _check(dx1, dx2, f"{which} dX")
    for a, b in zip(g1, g2):
        assert (a - b).abs().max().item() <= 1e-4 * b.abs().max().item() + 1e-6
