"""GPU: the LayerNorm parameter-gradient partials summed inside the backward kernel (reduce.h
tail_reduce: the last block of each group of 32 partial rows sums its group, the last group sums
the groups, in a fixed order) against the separate colsum launch (msu_tail_reduce_mode(0)):

* dgamma / dbeta agree with the colsum path to f32 rounding (a different but fixed summation
  order) and with an f64 sum of the LayerNorm gradient definition; dx is untouched (bitwise);
* bitwise run-to-run determinism of the tail path;
* the per-stream counters are left at zero by every launch: many launches, on two streams at
  once, of different partial counts (1, 7, 100, 512, 1024 rows of partials) stay correct;
* a misaligned dgamma falls back to the colsum launch (result unchanged).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib():
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    return _lib.lib()


def _ops():
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    return ops


class _Mode:
    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        self.prev = _lib().msu_tail_reduce_mode(self.mode)

    def __exit__(self, *a):
        _lib().msu_tail_reduce_mode(self.prev)


def _case(rows, C, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(rows, C, generator=g).to(DEV, torch.bfloat16)
    dy = torch.randn(rows, C, generator=g).to(DEV, torch.bfloat16)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    b = (0.1 * torch.randn(C, generator=g)).to(DEV)
    return x, dy, w, b


def _run(x, dy, w, b):
    ops = _ops()
    wp = torch.nn.Parameter(w.clone())
    bp = torch.nn.Parameter(b.clone())
    xg = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.layer_norm(xg, wp, bp)
    y.backward(dy)
    return xg.grad, wp.grad, bp.grad


def _ref(x, dy):
    """f64 dgamma / dbeta of the LayerNorm definition."""
    xf, d = x.double(), dy.double()
    mu = xf.mean(-1, keepdim=True)
    var = xf.var(-1, unbiased=False, keepdim=True)
    xh = (xf - mu) / torch.sqrt(var + 1e-5)
    return (d * xh).sum(0), d.sum(0)


# rows -> partial rows (msu_ln_part_blocks: rows / 16, capped at 1024, 512 at C >= 384)
@pytest.mark.parametrize("rows,C", [(16, 96), (112, 96), (1600, 96), (65536, 96), (262144, 96),
                                    (8192, 384), (32768, 192), (2048, 768), (4000, 128)])
def test_tail_matches_colsum_and_f64(rows, C):
    x, dy, w, b = _case(rows, C, rows + C)
    with _Mode(1):
        dx1, dg1, db1 = _run(x, dy, w, b)
    with _Mode(0):
        dx0, dg0, db0 = _run(x, dy, w, b)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0)
    rg, rb = _ref(x, dy)
    for got, col, ref in ((dg1, dg0, rg), (db1, db0, rb)):
        scale = ref.abs().max().item() + 1.0
        assert (got - col).abs().max().item() <= 2e-5 * scale * max(1.0, rows / 4096) ** 0.5
        assert (got.double() - ref).abs().max().item() <= 1e-3 * scale


def test_tail_is_deterministic():
    x, dy, w, b = _case(262144, 96, 5)
    with _Mode(1):
        first = _run(x, dy, w, b)
        for _ in range(4):
            again = _run(x, dy, w, b)
            for a, r in zip(again, first):
                assert torch.equal(a, r)


def test_counters_stay_clean_across_streams_and_sizes():
    cases = [_case(r, C, i) for i, (r, C) in enumerate([(16, 96), (112, 96), (1600, 96), (8192, 384),
                                                        (262144, 96), (16384, 192)])]
    with _Mode(0):
        want = [_run(*c) for c in cases]
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    got = []
    with _Mode(1):
        for rep in range(6):
            outs = []
            for i, c in enumerate(cases):
                st = s1 if (i + rep) % 2 else s2
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    outs.append(_run(*c))
            torch.cuda.synchronize()
            got.append(outs)
    for outs in got:
        for o, wnt, c in zip(outs, want, cases):
            scale = wnt[1].abs().max().item() + 1.0
            assert torch.equal(o[0], wnt[0])
            for a, r in zip(o[1:], wnt[1:]):
                assert (a - r).abs().max().item() <= 2e-5 * scale * 8
    # same stream, same inputs: bitwise the same on every repetition
    for outs in got[2:]:
        for o, r in zip(outs, got[0]):
            assert all(torch.equal(a, b) for a, b in zip(o, r))


def test_misaligned_output_falls_back_to_colsum():
    """dgamma / dbeta as views 4 B into a buffer: not 16-B aligned, the colsum launch sums them."""
    ops = _ops()
    x, dy, w, b = _case(4096, 96, 17)
    res = {}
    for mode in (1, 0):
        with _Mode(mode):
            wp = torch.nn.Parameter(w.clone())
            bp = torch.nn.Parameter(b.clone())
            flat = torch.zeros(2 * 96 + 1, device=DEV)
            wp.grad = flat[1:97]
            bp.grad = flat[97:]
            wp._msu_direct = bp._msu_direct = True
            xg = x.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = ops.layer_norm(xg, wp, bp)
            y.backward(dy)
            ops.join_side_streams()
            torch.cuda.synchronize()
            res[mode] = (wp.grad.clone(), bp.grad.clone())
    assert torch.equal(res[1][0], res[0][0]) and torch.equal(res[1][1], res[0][1])

