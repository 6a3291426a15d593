"""Per-op microbenchmarks at the Swin-T 1024^2 bs=8 training shapes (bf16).

    python tools/kbench.py [attn|wgrad|conv|ln|all]

Times each HIP op with HIP events on the current stream (median of N launches) and prints
achieved GB/s or TFLOP/s next to the algorithmic work.  Used to pick what to optimise.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from semantic_segmentation_of_stylegan2_artifacts_amd import ops  # noqa: E402

DEV = "cuda"
B = 8


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def attn():
    for stage, (res, nh) in enumerate([(256, 3), (128, 6), (64, 12), (32, 24)]):
        C = 32 * nh
        qkv = torch.randn(B, res, res, 3 * C, device=DEV, dtype=torch.bfloat16)
        qb = torch.randn(3 * C, device=DEV)
        tb = torch.randn(169, nh, device=DEV)
        nwin = B * ((res + 6) // 7) ** 2
        byts = B * res * res * (3 * C + C) * 2
        for p in (0.0, 0.05):
            for shift in (0, 3):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    f = lambda: ops.window_attention(qkv, qb, tb, nh, shift, p, 1)
                    ms = timeit(f)
                    q = qkv.clone().requires_grad_(True)
                    y = ops.window_attention(q, qb, tb, nh, shift, p, 1)
                    dy = torch.randn_like(y)

                    def bw():
                        torch.autograd.grad(y, q, dy, retain_graph=True)
                    msb = timeit(bw)
                print(f"attn stage{stage} res{res} nh{nh} p={p} shift={shift}: fwd {ms*1e3:7.1f} us "
                      f"({byts/ms/1e6:6.0f} GB/s, {nwin*nh/ms/1e3:6.1f} Mitem/s)  bwd {msb*1e3:7.1f} us")


def stream():
    """Reference streaming rates: torch copy / sum of a 512 MB bf16 tensor."""
    x = torch.randn(256 << 20, device=DEV, dtype=torch.bfloat16)
    y = torch.empty_like(x)
    ms = timeit(lambda: y.copy_(x))
    print(f"copy 512 MB: {ms*1e3:7.1f} us  {2 * x.numel() * 2 / ms / 1e6:6.0f} GB/s (read+write)")
    ms = timeit(lambda: x.sum())
    print(f"sum  512 MB: {ms*1e3:7.1f} us  {x.numel() * 2 / ms / 1e6:6.0f} GB/s (read)")


def wgrad():
    from semantic_segmentation_of_stylegan2_artifacts_amd import _lib
    shapes = [(B * 65536, 288, 96), (B * 65536, 96, 96), (B * 65536, 384, 96), (B * 65536, 96, 384),
              (B * 65536, 1536, 96), (B * 16384, 576, 192), (B * 16384, 768, 192), (B * 16384, 192, 768),
              (B * 16384, 192, 192), (B * 4096, 1152, 384), (B * 4096, 384, 384), (B * 4096, 1536, 384),
              (B * 4096, 384, 1536), (B * 1024, 2304, 768), (B * 1024, 768, 768), (B * 1024, 3072, 768),
              (B * 1024, 768, 3072)]
    only = os.environ.get("KB_STAGE")
    if only:
        shapes = [s for s in shapes if s[0] == B * {"0": 65536, "1": 16384, "2": 4096, "3": 1024}[only]]
    for M, N, K in shapes:
        dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
        x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        L = _lib.lib()
        ws = torch.empty(L.msu_wgrad_workspace(M, N, K), device=DEV)
        dw = torch.empty(N, K, device=DEV)
        db = torch.empty(N, device=DEV)
        s = torch.cuda.current_stream().cuda_stream
        f = lambda: _lib.call("msu_linear_wgrad", 1, dy.data_ptr(), x.data_ptr(), dw.data_ptr(), db.data_ptr(),
                              ws.data_ptr(), M, N, K, 0, s)
        ms = timeit(f)
        fl = 2.0 * M * N * K
        byts = M * (N + K) * 2
        mt = timeit(lambda: dy.t().matmul(x))
        print(f"wgrad M={M:8d} N={N:5d} K={K:5d}: {ms*1e3:7.1f} us {fl/ms/1e9:7.1f} TF/s "
              f"{byts/ms/1e6:6.0f} GB/s (min bytes)   hipBLASLt dY^T X {mt*1e3:7.1f} us")


def conv():
    """The MS-UNet head as the model runs it: refine_conv_act (activations precomputed by the
    producers), conv1 from the pre-d2s expand output with the dual epilogue, conv2 plain."""
    C, H = 96, 1024
    e = torch.randn(B, H // 4, H // 4, 16 * C, device=DEV, dtype=torch.bfloat16)
    a0 = torch.nn.functional.gelu(e)
    z1 = torch.randn(B, H, H, C, device=DEV, dtype=torch.bfloat16)
    a1 = torch.nn.functional.gelu(z1)
    w = torch.randn(C, C, 3, 3, device=DEV) * 0.03
    b = torch.randn(C, device=DEV)
    fl = 2.0 * B * H * H * C * C * 9
    with torch.autocast("cuda", dtype=torch.bfloat16):
        for name, x, a, d2s in (("conv1(d2s,dual)", e, a0, True), ("conv2", z1, a1, False)):
            ms = timeit(lambda: ops.refine_conv_act(x, a, w, b, d2s, (H, H), dual=d2s), 5)
            q = x.clone().requires_grad_(True)
            wq = w.clone().requires_grad_(True)
            z = ops.refine_conv_act(q, a, wq, b, d2s, (H, H), dual=d2s)
            z = z[0] if d2s else z
            dz = torch.randn_like(z)
            msb = timeit(lambda: torch.autograd.grad(z, (q, wq), dz, retain_graph=True), 5)
            print(f"{name}: fwd {ms:.3f} ms ({fl/ms/1e9:.0f} TF/s)  bwd(dgrad+wgrad) {msb:.3f} ms ({2*fl/msb/1e9:.0f} TF/s)")


def ln():
    for rows, C in ((B * 65536, 96), (B * 16384, 192), (B * 4096, 384), (B * 1048576, 96)):
        x = torch.randn(rows, C, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(C, device=DEV)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ms = timeit(lambda: ops.layer_norm(x, w, w))
            q = x.clone().requires_grad_(True)
            y = ops.layer_norm(q, w, w)
            dy = torch.randn_like(y)
            msb = timeit(lambda: torch.autograd.grad(y, q, dy, retain_graph=True))
        print(f"LN rows={rows} C={C}: fwd {ms*1e3:.1f} us ({2*rows*C*2/ms/1e6:.0f} GB/s) "
              f"bwd {msb*1e3:.1f} us ({3*rows*C*2/msb/1e6:.0f} GB/s)")


def lnadd():
    """Residual add + LN (the Swin block's norm2 / next norm1) backward with both output
    gradients, as the block runs it: dres = the residual stream's gradient."""
    for rows, C in ((B * 65536, 96), (B * 16384, 192), (B * 4096, 384)):
        a = torch.randn(rows, C, device=DEV, dtype=torch.bfloat16).requires_grad_(True)
        b = torch.randn(rows, C, device=DEV, dtype=torch.bfloat16).requires_grad_(True)
        w = torch.randn(C, device=DEV)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            s, y = ops.add_layer_norm(a, b, None, w, w)
        dy, ds = torch.randn_like(y), torch.randn_like(s)
        msb = timeit(lambda: torch.autograd.grad([y, s], [a, b], [dy, ds], retain_graph=True))
        print(f"LN+add rows={rows} C={C}: bwd {msb*1e3:.1f} us ({5*rows*C*2/msb/1e6:.0f} GB/s)", flush=True)


def tok():
    """Token GEMM vs hipBLASLt (F.linear) at the Swin-T 1024^2 bs8 shapes."""
    shapes = [(B * 65536, 288, 96), (B * 65536, 96, 96), (B * 65536, 384, 96), (B * 65536, 96, 384),
              (B * 65536, 96, 192), (B * 65536, 1536, 96), (B * 65536, 96, 48), (B * 16384, 192, 384),
              (B * 16384, 576, 192), (B * 16384, 192, 192), (B * 16384, 768, 192), (B * 16384, 192, 576),
              (B * 4096, 1152, 384), (B * 4096, 384, 384), (B * 4096, 1536, 384), (B * 4096, 384, 1152),
              (B * 1024, 2304, 768)]
    for M, N, K in shapes:
        a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
        bias = torch.randn(N, device=DEV)
        bb = bias.bfloat16()
        byts = M * (N + K) * 2
        fl = 2.0 * M * N * K
        mt = timeit(lambda: torch.nn.functional.linear(a, w, bb))
        line = f"tok M={M:7d} N={N:5d} K={K:5d}: hipBLASLt {mt*1e3:7.1f} us ({byts/mt/1e6:5.0f} GB/s)"
        if ops.tok_supported(M, N, K):
            ms = timeit(lambda: ops.tok_gemm(a, w, bias))
            line += f"  tok {ms*1e3:7.1f} us ({byts/ms/1e6:5.0f} GB/s, {fl/ms/1e9:6.1f} TF/s)"
            if K * 4 == N:
                md = timeit(lambda: ops.tok_gemm(a, w, bias, ops.TOK_GELU_DUAL))
                h = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
                dy = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
                wt = w.contiguous()
                mg = timeit(lambda: ops.tok_gemm(dy, wt, None, ops.TOK_GELU_GRAD, h=h))
                line += f" dual {md*1e3:6.1f} us ({(byts + M*N*2)/md/1e6:5.0f} GB/s) ggrad {mg*1e3:6.1f} us ({(byts + M*N*2)/mg/1e6:5.0f} GB/s)"
                # the unfused alternative: hipBLASLt + standalone GELU fwd / bwd kernels
                with torch.no_grad():
                    yb = torch.nn.functional.linear(a, w, bb)
                    mgf = timeit(lambda: ops.gelu(yb))
                    mdg = timeit(lambda: torch.matmul(dy, w.t()))  # dY[M,K] . W3^T with W3 = w^T: [M,N]
                    dh = torch.empty_like(h)
                    mgb = timeit(lambda: ops._lib.call("msu_gelu_bwd", ops._dt(h), ops._p(h), ops._p(yb),
                                                       ops._p(dh), h.numel(), ops._s(h)))
                line += f" | blas+gelu fwd {(mt+mgf)*1e3:6.1f} us, blas dgrad+gelu' {(mdg+mgb)*1e3:6.1f} us"
        print(line, flush=True)


def nt():
    """Tiled NT GEMM vs hipBLASLt (and the token GEMM) at the stage 1-3 forward and
    input-gradient shapes (M tokens, N outputs, K inputs)."""
    shapes = [(B * 16384, 192, 384), (B * 16384, 576, 192), (B * 16384, 192, 192), (B * 16384, 768, 192),
              (B * 16384, 192, 768), (B * 16384, 192, 576), (B * 16384, 384, 192),
              (B * 4096, 1152, 384), (B * 4096, 384, 1152), (B * 4096, 384, 384), (B * 4096, 1536, 384),
              (B * 4096, 384, 1536), (B * 4096, 384, 768), (B * 4096, 768, 384),
              (B * 1024, 2304, 768), (B * 1024, 768, 2304), (B * 1024, 768, 768), (B * 1024, 3072, 768),
              (B * 1024, 768, 3072), (B * 1024, 768, 1536), (B * 1024, 1536, 768)]
    for M, N, K in shapes:
        a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
        bias = torch.randn(N, device=DEV)
        bb = bias.bfloat16()
        fl = 2.0 * M * N * K
        mt = timeit(lambda: torch.nn.functional.linear(a, w, bb))
        line = f"nt M={M:7d} N={N:5d} K={K:5d}: hipBLASLt {mt*1e3:6.1f} us ({fl/mt/1e9:6.1f} TF/s)"
        if ops.nt_supported(M, N, K):
            ms = timeit(lambda: ops.nt_gemm(a, w, bias))
            ref = torch.nn.functional.linear(a.float(), w.float(), bias)
            err = ((ops.nt_gemm(a, w, bias).float() - ref).norm() / ref.norm()).item()
            line += f"  nt {ms*1e3:6.1f} us ({fl/ms/1e9:6.1f} TF/s, rel err {err:.1e})"
            wk = w.t().contiguous()  # [K][N]: an input-gradient GEMM's forward weight, read in place
            mkn = timeit(lambda: ops.nt_gemm_kn(a, wk))
            mlk = timeit(lambda: a.matmul(wk))
            line += f"  kn {mkn*1e3:6.1f} us (lib {mlk*1e3:6.1f})"
        if ops.tok_supported(M, N, K):
            mk = timeit(lambda: ops.tok_gemm(a, w, bias))
            line += f"  tok {mk*1e3:6.1f} us"
        print(line, flush=True)


def aug():
    """msu_augment_batch at the bench batch (8 x 1024^2): 4 B read + 16 B written per pixel."""
    import random
    import numpy as np
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset import augment as A
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset.dataset import augment_batch
    H = W = 1024
    img = torch.randint(0, 256, (B, H, W, 3), device=DEV, dtype=torch.uint8)
    lbl = torch.randint(0, 256, (B, H, W), device=DEV, dtype=torch.uint8)
    byts = B * H * W * 20
    for name, draw in (("none", lambda i: (0, 0, A.identity_luts())),
                       ("drawn", lambda i: A.draw(A.sample_rng(1, 0, i), True, True)),
                       ("hsv+blur5", lambda i: (A.BC | A.HSV | A.FLIP, 5, A.identity_luts())),
                       ("hsv", lambda i: (A.BC | A.HSV, 0, A.identity_luts()))):
        d = [draw(i) for i in range(B)]
        ops_t = torch.tensor([[o, k] for o, k, _ in d], dtype=torch.int32, device=DEV)
        luts = torch.from_numpy(np.stack([l for _, _, l in d])).to(DEV)
        ms = timeit(lambda: augment_batch(img, lbl, ops_t, luts))
        print(f"augment {name:10s} {ms*1e3:7.1f} us  {byts/ms/1e6:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    for name, fn in (("attn", attn), ("wgrad", wgrad), ("conv", conv), ("ln", ln), ("lnadd", lnadd), ("tok", tok), ("nt", nt), ("stream", stream), ("aug", aug)):
        if what in (name, "all"):
            fn()
