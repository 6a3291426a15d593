"""MS-UNet (Swin-T) training throughput on MI355X: images/sec at 1024^2, bs=8 per GPU.

    python bench.py [--gpus N --steps K --warmup W]        # N=1 default; N>1 starts N ranks itself
    torchrun --nproc-per-node N bench.py --gpus N ...     # one rank per GPU (RCCL), launcher-started

With ``--gpus N > 1`` and no ``WORLD_SIZE`` in the environment, this process touches no GPU: it
starts N child processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
a free MASTER_PORT), waits for them and exits with the first failing child's status.  Each
rank binds GPU LOCAL_RANK and joins an RCCL (``--dist-backend nccl``, default) process group
of exactly N ranks; ``--dist-backend gloo`` runs the same step with gloo collectives and lets
N ranks share one GPU (the one-GPU rehearsal of the N-rank path, tests/test_gpu_bench_dp.py).

A step = one full training step of the reference's trainer.py:308-316 on one batch per
rank: bf16-autocast forward of MS-UNet -> DynamicLoss -> backward -> bucketed RCCL
gradient all-reduce (N > 1) -> non-finite check -> fused AdamW.  The Trainer runs its first
four steps eagerly, times the last two, and replays the captured step as a HIP graph from then
on when the steadier of them was launch-bound (host issue time >= 0.9 x GPU time), else stays
eager (MSU_GRAPH=1/0 forces either; the decision falls inside the warmup when W >= 5).  Synthetic StyleGAN2-shaped inputs are generated in HBM before timing
and copied into the graph's input buffers inside every timed step.  Rank 0 prints ONE
JSON line.

Extra objects: ``roofline`` for the dominant kernel (timed live with HIP events on its
stream), ``roofline_attention`` (window attention), ``roofline_decoder`` (the decoder head
stack fwd+bwd against the HBM roofline) and ``cpu_baseline`` (the CPU oracle's training step,
Swin-T and Swin-B, on the box's host cores) and ``input_pipeline`` (the augmentation kernel's
HBM roofline, and training steps fed from PNG files through the GPU input pipeline: the
decode- and PCIe-inclusive rate next to the resident one).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BACKBONE_NAME = {"swin_t": "Swin-T", "swin_s": "Swin-S", "swin_b": "Swin-B"}
MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--img", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--backbone", default="swin_t")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-input-pipeline", action="store_true",
                    help="skip the PNG -> GpuBatchLoader -> train-step leg (runs after the timed region)")
    ap.add_argument("--skip-dead", action="store_true", help="skip the reference's discarded branches (exact)")
    ap.add_argument("--grad-wire", choices=["f32", "bf16", "fp16"], default="f32",
                    help="DP gradient all-reduce precision (BASELINE config 5: fp16 grads)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: RCCL (one GPU per rank) or gloo (ranks may share a GPU; rehearsal)")
    ap.add_argument("--dump-state", default=None,
                    help="write each rank's final flat parameters to <path>.rank<R>.pt (DP tests)")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """Start n rank processes of this script (no GPU call in this process: the children are
    fresh interpreters, not forks or execs of a GPU-initialised one) and return the exit status
    of the first that fails (0 when all succeed).  A failing rank ends the others, so a hung
    collective does not outlive it."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCH_NCCL_CUDA_EVENT_CACHE="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    status = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            rc = p.poll()
            if rc is None:
                continue
            alive.remove(p)
            if rc != 0 and status == 0:
                status = rc
                for q in alive:
                    q.terminate()
        time.sleep(0.2)
    return status if status >= 0 else 128 - status


def conv_roofline(device, batch, img, C):
    """Dominant kernel: the refine2 3x3 conv forward (implicit GEMM, bf16 MFMA) at the bench
    shape, as the model runs it (refine_conv_act: GELU(z1) precomputed by refine1's epilogue).
    achieved = 2*B*H*W*Cout*Cin*9 FLOP per launch / average launch time (HIP events on the
    launching stream, i.e. torch's current stream)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops, _lib
    g = torch.Generator(device="cpu").manual_seed(1)
    z1 = torch.randn(batch, img, img, C, generator=g).to(device, torch.bfloat16)
    a1 = ops.gelu(z1)
    w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(device)
    b = torch.zeros(C, device=device)
    # the launch itself, as refine_conv_act issues it (weights re-laid out once, outside)
    wt = w.permute(2, 3, 0, 1).reshape(9, C, C).to(torch.bfloat16).contiguous()
    z2 = torch.empty_like(a1)
    s = torch.cuda.current_stream(device)

    def launch():
        _lib.call("msu_conv3x3_fwd2", 1, 0, a1.data_ptr(), wt.data_ptr(), b.data_ptr(), z2.data_ptr(), None,
                  batch, img, img, C, C, s.cuda_stream)

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record(s)
    for _ in range(n):
        launch()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    flops = 2.0 * batch * img * img * C * C * 9
    achieved = flops / (ms * 1e-3) / 1e12
    traffic = None
    pmc = os.path.join(REPO, "profiles", "conv3x3_fwd_pmc.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    # the C-ABI dispatches C = 96 to the 16-row-tile v3 kernel (csrc/conv3x3.h)
    kname = "conv3x3_v3_kernel" if C == 96 else "conv3x3_v2_kernel"
    return {"kernel": f"{kname} (refine2 fwd, bf16 MFMA implicit GEMM)", "bound": "mfma",
            "achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
            "flops_per_launch": flops, "ms_per_launch": round(ms, 4)}


def attention_roofline(device, batch, img, C, heads, p_drop):
    """Window attention (the north star's second named kernel): the stage-0 shifted block's
    msu_win_attn_fwd and msu_win_attn_bwd launches at the bench shape with the training
    attention dropout, each timed with HIP events on the launching (current) stream.
    Algorithmic work per window x head: forward 4*49*49*32 FLOP (QK^T, PV), backward 2.5x that
    (QK^T and dO V^T recomputed, dV, dK, dQ); bytes: forward q, k, v in + o out, backward
    q, k, v, dO in + dq, dk, dv out (the forward's dropout keep bits, 128 B per window x head
    each way, are not counted).  The padded grid (ceil(H/7)^2 windows per image) is what the
    kernels compute.  Each timed call includes the tiny aux kernel (bias image, 16-bit qkv
    bias) that precedes every attention launch; the backward's parameter-gradient tail
    (reductions over workgroup partials) is included.  HBM-bound (AI ~ 25 FLOP/B)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    res = img // 4
    g = torch.Generator(device="cpu").manual_seed(2)
    qkv = torch.randn(batch, res, res, 3 * C, generator=g).to(device, torch.bfloat16)
    qb = torch.zeros(3 * C, device=device)
    tb = (0.02 * torch.randn(169, heads, generator=g)).to(device)
    dout = torch.randn(batch, res, res, C, generator=g).to(device, torch.bfloat16)
    s = torch.cuda.current_stream(device)

    def fwd():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return ops.window_attention(qkv, qb, tb, heads, 3, p_drop, 1)

    def graph_for_bwd():
        x = qkv.detach().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return ops.window_attention(x, qb, tb, heads, 3, p_drop, 1)

    def timed(run, args):
        # back-to-back launches between two events: the GPU never waits on the host
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for a in args:
            run(a)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / len(args)

    n = 10
    timed(lambda _: fwd(), range(3))
    ms_f = timed(lambda _: fwd(), range(n))
    timed(lambda y: y.backward(dout), [graph_for_bwd() for _ in range(3)])
    ms_b = timed(lambda y: y.backward(dout), [graph_for_bwd() for _ in range(n)])
    nwin = batch * ((res + 6) // 7) ** 2
    flops = 4.0 * 49 * 49 * 32 * nwin * heads
    tok = batch * res * res
    byts, byts_b = tok * 4 * C * 2, tok * 7 * C * 2

    def rate(b, ms):
        return b / (ms * 1e-3) / 1e9

    fused = fused_unit_roofline(device, batch, img, C, heads, p_drop)
    return {"kernel": "attn_fwd_mfma (stage-0 shifted window attention fwd, bf16 MFMA, dropout %g)" % p_drop,
            "fused_unit": fused,
            "bound": "hbm", "achieved": round(rate(byts, ms_f), 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(rate(byts, ms_f) / HBM_PEAK_GBS, 4),
            "mfma_tflops": round(flops / (ms_f * 1e-3) / 1e12, 1),
            "mfma_frac": round(flops / (ms_f * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
            "bytes_per_launch": byts, "flops_per_launch": flops, "ms_per_launch": round(ms_f, 4),
            "backward": {"kernel": "attn_bwd_mfma (+ aux, partial reductions)", "bound": "hbm",
                         "achieved": round(rate(byts_b, ms_b), 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(rate(byts_b, ms_b) / HBM_PEAK_GBS, 4),
                         "mfma_tflops": round(2.5 * flops / (ms_b * 1e-3) / 1e12, 1),
                         "bytes_per_launch": byts_b, "flops_per_launch": 2.5 * flops,
                         "ms_per_launch": round(ms_b, 4)}}


def fused_unit_roofline(device, batch, img, C, heads, p_drop):
    """The stage-0 fused unit (qkv Linear -> window attention -> proj Linear, all three in one
    kernel, msu_win_attn_qkv_fwd2 = attn_qkv_fwd_mfma<PROJ>) at the bench shape: inference (no qkv / o written) and the training
    forward (qkv and o kept for the backward, dropout keep bits), HIP events on the launching
    stream.  Algorithmic FLOP per launch = 2 M C 3C (qkv) + 4 49^2 32 per window x head (QK^T, PV
    over the padded window grid) + 2 M C C (proj); bytes = x in + y out (+ qkv and o kept in
    training); MFMA fraction against the dense bf16 peak."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    res = img // 4
    M = batch * res * res
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(batch, res, res, C, generator=g).to(device, torch.bfloat16)
    w = (torch.randn(3 * C, C, generator=g) / C ** 0.5).to(device)
    b = (0.1 * torch.randn(3 * C, generator=g)).to(device)
    tb = (0.02 * torch.randn(169, heads, generator=g)).to(device)
    wp = (torch.randn(C, C, generator=g) / C ** 0.5).to(device)
    bp = torch.zeros(C, device=device)
    s = torch.cuda.current_stream(device)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        if not ops.window_attention_qkv_fusable(x, heads, b):
            return None

    def run(store):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return torch.ops.msunet.window_attention_qkv(x, w, b, tb, wp, bp, heads, 3, p_drop, 1, None, store)

    def timed(store, n=10):
        for _ in range(2):
            run(store)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            run(store)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    nwin = batch * ((res + 6) // 7) ** 2
    flops = 2.0 * M * C * 3 * C + 4.0 * 49 * 49 * 32 * nwin * heads + 2.0 * M * C * C
    kern = "attn_qkv_fwd_mfma<PROJ> (qkv Linear + window attention + proj, one kernel)"
    out = {"kernel": kern,
           "flops_per_launch": flops}
    for name, store, byts in (("inference", False, 2 * M * C * 2), ("training_fwd", True, (2 * C + 3 * C + C) * M * 2)):
        ms = timed(store)
        tf = flops / (ms * 1e-3) / 1e12
        out[name] = {"ms_per_launch": round(ms, 4), "mfma_tflops": round(tf, 1),
                     "mfma_frac": round(tf / MFMA_BF16_PEAK_TFLOPS, 4), "bytes_per_launch": byts,
                     "hbm_frac": round(byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cpu_train_steps(backbone, steps=10, first=2):
    """The CPU oracle's fp32 training step (fwd + DynamicLoss + bwd + AdamW) of one backbone
    on 4 x 256^2 (BASELINE config 1) in training semantics: the config's drop-path (0.1) and
    attention dropout (0.05) drawn per step, as the reference's ``model.train()`` step does
    (config.py MODEL defaults; the reference's CPU profile spends ~12 % in ``bernoulli_``).
    Returns (images/s averaged over steps first..steps-1, s/step, list of step times)."""
    from oracle.msunet import make_cfg, init_params, msunet_forward, SWIN_T, SWIN_B
    from oracle.dynamic_loss import dynamic_loss
    from semantic_segmentation_of_stylegan2_artifacts_amd.config import load_config
    from semantic_segmentation_of_stylegan2_artifacts_amd.data import synthetic_batch
    arch = {"swin_t": SWIN_T, "swin_b": SWIN_B}[backbone]
    mc = load_config(None, backbone).MODEL
    cfg = make_cfg(img_size=256, drop_path_rate=mc.DROP_PATH_RATE, attn_drop_rate=mc.ATTN_DROP_RATE,
                   drop_rate=mc.DROP_RATE, **arch)
    p = init_params(cfg, seed=0)
    params = {k: v.requires_grad_(True) for k, v in p.items() if v.is_floating_point()}
    p.update(params)
    opt = torch.optim.AdamW(list(params.values()), lr=1e-5, weight_decay=1e-3)
    x, y = synthetic_batch(4, 256, "cpu", 120)
    gen = torch.Generator().manual_seed(0)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        out = msunet_forward(p, cfg, x, training=True, generator=gen)
        loss = dynamic_loss(out, y, 0.2, 0.8, 0.45)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
    steady = times[first:]
    sps = sum(steady) / len(steady)
    return 4 / sps, sps, times


def cpu_baseline():
    """the CPU oracle (pure PyTorch fp32 restatement of the reference step,
    validated against the imported reference in the dev container) on the host cores of this
    box, config 1 shapes (4 x 256^2), Swin-T (the bench backbone: ``value``) and Swin-B
    (config.yaml's default backbone), 10 steps each, steps 2-9 averaged.  Threads: the
    process's CPU share (OMP_NUM_THREADS when the scheduler sets it, else the affinity mask)."""
    affinity = len(os.sched_getaffinity(0))
    threads = int(os.environ.get("OMP_NUM_THREADS") or affinity)
    threads = max(1, min(threads, affinity))
    torch.set_num_threads(threads)
    t_ips, t_sps, t_times = _cpu_train_steps("swin_t")
    b_ips, b_sps, b_times = _cpu_train_steps("swin_b")
    return {"value": round(t_ips, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "cpus_in_affinity_mask": affinity,
            "sample": f"CPU oracle (torch fp32) MS-UNet train step with drop-path 0.1 and attention "
                      f"dropout 0.05 drawn, 4x256^2 (config 1), 10 steps, "
                      f"steps 2-9 averaged: Swin-T {t_sps:.2f} s/step",
            "swin_b": {"value": round(b_ips, 4), "unit": "images/s", "s_per_step": round(b_sps, 3)},
            "step_times_s": {"swin_t": [round(v, 3) for v in t_times], "swin_b": [round(v, 3) for v in b_times]}}


def decoder_roofline(device, batch, img, C):
    """North-star figure for the decoder head stack (SURVEY 8a rows 15 + 16): expand Linear
    (+GELU) -> refine1 (4x4 d2s on load) -> GELU -> refine2 -> LayerNorm + 1x1 head, forward
    AND backward, timed with HIP events around whole fwd+bwd passes of the model's own modules
    at the bench shape.  Algorithmic work per op = its FLOPs and the bytes of its inputs read
    once and outputs written once (bf16 activations, f32 logits / statistics); the roofline time
    is sum_op max(flops / MFMA peak, bytes / HBM peak).  Reported: HBM GB/s over the measured
    time (the north star's '>= 40 % HBM on the decoder conv stack') and roofline time /
    measured time."""
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import FinalPatchExpand_X4_V2
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    h = img // 4
    head = FinalPatchExpand_X4_V2((h, h), dim=C, dim_scale=4).to(device)
    out_w = (torch.randn(1, C, 1, 1, device=device) / C ** 0.5).requires_grad_(True)
    g = torch.Generator(device="cpu").manual_seed(5)
    x = (torch.randn(batch, h * h, C, generator=g)).to(device, torch.bfloat16).requires_grad_(True)
    dl = torch.randn(batch, 1, img, img, generator=g).to(device)

    def run():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            z2 = head.pre_norm(x)
            logit = ops.head_norm_output(z2, head.norm.weight, head.norm.bias, out_w, head.norm.eps)
        logit.backward(dl)

    for _ in range(2):
        run()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 5
    e0.record(s)
    for _ in range(n):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    M, P, E = batch * h * h, batch * img * img, 16 * C
    a16, f32 = 2, 4
    act = P * C * a16                      # one full-resolution bf16 activation
    conv_f = 2.0 * P * C * C * 9
    lin_f = 2.0 * M * C * E
    ops_ = {  # op: (flops, bytes)
        "expand_fwd": (lin_f, M * C * a16 + 2 * M * E * a16),
        "refine1_fwd": (conv_f, act + 2 * act),
        "refine2_fwd": (conv_f, act + act),
        "head_fwd": (8.0 * P * C, act + 3 * P * f32),
        "head_bwd": (10.0 * P * C, act + 3 * P * f32 + act),
        "refine2_dgrad": (conv_f, 3 * act),
        "refine2_wgrad": (conv_f, 2 * act),
        "refine1_dgrad": (conv_f, 3 * act),
        "refine1_wgrad": (conv_f, 2 * act),
        "expand_dgrad": (lin_f, M * E * a16 + M * C * a16),
        "expand_wgrad": (lin_f, M * E * a16 + M * C * a16),
    }
    flops = sum(f for f, _ in ops_.values())
    byts = sum(b for _, b in ops_.values())
    t_roof = sum(max(f / (MFMA_BF16_PEAK_TFLOPS * 1e12), b / (HBM_PEAK_GBS * 1e9)) for f, b in ops_.values())
    gbs = byts / (ms * 1e-3) / 1e9
    return {"stack": "FinalPatchExpand_X4_V2 + LN/1x1 head, fwd+bwd (rows 15+16)", "bound": "hbm",
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
            "ms_per_pass": round(ms, 3), "bytes_per_pass": byts, "flops_per_pass": flops,
            "mfma_tflops": round(flops / (ms * 1e-3) / 1e12, 1),
            "roofline_ms": round(t_roof * 1e3, 3), "roofline_frac": round(t_roof * 1e3 / ms, 4)}


def dice_vs_reference(device):
    """'Dice vs ref' of the metric: identical Swin-T weights and a 4 x 256^2 synthetic batch
    (BASELINE config 1) through the CPU oracle (the reference path restated, fp32) and
    through the HIP path (fp32 parity mode and bf16 training mode); soft Dice of both over
    the fake images (validation_functions.py:300-301), the GPU side by the msu_seg_metrics
    kernel.  Part of the cpu_baseline leg (the only bench leg that runs the oracle)."""
    from oracle.msunet import make_cfg, init_params, msunet_forward
    from oracle import metrics as om
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    from semantic_segmentation_of_stylegan2_artifacts_amd.data import synthetic_batch
    from semantic_segmentation_of_stylegan2_artifacts_amd import validation
    cfg = make_cfg(img_size=256, embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], drop_path_rate=0.0)
    params = init_params(cfg, seed=0)
    x, y = synthetic_batch(4, 256, "cpu", 120)
    with torch.no_grad():
        ref = msunet_forward(params, cfg, x)
    ref_per = [om.image_metrics(ref[b], y[b]) for b in range(4)]
    fake = [b for b in range(4) if y[b].sum() > 0]
    ref_dice = sum(ref_per[b]["soft_dice"] for b in fake) / len(fake)
    model = MSUNetSys(img_size=256, embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24],
                      drop_path_rate=0.0)
    model.load_state_dict(params, strict=True)
    model = model.to(device).eval()
    out = {"sample": "Swin-T 4x256^2 synthetic, oracle fp32 CPU vs HIP", "soft_dice_ref": round(ref_dice, 6)}
    with torch.no_grad():
        for name, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
            with torch.autocast("cuda", dtype=dt, enabled=dt != torch.float32):
                logits = model(x.to(device))
            per = validation.batch_metrics(logits, y.to(device))
            d = sum(per[b]["soft_dice"] for b in fake) / len(fake)
            out[f"soft_dice_hip_{name}"] = round(d, 6)
            out[f"abs_diff_{name}"] = float(f"{abs(d - ref_dice):.3g}")
            if dt == torch.float32:
                err = (logits.float().cpu() - ref).abs().max().item() / ref.abs().max().item()
                out["logits_max_rel_err_fp32"] = float(f"{err:.3g}")
    out["within_1e-3"] = out["abs_diff_fp32"] <= 1e-3
    return out


def _write_png_set(root, n_fake, n_real, img, seed, unique=4):
    """Synthetic StyleGAN2-shaped PNG files in the reference's layout (dataset.py:141-144):
    smooth colour fields + noise (compressible like a photo) and the synthetic artifact masks;
    ``unique`` distinct files per kind, the rest hard links (every file is decoded anyway)."""
    import numpy as np
    from PIL import Image
    from semantic_segmentation_of_stylegan2_artifacts_amd.data import synthetic_batch
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:img, 0:img].astype(np.float32) / img
    for kind, n in (("fake", n_fake), ("real", n_real)):
        os.makedirs(os.path.join(root, kind + "_images"), exist_ok=True)
        os.makedirs(os.path.join(root, kind + "_labels"), exist_ok=True)
        names = [f"{kind}{i:04d}" for i in range(n)]
        with open(os.path.join(root, kind + ".txt"), "w") as f:
            f.write("\n".join(names) + "\n")
        u = min(unique, n)
        _, masks = synthetic_batch(u, img, "cpu", seed + (kind == "real"), fake_ratio=1.0 if kind == "fake" else 0.0)
        for i, name in enumerate(names):
            ip = os.path.join(root, kind + "_images", name + ".png")
            lp = os.path.join(root, kind + "_labels", name + "_mask.png")
            if i >= u:
                os.link(os.path.join(root, kind + "_images", names[i % u] + ".png"), ip)
                os.link(os.path.join(root, kind + "_labels", names[i % u] + "_mask.png"), lp)
                continue
            a, b, c = g.random(3) * 6
            base = np.stack([np.sin(a * xx + b * yy), np.cos(b * xx - c * yy), np.sin(c * (xx + yy))], -1)
            im = np.clip((base * 0.4 + 0.5) * 255 + g.normal(0, 6, (img, img, 3)), 0, 255).astype(np.uint8)
            Image.fromarray(im).save(ip, compress_level=1)
            lab = masks[i].numpy() if kind == "fake" else np.zeros((img, img), np.float32)
            Image.fromarray((lab > 0).astype(np.uint8) * 255).save(lp, compress_level=1)


def input_pipeline_leg(device, trainer, batch, img, seed, resident_ms):
    """The reference's input path (PNG decode, augmentation, /255, H2D: trainer.py:239-245,
    :299-300) in front of the same training step: ``augment_kernel`` = msu_augment_batch at the
    bench batch against the HBM roofline (20 B / pixel); ``loader_fed`` = training steps fed by
    GpuBatchLoader from PNG files on the box's disk (decode on host threads, pinned uint8
    upload, GPU augmentation), i.e. the PCIe- and decode-inclusive rate next to the resident one."""
    import shutil
    import tempfile
    import numpy as np
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset import (GpuBatchLoader, RandomGenerator,
                                                                          SegArtifact_dataset, epoch_plan)
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset import augment as A
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset.dataset import augment_batch
    out = {}
    imgs = torch.randint(0, 256, (batch, img, img, 3), device=device, dtype=torch.uint8)
    lbls = torch.randint(0, 256, (batch, img, img), device=device, dtype=torch.uint8)
    draws = [A.draw(A.sample_rng(seed, 0, i), True, True) for i in range(batch)]
    ops_t = torch.tensor([[o, k] for o, k, _ in draws], dtype=torch.int32, device=device)
    luts = torch.from_numpy(np.stack([l for _, _, l in draws])).to(device)
    for _ in range(2):
        augment_batch(imgs, lbls, ops_t, luts)
    torch.cuda.synchronize()
    n = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        augment_batch(imgs, lbls, ops_t, luts)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    byts = batch * img * img * 20
    out["augment_kernel"] = {"kernel": "augment_kernel (msu_augment_batch, drawn ops)", "bound": "hbm",
                             "achieved": round(byts / ms / 1e6, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(byts / ms / 1e6 / HBM_PEAK_GBS, 4), "bytes_per_launch": byts,
                             "ms_per_launch": round(ms, 4),
                             "ops": [[int(o), int(k)] for o, k, _ in draws]}
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    root = tempfile.mkdtemp(prefix="msu_png_")
    try:
        n_fake, n_real = 6 * batch, 4 * batch
        _write_png_set(root, n_fake, n_real, img, seed)
        tf = RandomGenerator(output_size=[img, img], random_flip_flag=True, transform=True)
        db_fake = SegArtifact_dataset(root, root, "fake", transform=tf)
        db_real = SegArtifact_dataset(root, root, "real", transform=tf)
        t = time.perf_counter()
        for i in range(4):
            db_fake.read_raw(i)
        decode_ms = (time.perf_counter() - t) / 4 * 1e3
        mixed, sampler, _, _ = epoch_plan(db_fake, db_real, epoch_num=0, seed=seed)
        loader = GpuBatchLoader(mixed, sampler, device=device, num_threads=threads, slots=3, seed=seed,
                                epoch=0, batches_per_step=batch // 2)
        it = iter(loader)
        warm = 2
        for _ in range(warm):
            b = next(it)
            trainer.step(b["image"], b["label"])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        k = 0
        for b in it:
            last = trainer.step(b["image"], b["label"])
            k += 1
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out["loader_fed"] = {
            "value": round(k * batch / el, 3), "unit": "images/s", "steps": k, "warmup": warm,
            "ms_per_step": round(el / k * 1e3, 3), "resident_ms_per_step": round(resident_ms, 3),
            "decode_threads": threads, "png_decode_ms_per_image": round(decode_ms, 2),
            "final_loss": round(last.item(), 6),
            "sample": f"{n_fake} fake + {n_real} real synthetic {img}^2 PNGs (compress_level 1), epoch plan "
                      f"real ratio 0.4, BatchPatternSampler pairs x {batch // 2} per step, RandomGenerator "
                      f"(transform + flip) on the GPU"}
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        # ProcessGroupNCCL's event cache hands a retired work's events to new works; with a
        # captured step its watchdog then queries an event recorded in a capture and aborts
        # (DESIGN 4b).  Must be set before the process group exists.
        os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] = "0"
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    device = torch.device("cuda", local)

    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config, switches
    from semantic_segmentation_of_stylegan2_artifacts_amd.network import MSUNet
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    from semantic_segmentation_of_stylegan2_artifacts_amd.data import batch_pool

    cfg = load_config(None, args.backbone, **{"DATA.IMG_SIZE": args.img, "DATA.BATCH_SIZE": args.batch})
    torch.manual_seed(cfg.SEED)
    model = MSUNet(cfg, img_size=args.img, num_classes=1).to(device)
    model.ms_unet.skip_dead_branches = args.skip_dead
    wire = {"f32": None, "bf16": torch.bfloat16, "fp16": torch.float16}[args.grad_wire]
    trainer = Trainer(model, cfg, device, world_size=world,
                      process_group=dist.group.WORLD if world > 1 else None, rank=rank, seed=cfg.SEED,
                      grad_wire_dtype=wire)
    pool = batch_pool(2, args.batch, args.img, device, cfg.SEED + 1000 * rank)

    for i in range(args.warmup):
        trainer.step(*pool[i % len(pool)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        last = trainer.step(*pool[i % len(pool)])
    t_host = time.perf_counter() - t0  # host issue time of the K steps (no sync inside)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], device=device, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    elapsed = dt.item()
    loss_val = last.item() if last is not None else float("nan")

    if rank == 0:
        imgs = args.batch * world * args.steps
        res = {
            "metric": f"training images/sec at {args.img}^2 bs={args.batch} per GPU "
                      f"(MS-UNet {BACKBONE_NAME[args.backbone]}, fwd+DynamicLoss+bwd+AdamW)",
            "value": round(imgs / elapsed, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "host_ms_per_step": round(t_host / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uniform RGB /255 + ellipse artifact masks, 60% fake), random-init weights",
            "config": {"workload": f"1xMI355X {args.img}x{args.img} bs={args.batch} {BACKBONE_NAME[args.backbone]} "
                                   f"MS-UNet train step" if world == 1 else
                                   f"{world}xMI355X DP {args.img}x{args.img} global bs={args.batch * world} "
                                   f"{BACKBONE_NAME[args.backbone]} MS-UNet train step",
                       "model": f"MS-UNet {args.backbone}", "global_batch": args.batch * world,
                       "world_size": dist.get_world_size() if world > 1 else 1,
                       "dist_backend": (args.dist_backend if world > 1 else None),
                       "img_size": args.img, "parallelism": f"dp{world}", "grad_allreduce": args.grad_wire,
                       "dead_branches": "skipped" if args.skip_dead else "executed (no grad)",
                       "step_execution": "hip_graph_replay" if trainer._graph is not None else "eager",
                       "graph_probe": getattr(trainer, "graph_probe", None),
                       "params": trainer.num_params(), "final_loss": round(loss_val, 6),
                       # environment switches away from their defaults (+ unknown MSU_* names):
                       # empty for the product configuration (switches.py)
                       "switches": switches.report()},
        }
        if not args.no_roofline:
            res["roofline"] = conv_roofline(device, args.batch, args.img, cfg.MODEL.SWIN.EMBED_DIM)
            res["roofline_attention"] = attention_roofline(device, args.batch, args.img, cfg.MODEL.SWIN.EMBED_DIM,
                                                           cfg.MODEL.SWIN.NUM_HEADS[0], cfg.MODEL.ATTN_DROP_RATE)
            res["roofline_decoder"] = decoder_roofline(device, args.batch, args.img, cfg.MODEL.SWIN.EMBED_DIM)
        if not args.no_input_pipeline and world == 1:
            res["input_pipeline"] = input_pipeline_leg(device, trainer, args.batch, args.img, cfg.SEED,
                                                       elapsed / args.steps * 1e3)
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline()
            res["dice_vs_ref"] = dice_vs_reference(device)
        print(json.dumps(res), flush=True)
    if args.dump_state:
        torch.save({"data": [g.data.detach().cpu() for g in trainer.groups], "loss": loss_val,
                    "world": world, "rank": rank}, f"{args.dump_state}.rank{rank}.pt")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
