"""MS-UNet (Swin-T) training throughput on MI355X: images/sec at 1024^2, bs=8 per GPU.

    python bench.py [--gpus N --steps K --warmup W]        # N=1 default
    torchrun --nproc-per-node N bench.py --gpus N ...     # one rank per GPU (RCCL)

A step = one full training step of the reference's trainer.py:308-316 on one batch per
rank: bf16-autocast forward of MS-UNet -> DynamicLoss -> backward -> bucketed RCCL
gradient all-reduce (N > 1) -> fused AdamW.  Synthetic StyleGAN2-shaped inputs are
generated in HBM before timing.  Rank 0 prints ONE JSON line.

Extra objects: ``roofline`` for the dominant kernel (timed live with HIP events on its
stream) and ``cpu_baseline`` (the CPU oracle's training step on a bounded sample).
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

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--img", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--backbone", default="swin_t")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--skip-dead", action="store_true", help="skip the reference's discarded branches (exact)")
    return ap.parse_args()


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
    return {"kernel": "conv3x3_v2_kernel (refine2 fwd, bf16 MFMA implicit GEMM)", "bound": "mfma",
            "achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
            "flops_per_launch": flops, "ms_per_launch": round(ms, 4)}


def attention_roofline(device, batch, img, C, heads):
    """Window attention (the north star's second named kernel): the stage-0 shifted block's
    msu_win_attn_fwd launch at the bench shape, timed with HIP events on the launching
    (current) stream.  Algorithmic work per window x head: 4*49*49*32 FLOP (QK^T and PV) and
    q, k, v in + o out; the padded grid (ceil(H/7)^2 windows per image) is what the kernel
    computes.  The timed call includes the tiny aux kernel (bias image, scaled qkv bias) that
    precedes every attention launch.  HBM-bound (AI ~ 25 FLOP/B); both fractions are reported."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    res = img // 4
    g = torch.Generator(device="cpu").manual_seed(2)
    qkv = torch.randn(batch, res, res, 3 * C, generator=g).to(device, torch.bfloat16)
    qb = torch.zeros(3 * C, device=device)
    tb = (0.02 * torch.randn(169, heads, generator=g)).to(device)
    s = torch.cuda.current_stream(device)

    def launch():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            ops.window_attention(qkv, qb, tb, heads, 3, 0.0, 1)

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
    nwin = batch * ((res + 6) // 7) ** 2
    flops = 4.0 * 49 * 49 * 32 * nwin * heads
    byts = batch * res * res * 4 * C * 2
    return {"kernel": "attn_fwd_mfma (stage-0 shifted window attention fwd, bf16 MFMA)", "bound": "hbm",
            "achieved": round(byts / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "mfma_tflops": round(flops / (ms * 1e-3) / 1e12, 1),
            "mfma_frac": round(flops / (ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
            "bytes_per_launch": byts, "flops_per_launch": flops, "ms_per_launch": round(ms, 4)}


def cpu_baseline(seconds_budget=25.0):
    """The CPU oracle (pure PyTorch fp32 restatement of the reference path) timing one
    training step (fwd + DynamicLoss + bwd + AdamW) of Swin-T MS-UNet on 4 x 256^2
    (BASELINE config 1); bounded to a few steps."""
    from oracle.msunet import make_cfg, init_params, msunet_forward
    from oracle.dynamic_loss import dynamic_loss
    from semantic_segmentation_of_stylegan2_artifacts_amd.data import synthetic_batch
    cores = len(os.sched_getaffinity(0))
    cores = max(1, min(cores, 16))
    torch.set_num_threads(cores)
    cfg = make_cfg(img_size=256, embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24],
                   drop_path_rate=0.0)
    p = init_params(cfg, seed=0)
    params = {k: v.requires_grad_(True) for k, v in p.items() if v.is_floating_point()}
    p.update(params)
    opt = torch.optim.AdamW(list(params.values()), lr=1e-5, weight_decay=1e-3)
    x, y = synthetic_batch(4, 256, "cpu", 120)
    times = []
    t_start = time.perf_counter()
    for i in range(6):
        t0 = time.perf_counter()
        out = msunet_forward(p, cfg, x)
        loss = dynamic_loss(out, y, 0.2, 0.8, 0.45)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > seconds_budget and i >= 1:
            break
    steady = times[1:] if len(times) > 1 else times
    sps = sum(steady) / len(steady)
    return {"value": round(4 / sps, 4), "unit": "images/s", "cores": cores, "kind": "port",
            "sample": f"CPU oracle (torch fp32) Swin-T MS-UNet train step, 4x256^2 (config 1), "
                      f"{len(steady)} steady steps of {len(times)}, {sps:.2f} s/step"}


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


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)

    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config
    from semantic_segmentation_of_stylegan2_artifacts_amd.network import MSUNet
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    from semantic_segmentation_of_stylegan2_artifacts_amd.data import batch_pool

    cfg = load_config(None, args.backbone, **{"DATA.IMG_SIZE": args.img, "DATA.BATCH_SIZE": args.batch})
    torch.manual_seed(cfg.SEED)
    model = MSUNet(cfg, img_size=args.img, num_classes=1).to(device)
    model.ms_unet.skip_dead_branches = args.skip_dead
    trainer = Trainer(model, cfg, device, world_size=world,
                      process_group=dist.group.WORLD if world > 1 else None, rank=rank, seed=cfg.SEED)
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
            "metric": "training images/sec at 1024^2 bs=8 per GPU (MS-UNet Swin-T, fwd+DynamicLoss+bwd+AdamW)",
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
            "config": {"workload": f"1xMI355X {args.img}x{args.img} bs={args.batch} Swin-T MS-UNet train step"
                       if world == 1 else f"{world}xMI355X DP {args.img}x{args.img} global bs={args.batch * world}",
                       "model": f"MS-UNet {args.backbone}", "global_batch": args.batch * world,
                       "img_size": args.img, "parallelism": f"dp{world}",
                       "dead_branches": "skipped" if args.skip_dead else "executed (no grad)",
                       "params": trainer.num_params(), "final_loss": round(loss_val, 6)},
        }
        if not args.no_roofline:
            res["roofline"] = conv_roofline(device, args.batch, args.img, cfg.MODEL.SWIN.EMBED_DIM)
            res["roofline_attention"] = attention_roofline(device, args.batch, args.img, cfg.MODEL.SWIN.EMBED_DIM,
                                                           cfg.MODEL.SWIN.NUM_HEADS[0])
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline()
            res["dice_vs_ref"] = dice_vs_reference(device)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
