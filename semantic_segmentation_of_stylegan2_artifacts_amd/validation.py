"""Validation metrics of ``scripts/validation_functions.py`` computed on the GPU.

The reference loops over single images, moves every prediction to the host and calls medpy
(``calculate_metrics`` :37-178, ``calculate_metrics_real`` :214-244, ``calculate_metrics_fake``
:247-309).  Here one HIP pass (``msu_seg_metrics``) reduces a whole batch of logits to per-image
sums; only ``[B, 12]`` doubles come back, and the formulas below are the reference's:

* an image is "real" when its ground truth is empty (``:111``), else "fake";
* fake: binary Dice / IoU / recall / precision with medpy's published definitions
  (``dc`` = 2|A&B| / (|A| + |B|), 0 when both are empty; ``jc`` = |A&B| / |A|B|; recall /
  precision 0 on an empty denominator), ``bin_f1`` with smooth 1e-8 (``:264``), soft Dice
  (``:300-301``) and soft IoU (``:304``) with smooth 1e-8;
* real: FPR = fp / (fp + tn) (``:235``);
* both: binary accuracy and the binary / soft confusion matrices;
* ``Score = mean_soft_dice - 10 * mean_FPR`` (``:180``).
"""
import torch

from . import _lib, ops

SMOOTH = 1e-8

# column order of msu_seg_metrics' output rows
COLS = ("inter", "sum_p2", "sum_g", "sum_p", "soft_fp", "soft_fn", "soft_tn", "tp", "fp", "fn", "tn")


def image_sums(logits, labels, threshold=0.5):
    """Per-image metric sums on the GPU: logits [B, 1, H, W] (f32 / bf16 / f16), labels [B, H, W]
    or [B, 1, H, W] -> float64 tensor [B, 12] (host)."""
    ops._need_cuda(logits, labels)
    B = logits.shape[0]
    if labels.shape[0] != B:
        raise ValueError(f"batch mismatch: logits {B}, labels {labels.shape[0]}")
    x = logits.contiguous()
    if x.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        x = x.float()
    lab = ops._f32(labels)
    N = x[0].numel()
    if lab[0].numel() != N:
        raise ValueError(f"label size {tuple(labels.shape)} does not match logits {tuple(logits.shape)}")
    L = _lib.lib()
    nblk = L.msu_metrics_nblk(N)
    part = torch.empty(B * nblk * 12, device=x.device, dtype=torch.float32)
    out = torch.empty(B, 12, device=x.device, dtype=torch.float64)
    _lib.call("msu_seg_metrics", ops._dt(x), ops._p(x), ops._p(lab), B, N, float(threshold), ops._p(part), nblk,
              ops._p(out), ops._s(x))
    return out.cpu()


def metrics_from_sums(row):
    """One image's metrics from its ``image_sums`` row (reference formulas, see module doc)."""
    c = {k: float(v) for k, v in zip(COLS, row.tolist())}
    tp, fp, fn, tn = (int(round(c[k])) for k in ("tp", "fp", "fn", "tn"))
    total = tp + fp + fn + tn
    if total <= 0:
        raise ValueError(f"metric calculation failed because total = {total}")
    m = {"tp": tp, "fp": fp, "fn": fn, "tn": tn, "accuracy": (tp + tn) / total,
         "confusion_matrix_bin": [[tp, fp], [fn, tn]],
         "confusion_matrix_soft": [[c["inter"], c["soft_fp"]], [c["soft_fn"], c["soft_tn"]]],
         "real": c["sum_g"] == 0.0}
    if m["real"]:
        m["fpr"] = fp / (fp + tn)
        return m
    m["bin_dice"] = 2.0 * tp / (2 * tp + fp + fn) if (2 * tp + fp + fn) > 0 else 0.0
    m["bin_iou"] = tp / (tp + fp + fn)
    m["recall"] = tp / (tp + fn) if (tp + fn) > 0 else 0.0
    m["precision"] = tp / (tp + fp) if (tp + fp) > 0 else 0.0
    m["bin_f1"] = 2 * (m["precision"] * m["recall"]) / (m["precision"] + m["recall"] + SMOOTH)
    # sum(g^2) == sum(g) for a binary ground truth
    m["soft_dice"] = (2.0 * c["inter"] + SMOOTH) / (c["sum_p2"] + c["sum_g"] + SMOOTH)
    m["soft_iou"] = (c["inter"] + SMOOTH) / (c["sum_p"] + c["sum_g"] - c["inter"] + SMOOTH)
    return m


def batch_metrics(logits, labels, threshold=0.5):
    """List of per-image metric dicts for a batch (one GPU pass)."""
    return [metrics_from_sums(r) for r in image_sums(logits, labels, threshold)]


def summarize(per_image):
    """Epoch summary of ``calculate_metrics`` (:152-180): mean soft Dice / IoU and binary
    metrics over fake images, mean FPR over real images, Score = soft Dice - 10 * FPR."""
    fake = [m for m in per_image if not m["real"]]
    real = [m for m in per_image if m["real"]]

    def mean(ms, k):
        return sum(m[k] for m in ms) / len(ms) if ms else float("nan")

    out = {k: mean(fake, k) for k in ("soft_dice", "soft_iou", "bin_dice", "bin_iou", "recall", "precision",
                                      "bin_f1", "accuracy")}
    out["mean_fpr"] = mean(real, "fpr")
    out["accuracy_all"] = mean(per_image, "accuracy")
    out["score"] = out["soft_dice"] - 10.0 * out["mean_fpr"]
    out["n_fake"], out["n_real"] = len(fake), len(real)
    return out


@torch.no_grad()
def evaluate(model, batches, threshold=0.5, amp_dtype=torch.bfloat16):
    """Run ``model`` in eval mode over ``(images, labels)`` batches on the GPU and summarise
    (the metric part of ``calculate_metrics``; no CSV / checkpoint side effects)."""
    model.eval()
    per_image = []
    for images, labels in batches:
        with torch.autocast("cuda", dtype=amp_dtype, enabled=amp_dtype != torch.float32):
            logits = model(images)
        per_image += batch_metrics(logits, labels, threshold)
    return summarize(per_image)
