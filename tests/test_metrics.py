"""Validation metrics (scripts/validation_functions.py:37-309): the GPU reduction
(msu_seg_metrics) and the host formulas (validation.metrics_from_sums) against the oracle
restatement (oracle/metrics.py).

Parity: binary confusion counts exact; soft sums within 1e-5 relative (f32 partials,
double totals, different summation order than torch).  medpy's degenerate cases (both
masks empty) are "parity unpinned" (medpy is not installed; its published definitions are
restated in oracle/metrics.py)."""
import pytest
import torch

from oracle import metrics as om


def _case(B, H, W, seed, empty=(), full=()):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, 1, H, W, generator=g) * 3
    labels = (torch.rand(B, H, W, generator=g) < 0.05).float()
    for b in empty:
        labels[b] = 0
    for b in full:
        labels[b] = 1
    return logits, labels


def _sums_row(c):
    from semantic_segmentation_of_stylegan2_artifacts_amd.validation import COLS
    vals = {"inter": c["inter"], "sum_p2": c["sum_p2"], "sum_g": c["sum_g"], "sum_p": c["sum_p"],
            "soft_fp": c["soft_fp"], "soft_fn": c["soft_fn"], "soft_tn": c["soft_tn"],
            "tp": c["tp"], "fp": c["fp"], "fn": c["fn"], "tn": c["tn"]}
    return torch.tensor([vals[k] for k in COLS] + [0.0], dtype=torch.float64)


def test_host_formulas_match_oracle():
    """metrics_from_sums on oracle-computed sums reproduces the oracle's per-image metrics."""
    from semantic_segmentation_of_stylegan2_artifacts_amd.validation import metrics_from_sums, summarize
    logits, labels = _case(4, 32, 40, 0, empty=(1,))
    per = []
    for b in range(4):
        ref = om.image_metrics(logits[b], labels[b])
        m = metrics_from_sums(_sums_row(om.soft_counts(logits[b], labels[b])))
        per.append(m)
        assert m["real"] == (b == 1)
        assert m["accuracy"] == pytest.approx(ref["accuracy"])
        if m["real"]:
            assert m["fpr"] == pytest.approx(ref["fpr"])
        else:
            for k in ("soft_dice", "soft_iou", "bin_dice", "bin_iou", "recall", "precision"):
                assert m[k] == pytest.approx(ref[k], rel=1e-12, abs=1e-15), k
    s = summarize(per)
    assert s["n_real"] == 1 and s["n_fake"] == 3
    assert s["score"] == pytest.approx(s["soft_dice"] - 10 * s["mean_fpr"])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gpu_metrics_match_oracle(dtype):
    from semantic_segmentation_of_stylegan2_artifacts_amd.validation import image_sums, COLS
    logits, labels = _case(5, 96, 160, 1, empty=(0,), full=(3,))
    logits = logits.to(dtype)
    sums = image_sums(logits.cuda(), labels.cuda())
    for b in range(5):
        c = om.soft_counts(logits[b].float(), labels[b])
        row = dict(zip(COLS, sums[b].tolist()))
        for k in ("tp", "fp", "fn", "tn"):
            assert row[k] == c[k], (b, k, row[k], c[k])
        for k in ("inter", "sum_p2", "sum_p", "soft_fp", "soft_fn", "soft_tn"):
            assert row[k] == pytest.approx(c[k], rel=1e-5, abs=1e-6), (b, k)
        assert row["sum_g"] == c["sum_g2"]


@pytest.mark.gpu
def test_gpu_metrics_1024_soft_dice_within_1e3():
    """At the bench resolution the GPU soft Dice equals the oracle's within 1e-3."""
    from semantic_segmentation_of_stylegan2_artifacts_amd.validation import batch_metrics
    logits, labels = _case(2, 1024, 1024, 2)
    per = batch_metrics(logits.cuda(), labels.cuda())
    for b in range(2):
        ref = om.image_metrics(logits[b], labels[b])
        assert abs(per[b]["soft_dice"] - ref["soft_dice"]) <= 1e-3
        assert per[b]["tp"] == ref["tp"] and per[b]["fp"] == ref["fp"]
