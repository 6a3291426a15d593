"""Oracle: validation metric formulas (TEST INFRASTRUCTURE ONLY).

Restates ``scripts/validation_functions.py``:

* ``calculate_metrics_fake`` ``:247-309``: binary TP/FP/FN/TN at ``pred > threshold``
  vs ``gt = label > 0``; medpy ``dc``/``jc``/``recall``/``precision`` (medpy is absent
  here; its published definitions are restated: dc = 2|A^B|/(|A|+|B|) (0 if both empty),
  jc = |A^B|/|A v B| (1 if both empty... medpy returns 0 for an empty union? -- see note),
  recall = tp/(tp+fn), precision = tp/(tp+fp), 0 when the denominator is 0);
  soft Dice = (2*sum(p*g)+1e-8)/(sum(p^2)+sum(g^2)+1e-8) (``:300-301``); soft IoU =
  (sum(p*g)+1e-8)/(sum(p)+sum(g)-sum(p*g)+1e-8) (``:304``).
* ``calculate_metrics_real`` ``:214-244``: FPR = fp/(fp+tn).
* ``Score = mean_soft_dice - 10*mean_FPR`` (``:180``).

medpy note: medpy 0.4/0.5 ``jc`` divides by the union without a guard and ``dc`` returns
0.0 when both masks are empty; parity for those degenerate cases is unpinned.
"""
import torch


def soft_counts(logits, label, threshold=0.5):
    p = torch.sigmoid(logits.float()).reshape(-1)
    g = (label.reshape(-1) > 0).float()
    pb = (p > threshold)
    gb = g > 0
    return dict(
        inter=float((p * g).sum()), sum_p2=float((p * p).sum()), sum_g2=float((g * g).sum()),
        sum_p=float(p.sum()), sum_g=float(g.sum()),
        tp=int((pb & gb).sum()), fp=int((pb & ~gb).sum()),
        fn=int((~pb & gb).sum()), tn=int((~pb & ~gb).sum()),
        soft_fp=float(((1 - g) * p).sum()), soft_fn=float((g * (1 - p)).sum()),
        soft_tn=float(((1 - p) * (1 - g)).sum()))


def image_metrics(logits, label, threshold=0.5, smooth=1e-8):
    c = soft_counts(logits, label, threshold)
    tp, fp, fn, tn = c["tp"], c["fp"], c["fn"], c["tn"]
    out = dict(c)
    out["soft_dice"] = (2.0 * c["inter"] + smooth) / (c["sum_p2"] + c["sum_g2"] + smooth)
    out["soft_iou"] = (c["inter"] + smooth) / (c["sum_p"] + c["sum_g"] - c["inter"] + smooth)
    out["accuracy"] = (tp + tn) / (tp + tn + fp + fn)
    out["bin_dice"] = 2.0 * tp / (2 * tp + fp + fn) if (2 * tp + fp + fn) > 0 else 0.0
    out["bin_iou"] = tp / (tp + fp + fn) if (tp + fp + fn) > 0 else 0.0
    out["recall"] = tp / (tp + fn) if (tp + fn) > 0 else 0.0
    out["precision"] = tp / (tp + fp) if (tp + fp) > 0 else 0.0
    out["fpr"] = fp / (fp + tn) if (fp + tn) > 0 else 0.0
    return out
