"""Synthetic StyleGAN2-artifact batches, generated directly in HBM.

Stands in for ``dataset/dataset.py`` + ``scripts/batch_data_loader_V2.py`` (no dataset or
network here):
* images: uniform RGB quantised to k/255 (PNG / 255 normalisation, ``dataset.py:62``),
  f32 [B, 3, H, W];
* labels: f32 {0, 1} [B, H, W]; 60 % "fake" samples carry 1-8 filled ellipses covering
  ~0.5-5 % of the pixels, biased towards the lower third and the face sides (the artifact
  location prior of ``dataset/artifact_distibution``); 40 % "real" samples are empty
  (``real_ratio`` 0.4, ``trainer.py:208``); at least one fake per batch
  (``batch_data_loader_V2.py:52-69``).
"""
import math

import torch


def synthetic_batch(batch, img_size, device, seed, fake_ratio=0.6):
    g = torch.Generator(device="cpu").manual_seed(seed)
    H = W = img_size
    img = torch.randint(0, 256, (batch, 3, H, W), generator=g, dtype=torch.int32)
    img = (img.float() / 255.0).to(device)
    fake = (torch.rand(batch, generator=g) < fake_ratio).tolist()
    if not any(fake):
        fake[0] = True
    labels = torch.zeros(batch, H, W, device=device)
    yy = torch.arange(H, device=device, dtype=torch.float32).view(H, 1)
    xx = torch.arange(W, device=device, dtype=torch.float32).view(1, W)
    for b in range(batch):
        if not fake[b]:
            continue
        n = int(torch.randint(1, 9, (1,), generator=g))
        target_frac = 0.005 + 0.045 * float(torch.rand(1, generator=g))
        area = target_frac * H * W / n
        for _ in range(n):
            r = math.sqrt(area / math.pi) * (0.6 + 0.8 * float(torch.rand(1, generator=g)))
            aspect = 0.5 + float(torch.rand(1, generator=g))
            ry, rx = r * aspect, r / aspect
            cy = H * (0.45 + 0.55 * float(torch.rand(1, generator=g)))  # lower part of the face
            side = float(torch.rand(1, generator=g))
            cx = W * (0.1 + 0.25 * side if torch.rand(1, generator=g) < 0.5 else 0.9 - 0.25 * side)
            m = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
            labels[b][m] = 1.0
    return img, labels


def batch_pool(n, batch, img_size, device, seed):
    """``n`` resident batches (inputs stay in HBM across the timed region)."""
    return [synthetic_batch(batch, img_size, device, seed + 7919 * i) for i in range(n)]
