"""Host half of the GPU augmentation: per-sample draws and their uint8 LUTs.

The reference augments each sample on the CPU inside a DataLoader worker
(``dataset/dataset.py:20-95``: ``RandomGenerator`` = albumentations Compose + flip + /255).
Here the host only draws *what* to do to each sample and builds the 256-entry uint8 tables the
way albumentations 1.x builds them (same numpy dtypes and operation order, so the tables are
the library's); ``msu_augment_batch`` (``csrc/augment.hip``) then applies a whole batch in
one HBM pass.  Table layout per sample: ``[5, 256]`` u8 -- 0 brightness/contrast, 1 hue,
2 saturation, 3 value, 4 gamma.

Draw distributions (the reference's parameters, ``dataset.py:26-34, :54, :58``):

* the Compose runs with probability 0.9 (``random.random() > 0.1``) when ``transform``;
* ToGray p 0.05; RandomBrightnessContrast p 0.8, alpha = 1 + U(-.1, .1), beta = U(-.1, .1);
  HueSaturationValue p 0.8, shifts U(-4, 4), U(-20, 20), U(-2, 2) (skipped when all are 0,
  as albumentations does);
* OneOf p 0.7 choosing by the children's p (1.0 : 0.5): RandomGamma with gamma =
  U(90, 110) / 100, or GaussianBlur with ksize = randrange(3, 6) made odd as albumentations
  1.x does (4 -> 5: P(3) = 1/3, P(5) = 2/3) and sigma 0;
* horizontal flip p 0.5 when ``random_flip_flag``.

RNG: each sample gets its own ``random.Random`` keyed by (seed, epoch, dataset index), so a
sample's augmentation does not depend on how batches are spread over threads or ranks (the
reference's draws depend on its DataLoader worker assignment, ``trainer.py:449-453``, so its
exact random stream is not reproducible per sample anyway).
"""
import random

import numpy as np

GRAY, BC, HSV, GAMMA, FLIP = 1, 2, 4, 8, 16
N_LUT = 5


def identity_luts():
    return np.tile(np.arange(256, dtype=np.uint8), (N_LUT, 1))


def bc_lut(alpha, beta):
    """albumentations 1.x ``_brightness_contrast_adjust_uint`` (beta_by_max=True)."""
    lut = np.arange(0, 256).astype("float32")
    if alpha != 1:
        lut *= alpha
    if beta != 0:
        lut += beta * 255
    return np.clip(lut, 0, 255).astype(np.uint8)


def hsv_luts(hue_shift, sat_shift, val_shift):
    """albumentations 1.x ``_shift_hsv_uint8``: hue mod 180, saturation / value clipped."""
    base = np.arange(0, 256, dtype=np.int16)
    hue = np.mod(base + hue_shift, 180).astype(np.uint8) if hue_shift != 0 else base.astype(np.uint8)
    sat = np.clip(base + sat_shift, 0, 255).astype(np.uint8) if sat_shift != 0 else base.astype(np.uint8)
    val = np.clip(base + val_shift, 0, 255).astype(np.uint8) if val_shift != 0 else base.astype(np.uint8)
    return hue, sat, val


def gamma_lut(gamma):
    """albumentations 1.x ``gamma_transform`` for uint8."""
    table = (np.arange(0, 256.0 / 255, 1.0 / 255) ** gamma) * 255
    return table[:256].astype(np.uint8)


def sample_rng(seed, epoch, index):
    """Per-(seed, epoch, sample) draw stream: the three keys sit in disjoint 64-bit fields
    (random.Random hashes arbitrarily long ints), so no (epoch, index) pair aliases another."""
    key = ((int(seed) & (2**64 - 1)) << 128) | ((int(epoch) & (2**64 - 1)) << 64) | (int(index) & (2**64 - 1))
    return random.Random(key)


def draw(rng, transform=True, flip=False):
    """One sample's operations: (op bits, blur ksize 0/3/5, luts [5, 256] u8)."""
    luts = identity_luts()
    op, ks = 0, 0
    if rng.random() > 0.1 and transform:
        if rng.random() < 0.05:
            op |= GRAY
        if rng.random() < 0.8:
            alpha = 1.0 + rng.uniform(-0.1, 0.1)
            beta = 0.0 + rng.uniform(-0.1, 0.1)
            luts[0] = bc_lut(alpha, beta)
            op |= BC
        if rng.random() < 0.8:
            hue = rng.uniform(-4, 4)
            sat = rng.uniform(-20, 20)
            val = rng.uniform(-2, 2)
            if hue != 0 or sat != 0 or val != 0:
                luts[1], luts[2], luts[3] = hsv_luts(hue, sat, val)
                op |= HSV
        if rng.random() < 0.7:
            if rng.random() < 1.0 / 1.5:
                luts[4] = gamma_lut(rng.uniform(90, 110) / 100.0)
                op |= GAMMA
            else:
                k = rng.randrange(3, 6)
                ks = k if k % 2 == 1 else (k + 1) % 6
    if flip and rng.random() > 0.5:
        op |= FLIP
    return op, ks, luts
