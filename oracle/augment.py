"""Oracle: the reference's per-sample augmentation + normalisation (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` import this module, as the checker of ``msu_augment_batch`` and of the host
LUT builders in ``dataset/augment.py``.  numpy restatement of:

* ``dataset/dataset.py:20-95`` ``RandomGenerator`` / ``DataPrepartion``: the albumentations
  Compose (``:26-34``) -- ToGray(p .05), RandomBrightnessContrast(.1, .1, p .8),
  HueSaturationValue(4, 20, 2, p .8), OneOf([RandomGamma((90, 110)), GaussianBlur((3, 5),
  p .5)], p .7) -- gated by ``random.random() > 0.1`` (``:54``), then ``random_flip``
  (``:13-16``, ``:58-60``), ``image / 255`` in f32 (``:65``), ``label > 127`` (``:66``),
  HWC -> CHW (``:83``).
* albumentations and cv2 are absent from this container (and un-pinned by the reference: no
  requirements file), so their published uint8 algorithms are restated here -- albumentations
  1.x ``brightness_contrast_adjust`` / ``shift_hsv_uint8`` / ``gamma_transform`` /
  ``gaussian_blur`` and OpenCV 4's 8U kernels: ``COLOR_RGB2GRAY`` (fixed point, shift 14),
  ``RGB2HSV_b`` (integer tables, shift 12), ``HSV2RGB_b`` (f32 sector formula, cvRound),
  ``GaussianBlur`` with sigma 0 (the binomial small-kernel table, bit-exact fixed-point path,
  BORDER_REFLECT_101).  Against the libraries themselves this is *parity unpinned*; the
  known-answer checks in ``tests/test_input_pipeline.py`` (pure colours, cv2's documented
  grey weights) pin the conversions' published values.
"""
import numpy as np

F32 = np.float32


# ------------------------------------------------------------------ LUTs (albumentations 1.x)
def bc_lut(alpha, beta):
    """brightness_contrast_adjust, uint8, beta_by_max: clip(i * alpha + beta * 255) -> u8."""
    out = np.empty(256, np.uint8)
    for i in range(256):
        v = F32(i)
        if alpha != 1:
            v = F32(v * F32(alpha))
        if beta != 0:
            v = F32(v + F32(beta * 255))
        out[i] = int(min(max(v, F32(0)), F32(255)))  # astype(uint8) truncates
    return out


def hue_lut(shift):
    return np.array([int((i + shift) % 180) if shift != 0 else i for i in range(256)], np.uint8)


def clip_lut(shift):
    return np.array([int(min(max(i + shift, 0), 255)) if shift != 0 else i for i in range(256)], np.uint8)


def gamma_lut(gamma):
    # np.arange(0, 256/255, 1/255) holds i * (1/255), not i / 255
    return np.array([int(((i * (1.0 / 255)) ** gamma) * 255) for i in range(256)], np.uint8)


# ------------------------------------------------------------------ cv2 8U conversions
def rgb2gray(img):
    r, g, b = (img[..., c].astype(np.int32) for c in range(3))
    y = (r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14
    return np.repeat(y[..., None], 3, axis=-1).astype(np.uint8)


def _tables():
    i = np.arange(256, dtype=np.float64)
    with np.errstate(divide="ignore"):
        sdiv = np.where(i == 0, 0, np.rint((255 << 12) / i)).astype(np.int64)
        hdiv = np.where(i == 0, 0, np.rint((180 << 12) / (6.0 * i))).astype(np.int64)
    return sdiv, hdiv


def rgb2hsv(img):
    sdiv, hdiv = _tables()
    r, g, b = (img[..., c].astype(np.int64) for c in range(3))
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    s = (diff * sdiv[v] + (1 << 11)) >> 12
    h = np.where(v == r, g - b, np.where(v == g, b - r + 2 * diff, r - g + 4 * diff))
    h = (h * hdiv[diff] + (1 << 11)) >> 12
    h = np.where(h < 0, h + 180, h)
    return np.stack([np.clip(h, 0, 255), s, v], axis=-1).astype(np.uint8)


def hsv2rgb(hsv):
    inv = F32(1) / F32(255)
    h = hsv[..., 0].astype(F32)
    s = hsv[..., 1].astype(F32) * inv
    v = hsv[..., 2].astype(F32) * inv
    h = h * (F32(6) / F32(180))
    h = np.where(h >= F32(6), h - F32(6), h).astype(F32)
    sector = np.floor(h).astype(np.int64)
    h = (h - sector.astype(F32)).astype(F32)
    one = F32(1)
    tab = np.stack([v, v * (one - s), v * (one - s * h), v * (one - s * (one - h))], axis=-1)
    sd = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    idx = sd[sector]  # (b, g, r) tab indices
    bgr = np.take_along_axis(tab, idx, axis=-1)
    gray = (s == 0)[..., None]
    bgr = np.where(gray, np.repeat(v[..., None], 3, -1), bgr).astype(F32)
    out = np.clip(np.rint(bgr * F32(255)), 0, 255).astype(np.uint8)
    return out[..., ::-1].copy()  # -> r, g, b


def gaussian_blur(img, ksize):
    a = {3: np.array([1, 2, 1]), 5: np.array([1, 4, 6, 4, 1])}[ksize]
    shift = {3: 4, 5: 8}[ksize]
    r = ksize // 2
    H, W = img.shape[:2]
    p = np.pad(img.astype(np.int64), ((r, r), (r, r), (0, 0)), mode="reflect")  # = REFLECT_101
    acc = np.zeros(img.shape, np.int64)
    for dy in range(ksize):
        for dx in range(ksize):
            acc += a[dy] * a[dx] * p[dy:dy + H, dx:dx + W]
    return ((acc + (1 << (shift - 1))) >> shift).astype(np.uint8)


# ------------------------------------------------------------------ one sample
GRAY, BC, HSV, GAMMA, FLIP = 1, 2, 4, 8, 16


def augment_sample(img, label, op, ksize, luts):
    """img [H, W, 3] u8, label [H, W] u8 or None, op bits / blur ksize / luts [5, 256] as the
    host drew them -> (image f32 [3, H, W], label f32 [H, W] or None)."""
    x = img.copy()
    if op & GRAY:
        x = rgb2gray(x)
    if op & BC:
        x = luts[0][x]
    if op & HSV:
        hsv = rgb2hsv(x)
        hsv = np.stack([luts[1][hsv[..., 0]], luts[2][hsv[..., 1]], luts[3][hsv[..., 2]]], -1)
        x = hsv2rgb(hsv)
    if op & GAMMA:
        x = luts[4][x]
    if ksize:
        x = gaussian_blur(x, ksize)
    lab = label
    if op & FLIP:
        x = np.flip(x, axis=1)
        lab = None if label is None else np.flip(label, axis=1)
    image = (x.astype(F32) / F32(255.0)).transpose(2, 0, 1).copy()
    lab_f = None if lab is None else (lab > 127).astype(F32)
    return image, lab_f
