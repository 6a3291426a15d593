"""Datasets and per-sample transforms with the reference's interface
(``dataset/dataset.py``: ``random_flip`` :13-16, ``RandomGenerator`` :20-95,
``DataPrepartion`` :97-119, ``SegArtifact_dataset`` :123-170,
``SegArtifact_no_label_dataset`` :173-211).

File layout, lookup order and exceptions are the reference's: ``<base>/real_images/<name>.png``
first, then ``fake_images``; labels ``<name>_mask.png`` in ``real_labels`` / ``fake_labels``;
``FileNotFoundError`` with the same messages.  PNGs are decoded with PIL (as the reference
does) to uint8; everything after the decode -- augmentation, flip, /255, label threshold,
HWC -> CHW -- runs in ``msu_augment_batch`` on the GPU.  ``RandomGenerator`` /
``DataPrepartion`` called on one sample therefore return *device* tensors (the reference
returns CPU tensors that its trainer moves with ``.cuda()``, a no-op here); the batched path
that keeps up with training is ``dataset.loader.GpuBatchLoader``.
"""
import os
import random

import numpy as np
import torch
from PIL import Image
from torch.utils.data import Dataset

from .. import _lib
from . import augment


def random_flip(image, label):
    """Horizontal flip of a [H, W, ...] image and its [H, W] label (numpy, ``:13-16``)."""
    return np.flip(image, axis=1).copy(), np.flip(label, axis=1).copy()


def augment_batch(img_u8, lbl_u8, ops=None, luts=None):
    """Device batch: img [B, H, W, 3] u8, label [B, H, W] u8 or None, ops [B, 2] i32 and
    luts [B, 5, 256] u8 (or both None: normalisation only) -> (image f32 [B, 3, H, W],
    label f32 [B, H, W] or None), launched on the current stream of img's device."""
    if not img_u8.is_cuda:
        raise RuntimeError("augment_batch needs tensors on a HIP device (no CPU fallback)")
    if img_u8.dtype != torch.uint8 or img_u8.dim() != 4 or img_u8.shape[-1] != 3:
        raise ValueError(f"image batch must be uint8 [B, H, W, 3], got {tuple(img_u8.shape)} {img_u8.dtype}")
    B, H, W, _ = img_u8.shape
    img_u8 = img_u8.contiguous()
    if lbl_u8 is not None:
        if lbl_u8.dtype != torch.uint8 or tuple(lbl_u8.shape) != (B, H, W):
            raise ValueError(f"label batch must be uint8 [B, H, W] = {(B, H, W)}, got {tuple(lbl_u8.shape)}")
        lbl_u8 = lbl_u8.contiguous()
    if (ops is None) != (luts is None):
        raise ValueError("ops and luts go together")
    if ops is not None:
        if tuple(ops.shape) != (B, 2) or ops.dtype != torch.int32:
            raise ValueError(f"ops must be int32 [B, 2], got {tuple(ops.shape)} {ops.dtype}")
        if tuple(luts.shape) != (B, augment.N_LUT, 256) or luts.dtype != torch.uint8:
            raise ValueError(f"luts must be uint8 [B, 5, 256], got {tuple(luts.shape)} {luts.dtype}")
        ops, luts = ops.contiguous(), luts.contiguous()
    dev = img_u8.device
    out = torch.empty(B, 3, H, W, device=dev, dtype=torch.float32)
    out_l = None if lbl_u8 is None else torch.empty(B, H, W, device=dev, dtype=torch.float32)

    def p(t):
        return None if t is None else t.data_ptr()

    _lib.call("msu_augment_batch", p(img_u8), p(lbl_u8), p(ops), p(luts), p(out), p(out_l), B, H, W,
              torch._C._cuda_getCurrentRawStream(dev.index))
    return out, out_l


def _device():
    return torch.device("cuda", torch.cuda.current_device())


class RandomGenerator(object):
    """``RandomGenerator(output_size, random_flip_flag=False, transform=True)`` (``:20-95``)."""

    def __init__(self, output_size, random_flip_flag=False, transform=True):
        self.output_size = output_size
        self.random_flip_flag = random_flip_flag
        self.transform = True if transform is True else None

    def draw(self, rng):
        """(op bits, blur ksize, luts [5, 256]) for one sample from ``rng``."""
        return augment.draw(rng, transform=self.transform is not None, flip=self.random_flip_flag)

    def check(self, image):
        H, W = image.shape[:2]
        if (H, W) != tuple(self.output_size):
            raise ValueError(f"RandomGenerator: Wrong image size: {H, W}")
        if image.ndim != 3 or image.shape[2] != 3:
            raise ValueError("RandomGenerator: Image does not have 3 channels")

    def __call__(self, sample):
        image = np.array(sample['image'], dtype=np.uint8)
        label = np.array(sample['label'], dtype=np.uint8)
        self.check(image)
        op, ks, luts = self.draw(random)  # the reference draws from the global `random` stream
        dev = _device()
        img_d = torch.from_numpy(image).to(dev)[None]
        lbl_d = torch.from_numpy(label).to(dev)[None]
        ops_d = torch.tensor([[op, ks]], dtype=torch.int32, device=dev)
        luts_d = torch.from_numpy(luts).to(dev)[None]
        x, y = augment_batch(img_d, lbl_d, ops_d, luts_d)
        return {'image': x[0], 'label': y[0]}


class DataPrepartion(object):
    """Unlabelled normalisation (``:97-119``): image f32 [3, H, W] = u8 / 255."""

    def __init__(self, output_size):
        self.output_size = output_size

    def check(self, image):
        H, W = image.shape[:2]
        if (H, W) != tuple(self.output_size):
            raise ValueError(f"RandomGenerator: Wrong image size: {H, W}")
        if image.ndim != 3 or image.shape[2] != 3:
            raise ValueError("RandomGenerator: Image does not have 3 channels")

    def __call__(self, sample):
        image = np.array(sample['image'], dtype=np.uint8)
        self.check(image)
        x, _ = augment_batch(torch.from_numpy(image).to(_device())[None], None)
        return {'image': x[0]}


class _ListDataset(Dataset):
    def __init__(self, base_dir, list_dir, split, transform=None):
        self.transform = transform
        self.split = split
        with open(os.path.join(list_dir, self.split + '.txt'), 'r', encoding='utf-8') as f:
            self.sample_list = [ln.strip() for ln in f if ln.strip()]
        self.data_dir = base_dir

    def __len__(self):
        return len(self.sample_list)

    def _path(self, kind, name, suffix=""):
        return os.path.join(self.data_dir, kind, name + suffix + ".png")


class SegArtifact_dataset(_ListDataset):
    """Labelled real / fake faces (``:123-170``)."""

    with_labels = True

    def paths(self, idx):
        name = self.sample_list[idx]
        for kind in ("real", "fake"):
            img = self._path(kind + "_images", name)
            if os.path.exists(img):
                lab = self._path(kind + "_labels", name, "_mask")
                if not os.path.exists(lab):
                    raise FileNotFoundError(f"Label {name} not found in {kind}_labels")
                return img, lab
        raise FileNotFoundError(f"Sample {name} not found in real_images/ or fake_images/")

    def read_raw(self, idx):
        """Decoded uint8 (image [H, W, 3], label [H, W]) of sample ``idx``."""
        img_p, lab_p = self.paths(idx)
        with Image.open(img_p) as im, Image.open(lab_p) as lb:
            return np.asarray(im.convert("RGB")), np.asarray(lb.convert("L"))

    def __getitem__(self, idx):
        img_p, lab_p = self.paths(idx)
        sample = {'image': Image.open(img_p).convert("RGB"), 'label': Image.open(lab_p).convert("L")}
        if self.transform:
            sample = self.transform(sample)
        sample['case_name'] = self.sample_list[idx].strip('\n')
        return sample


class SegArtifact_no_label_dataset(_ListDataset):
    """Unlabelled images (``:173-211``)."""

    with_labels = False

    def paths(self, idx):
        name = self.sample_list[idx]
        for kind in ("real", "fake"):
            img = self._path(kind + "_images", name)
            if os.path.exists(img):
                return img, None
        raise FileNotFoundError(f"Sample {name} not found in real_images/ or fake_images/")

    def read_raw(self, idx):
        img_p, _ = self.paths(idx)
        with Image.open(img_p) as im:
            return np.asarray(im.convert("RGB")), None

    def __getitem__(self, idx):
        img_p, _ = self.paths(idx)
        sample = {'image': Image.open(img_p).convert("RGB")}
        if self.transform:
            sample = self.transform(sample)
        sample['case_name'] = self.sample_list[idx].strip('\n')
        return sample
