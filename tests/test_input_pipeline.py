"""CPU: the input pipeline's host half -- BatchPatternSampler against the reference's own
batches (tests/golden/batch_sampler.json, made by importing the reference), the epoch plan of
trainer.py:195-237, the albumentations LUT builders against the oracle restatement, the draw
distributions, the cv2 conversion known answers of the oracle, and the dataset's file layout
and errors (dataset/dataset.py:123-211).  The GPU kernel itself: test_gpu_input_pipeline.py."""
import json
import os
import random

import numpy as np
import pytest
import torch
from PIL import Image
from torch.utils.data import ConcatDataset, Subset

from oracle import augment as oa
from semantic_segmentation_of_stylegan2_artifacts_amd.dataset import augment as aug
from semantic_segmentation_of_stylegan2_artifacts_amd.dataset.dataset import (SegArtifact_dataset,
                                                                              SegArtifact_no_label_dataset)
from semantic_segmentation_of_stylegan2_artifacts_amd.dataset.loader import (GpuBatchLoader, epoch_plan, num_real_for,
                                                                             real_ratio_for_epoch, resolve)
from semantic_segmentation_of_stylegan2_artifacts_amd.scripts.batch_data_loader_V2 import BatchPatternSampler

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "batch_sampler.json")


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as f:
        return json.load(f)


# ------------------------------------------------------------------ sampler (reference-pinned)
def test_sampler_matches_reference_batches(gold):
    for c in gold["cases"]:
        fake = list(range(c["n_fake"]))
        real = list(range(c["n_fake"], c["n_fake"] + c["n_real"]))
        s = BatchPatternSampler(fake, real, (len(fake) + len(real)) // 2, 2, c["epoch"])
        assert len(s) == c["len"]
        assert [list(b) for b in s] == c["passes"][0], c
        assert [list(b) for b in s] == c["passes"][1], c  # pattern reshuffled in place
        s.set_epoch(c["epoch"] + 5)
        assert [list(b) for b in s] == c["passes"][2], c
        for b in c["passes"][0]:
            assert any(i < c["n_fake"] for i in b)  # at least one fake per batch


def test_sampler_errors_match_reference(gold):
    for e in gold["errors"]:
        if e["error"] is None:
            BatchPatternSampler(*e["args"])
            continue
        with pytest.raises(ValueError) as ex:
            BatchPatternSampler(*e["args"])
        assert str(ex.value) == e["error"]


def test_randperm_subset_matches_reference_generator(gold):
    for p in gold["randperm"]:
        g = torch.Generator().manual_seed(p["seed"] + p["epoch"])
        assert torch.randperm(p["total"], generator=g).tolist() == p["perm"]


# ------------------------------------------------------------------ epoch plan
def test_real_ratio_schedule():
    expect = {0: 0.1, 8: 0.1, 9: 0.13, 14: 0.28, 19: 0.43, 20: 0.4, 29: 0.4, 30: 0.2, 34: 0.2, 35: 0.4, 80: 0.4}
    for e, r in expect.items():
        assert real_ratio_for_epoch(e, True) == pytest.approx(r, abs=1e-12), e
        assert real_ratio_for_epoch(e, False) == 0.4


def test_num_real_rule():
    assert num_real_for(800, 1000, 0.4) == 532  # int(533.33) = 533 -> odd total -> 532
    assert num_real_for(800, 1000, 0.1) == 88
    assert (num_real_for(801, 1000, 0.4) + 801) % 2 == 0
    with pytest.raises(ValueError):
        num_real_for(800, 100, 0.4)


class _Idx(torch.utils.data.Dataset):
    def __init__(self, n, tag):
        self.n, self.tag = n, tag

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return (self.tag, i)


def test_epoch_plan_and_resolve(gold):
    fake, real = _Idx(10, "fake"), _Idx(30, "real")
    mixed, sampler, ratio, idx_real = epoch_plan(fake, real, epoch_num=3, seed=1234, dynamic_loader=False)
    assert ratio == 0.4 and len(idx_real) == num_real_for(10, 30, 0.4)
    g = torch.Generator().manual_seed(1234 + 3)
    assert idx_real.tolist() == torch.randperm(30, generator=g)[:len(idx_real)].tolist()
    assert len(mixed) == 10 + len(idx_real) and sampler.epoch == 4
    for batch in sampler:
        tags = [resolve(mixed, i)[0].tag for i in batch]
        assert "fake" in tags
        for i in batch:
            ds, j = resolve(mixed, i)
            assert ds[j] == mixed[i]


def test_steps_split_over_ranks():
    fake, real = list(range(12)), list(range(12, 20))
    all_b = [list(b) for b in BatchPatternSampler(fake, real, 10, 2, 1)]
    got = []
    for r in range(2):  # each rank holds its own sampler of the same epoch (same batches)
        s = BatchPatternSampler(fake, real, 10, 2, 1)
        ld = GpuBatchLoader(None, s, device="cuda:0", rank=r, world_size=2, batches_per_step=2)
        got.append(list(ld.steps()))
        assert len(got[r]) == len(ld) == 2
    for k in range(2):
        assert got[0][k] == all_b[4 * k] + all_b[4 * k + 1]
        assert got[1][k] == all_b[4 * k + 2] + all_b[4 * k + 3]


# ------------------------------------------------------------------ LUTs and draws
def test_lut_builders_match_oracle():
    rng = random.Random(5)
    for _ in range(200):
        a, b = 1 + rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1)
        assert np.array_equal(aug.bc_lut(a, b), oa.bc_lut(a, b))
        h, s, v = rng.uniform(-4, 4), rng.uniform(-20, 20), rng.uniform(-2, 2)
        hl, sl, vl = aug.hsv_luts(h, s, v)
        assert np.array_equal(hl, oa.hue_lut(h)) and np.array_equal(sl, oa.clip_lut(s))
        assert np.array_equal(vl, oa.clip_lut(v))
        g = rng.uniform(90, 110) / 100
        assert np.array_equal(aug.gamma_lut(g), oa.gamma_lut(g))
    assert np.array_equal(aug.bc_lut(1, 0), np.arange(256, dtype=np.uint8))
    assert aug.gamma_lut(1.0)[255] == 255


def test_draw_distributions():
    n = 40000
    rng = random.Random(11)
    cnt = dict(gray=0, bc=0, hsv=0, gamma=0, k3=0, k5=0, flip=0)
    for _ in range(n):
        op, ks, _ = aug.draw(rng, transform=True, flip=True)
        cnt["gray"] += bool(op & aug.GRAY)
        cnt["bc"] += bool(op & aug.BC)
        cnt["hsv"] += bool(op & aug.HSV)
        cnt["gamma"] += bool(op & aug.GAMMA)
        cnt["k3"] += ks == 3
        cnt["k5"] += ks == 5
        cnt["flip"] += bool(op & aug.FLIP)
        assert not (op & aug.GAMMA and ks)  # OneOf
    expect = dict(gray=.9 * .05, bc=.9 * .8, hsv=.9 * .8, gamma=.9 * .7 * 2 / 3, k3=.9 * .7 / 3 / 3,
                  k5=.9 * .7 / 3 * 2 / 3, flip=.5)
    for k, p in expect.items():
        assert abs(cnt[k] / n - p) < 4 * np.sqrt(p * (1 - p) / n) + 1e-3, (k, cnt[k] / n, p)
    # transform=False: normalisation only; flip still drawn
    op, ks, luts = aug.draw(random.Random(0), transform=False, flip=False)
    assert op == 0 and ks == 0 and np.array_equal(luts, aug.identity_luts())


def test_sample_rng_is_keyed():
    a = aug.draw(aug.sample_rng(1, 2, 3), True, True)
    b = aug.draw(aug.sample_rng(1, 2, 3), True, True)
    assert a[0] == b[0] and a[1] == b[1] and np.array_equal(a[2], b[2])
    ops = {aug.draw(aug.sample_rng(1, 2, i), True, True)[0] for i in range(64)}
    assert len(ops) > 4
    # indices >= 2^20 must not alias (epoch, index) pairs of other epochs
    big = 1 << 20
    sig = lambda e, i: aug.sample_rng(1, e, i).getrandbits(64)  # noqa: E731
    assert sig(0, big) != sig(1, 0) and sig(0, big + 5) != sig(1, 5) and sig(3, 7) != sig(7, 3)


# ------------------------------------------------------------------ oracle known answers (cv2 8U)
def test_oracle_cv2_known_answers():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [255, 255, 0]]], np.uint8)
    assert oa.rgb2gray(px)[0, :, 0].tolist() == [76, 150, 29, 255, 0, 226]
    hsv = oa.rgb2hsv(px)
    assert hsv[0].tolist() == [[0, 255, 255], [60, 255, 255], [120, 255, 255], [0, 0, 255], [0, 0, 0],
                               [30, 255, 255]]
    assert np.array_equal(oa.hsv2rgb(hsv), px)
    rng = np.random.default_rng(0)
    x = rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)
    back = oa.hsv2rgb(oa.rgb2hsv(x)).astype(int)
    assert np.abs(back - x).max() <= 8 and np.abs(back - x).mean() < 1  # 8-bit HSV (H in 2-degree steps) is lossy


def test_oracle_blur():
    x = np.full((9, 11, 3), 77, np.uint8)
    for k in (3, 5):
        assert np.array_equal(oa.gaussian_blur(x, k), x)
    imp = np.zeros((7, 7, 3), np.uint8)
    imp[3, 3] = 255
    out = oa.gaussian_blur(imp, 3)[..., 0]
    assert out[3, 3] == (4 * 255 + 8) >> 4 and out[2, 3] == (2 * 255 + 8) >> 4 and out[2, 2] == (255 + 8) >> 4


# ------------------------------------------------------------------ dataset files
def _write_set(root, names, kind, size=(12, 10), label=True, seed=0):
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, kind + "_images"), exist_ok=True)
    os.makedirs(os.path.join(root, kind + "_labels"), exist_ok=True)
    out = {}
    for n in names:
        im = rng.integers(0, 256, (size[0], size[1], 3), dtype=np.uint8)
        lb = (rng.random(size) > 0.7).astype(np.uint8) * 255
        Image.fromarray(im).save(os.path.join(root, kind + "_images", n + ".png"))
        if label:
            Image.fromarray(lb).save(os.path.join(root, kind + "_labels", n + "_mask.png"))
        out[n] = (im, lb)
    return out


def test_dataset_layout_and_errors(tmp_path):
    root = str(tmp_path)
    real = _write_set(root, ["r0", "both"], "real", seed=1)
    fake = _write_set(root, ["f0", "both"], "fake", seed=2)
    _write_set(root, ["nolab"], "fake", label=False, seed=3)
    with open(os.path.join(root, "train.txt"), "w") as f:
        f.write("r0\nf0\n\nboth\nnolab\nmissing\n")
    ds = SegArtifact_dataset(root, root, "train")
    assert len(ds) == 5 and ds.sample_list[2] == "both"
    im, lb = ds.read_raw(0)
    assert np.array_equal(im, real["r0"][0]) and np.array_equal(lb, real["r0"][1])
    im, lb = ds.read_raw(1)
    assert np.array_equal(im, fake["f0"][0])
    im, _ = ds.read_raw(2)
    assert np.array_equal(im, real["both"][0])  # real_images is looked up first
    s = ds[1]
    assert s["case_name"] == "f0" and s["image"].mode == "RGB" and s["label"].mode == "L"
    with pytest.raises(FileNotFoundError, match="Label nolab not found in fake_labels"):
        ds.read_raw(3)
    with pytest.raises(FileNotFoundError, match="Sample missing not found in real_images/ or fake_images/"):
        ds[4]
    nl = SegArtifact_no_label_dataset(root, root, "train")
    im, lb = nl.read_raw(3)
    assert lb is None and im.shape == (12, 10, 3)
    assert nl[0]["case_name"] == "r0"
    # wrappers resolve to the base dataset
    mixed = ConcatDataset([Subset(ds, [2, 0]), ds])
    assert resolve(mixed, 1) == (ds, 0) and resolve(mixed, 3) == (ds, 1)
