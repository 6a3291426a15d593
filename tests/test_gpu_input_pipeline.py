"""GPU: ``msu_augment_batch`` (the reference's per-sample RandomGenerator / DataPrepartion,
dataset/dataset.py:20-119) bit-exact against the numpy oracle (oracle/augment.py) for every
operation alone and in the combinations the host draws, on ragged sizes (tiles cut by the
image edge, reflect-101 borders on tiny images), with and without labels; and the
GpuBatchLoader end to end over PNG files (decode -> pinned upload -> kernel) = the oracle
applied to the decoded files with the same draws.  Integer / byte work: equality, no tolerance."""
import os
import random

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import augment as oa
from semantic_segmentation_of_stylegan2_artifacts_amd.dataset import augment as aug

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(imgs, lbls, ops_list):
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset.dataset import augment_batch
    img_d = torch.from_numpy(np.stack(imgs)).to(DEV)
    lbl_d = None if lbls is None else torch.from_numpy(np.stack(lbls)).to(DEV)
    if ops_list is None:
        x, y = augment_batch(img_d, lbl_d)
    else:
        ops = torch.tensor([[o, k] for o, k, _ in ops_list], dtype=torch.int32, device=DEV)
        luts = torch.from_numpy(np.stack([l for _, _, l in ops_list])).to(DEV)
        x, y = augment_batch(img_d, lbl_d, ops, luts)
    torch.cuda.synchronize()
    return x.cpu().numpy(), None if y is None else y.cpu().numpy()


def _check(imgs, lbls, ops_list):
    x, y = _run(imgs, lbls, ops_list)
    for i, im in enumerate(imgs):
        op, ks, luts = ops_list[i] if ops_list is not None else (0, 0, aug.identity_luts())
        ex, ey = oa.augment_sample(im, None if lbls is None else lbls[i], op, ks, luts)
        assert np.array_equal(x[i], ex), (i, op, ks, np.argwhere(x[i] != ex)[:5])
        if lbls is not None:
            assert np.array_equal(y[i], ey), (i, op)


def _rand_luts(rng):
    luts = aug.identity_luts()
    luts[0] = aug.bc_lut(1 + rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1))
    luts[1], luts[2], luts[3] = aug.hsv_luts(rng.uniform(-4, 4), rng.uniform(-20, 20), rng.uniform(-2, 2))
    luts[4] = aug.gamma_lut(rng.uniform(90, 110) / 100)
    return luts


SIZES = [(64, 64), (37, 53), (130, 200), (5, 7), (3, 3), (16, 129), (2, 70)]


@pytest.mark.parametrize("H,W", SIZES)
def test_each_operation_alone(H, W):
    rng = random.Random(H * 1000 + W)
    nrng = np.random.default_rng(H * 7 + W)
    single = [(0, 0), (aug.GRAY, 0), (aug.BC, 0), (aug.HSV, 0), (aug.GAMMA, 0), (0, 3), (0, 5), (aug.FLIP, 0),
              (aug.FLIP, 5)]
    if min(H, W) < 3:
        single = [s for s in single if s[1] == 0]  # cv2's reflect-101 needs 2 pixels per side for 5x5
    imgs = [nrng.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in single]
    lbls = [(nrng.integers(0, 256, (H, W), dtype=np.uint8)) for _ in single]
    ops = [(o, k, _rand_luts(rng)) for o, k in single]
    _check(imgs, lbls, ops)


@pytest.mark.parametrize("H,W", [(64, 64), (100, 77), (256, 256)])
def test_drawn_combinations(H, W):
    nrng = np.random.default_rng(H + W)
    B = 24
    ops = [aug.draw(aug.sample_rng(7, 1, i), transform=True, flip=True) for i in range(B)]
    ops[0] = (aug.GRAY | aug.BC | aug.HSV | aug.FLIP, 5, _rand_luts(random.Random(1)))  # everything at once
    ops[1] = (aug.GRAY | aug.BC | aug.HSV | aug.GAMMA, 0, _rand_luts(random.Random(2)))
    imgs = [nrng.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in range(B)]
    # smooth images too (the HSV round trip on neighbouring values)
    yy, xx = np.mgrid[0:H, 0:W]
    imgs[2] = np.stack([(xx * 255 // max(W - 1, 1)), (yy * 255 // max(H - 1, 1)), (xx + yy) % 256], -1).astype(np.uint8)
    lbls = [nrng.integers(0, 256, (H, W), dtype=np.uint8) for _ in range(B)]
    _check(imgs, lbls, ops)


def test_normalisation_only_and_no_labels():
    nrng = np.random.default_rng(3)
    imgs = [nrng.integers(0, 256, (40, 72, 3), dtype=np.uint8) for _ in range(3)]
    lbls = [nrng.integers(0, 256, (40, 72), dtype=np.uint8) for _ in range(3)]
    x, y = _run(imgs, lbls, None)
    for i in range(3):
        # reference: image.astype(float32) / 255.0, HWC -> CHW; (label > 127) as float32
        assert np.array_equal(x[i], (imgs[i].astype(np.float32) / 255.0).transpose(2, 0, 1))
        assert np.array_equal(y[i], (lbls[i] > 127).astype(np.float32))
    x2, y2 = _run(imgs, None, None)
    assert y2 is None and np.array_equal(x2, x)


def test_full_size_batch_matches_oracle_on_sampled_rows():
    """8 x 1024^2 (the bench batch): the whole batch through the kernel, the oracle on two
    samples (whole images) -- the per-sample draws are the loader's."""
    nrng = np.random.default_rng(9)
    B, H, W = 8, 1024, 1024
    ops = [aug.draw(aug.sample_rng(120, 0, i), transform=True, flip=True) for i in range(B)]
    ops[3] = (aug.BC | aug.HSV | aug.FLIP, 5, _rand_luts(random.Random(3)))
    imgs = [nrng.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in range(B)]
    lbls = [(nrng.random((H, W)) > 0.97).astype(np.uint8) * 255 for _ in range(B)]
    x, y = _run(imgs, lbls, ops)
    for i in (0, 3):
        ex, ey = oa.augment_sample(imgs[i], lbls[i], *ops[i])
        assert np.array_equal(x[i], ex) and np.array_equal(y[i], ey)


def test_random_generator_call_and_data_preparation():
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset.dataset import DataPrepartion, RandomGenerator
    nrng = np.random.default_rng(4)
    im = nrng.integers(0, 256, (48, 48, 3), dtype=np.uint8)
    lb = (nrng.random((48, 48)) > 0.5).astype(np.uint8) * 255
    sample = {'image': Image.fromarray(im), 'label': Image.fromarray(lb)}
    out = RandomGenerator(output_size=[48, 48], random_flip_flag=False, transform=False)(sample)
    assert out['image'].shape == (3, 48, 48) and out['image'].dtype == torch.float32
    assert np.array_equal(out['image'].cpu().numpy(), (im.astype(np.float32) / 255.0).transpose(2, 0, 1))
    assert np.array_equal(out['label'].cpu().numpy(), (lb > 127).astype(np.float32))
    random.seed(0)
    out = RandomGenerator(output_size=[48, 48], random_flip_flag=True, transform=True)(sample)
    random.seed(0)
    op, ks, luts = aug.draw(random, True, True)
    ex, ey = oa.augment_sample(im, lb, op, ks, luts)
    assert np.array_equal(out['image'].cpu().numpy(), ex) and np.array_equal(out['label'].cpu().numpy(), ey)
    with pytest.raises(ValueError, match="Wrong image size"):
        RandomGenerator(output_size=[32, 48])(sample)
    d = DataPrepartion(output_size=[48, 48])({'image': Image.fromarray(im)})
    assert np.array_equal(d['image'].cpu().numpy(), (im.astype(np.float32) / 255.0).transpose(2, 0, 1))


def test_loader_end_to_end(tmp_path):
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset import (GpuBatchLoader, RandomGenerator,
                                                                          SegArtifact_dataset, epoch_plan)
    root = str(tmp_path)
    nrng = np.random.default_rng(5)
    H, W = 96, 80
    files = {}
    for kind, names in (("fake", [f"f{i}" for i in range(10)]), ("real", [f"r{i}" for i in range(8)])):
        os.makedirs(os.path.join(root, kind + "_images"))
        os.makedirs(os.path.join(root, kind + "_labels"))
        with open(os.path.join(root, kind + ".txt"), "w") as f:
            f.write("\n".join(names) + "\n")
        for n in names:
            im = nrng.integers(0, 256, (H, W, 3), dtype=np.uint8)
            lb = ((nrng.random((H, W)) > 0.9) if kind == "fake" else np.zeros((H, W), bool)).astype(np.uint8) * 255
            Image.fromarray(im).save(os.path.join(root, kind + "_images", n + ".png"))
            Image.fromarray(lb).save(os.path.join(root, kind + "_labels", n + "_mask.png"))
            files[n] = (im, lb)
    tf = RandomGenerator(output_size=[H, W], random_flip_flag=True, transform=True)
    db_fake = SegArtifact_dataset(root, root, "fake", transform=tf)
    db_real = SegArtifact_dataset(root, root, "real", transform=tf)
    mixed, sampler, _, _ = epoch_plan(db_fake, db_real, epoch_num=2, seed=120)
    ld = GpuBatchLoader(mixed, sampler, device=DEV, num_threads=4, slots=2, seed=120, epoch=2, batches_per_step=2)
    from semantic_segmentation_of_stylegan2_artifacts_amd.dataset.loader import resolve
    # the expected index lists from a second plan of the same epoch (a sampler pass reshuffles
    # its pattern in place, so a pass over ld's own sampler here would change ld's batches)
    _, sampler2, _, _ = epoch_plan(db_fake, db_real, epoch_num=2, seed=120)
    steps = list(GpuBatchLoader(mixed, sampler2, device=DEV, batches_per_step=2).steps())
    seen = 0
    for k, batch in enumerate(ld):
        idx = steps[k]
        assert batch['image'].shape == (4, 3, H, W) and batch['label'].shape == (4, H, W)
        torch.cuda.synchronize()
        x, y = batch['image'].cpu().numpy(), batch['label'].cpu().numpy()
        for j, i in enumerate(idx):
            ds, r = resolve(mixed, i)
            name = ds.sample_list[r]
            assert batch['case_name'][j] == name
            op, ks, luts = tf.draw(aug.sample_rng(120, 2, i))
            ex, ey = oa.augment_sample(files[name][0], files[name][1], op, ks, luts)
            assert np.array_equal(x[j], ex) and np.array_equal(y[j], ey), (k, j, name)
        seen += 1
    assert seen == len(ld) == len(steps) >= 3  # more steps than slots: slots were reused
