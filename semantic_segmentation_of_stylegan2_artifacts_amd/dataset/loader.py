"""The training input pipeline on the GPU: per-epoch real/fake plan, batch sampling, PNG
decode into pinned memory, uint8 upload and one augmentation pass per batch.

Reference (what this replaces):

* ``trainer.py:195-237``: each epoch a real ratio (``DYNAMIC_LOADER`` schedule), a real-image
  subset drawn by ``torch.randperm`` seeded with ``SEED + epoch``, ``ConcatDataset([fake,
  Subset(real, idx)])`` and a ``BatchPatternSampler`` over it (``epoch_plan`` below);
* ``trainer.py:239-245``: a ``DataLoader`` whose workers decode PNGs and run the
  albumentations pipeline per sample on the CPU, then collate f32 batches that cross PCIe as
  16 B / pixel (``GpuBatchLoader``).

``GpuBatchLoader`` instead: a producer thread decodes each step's samples with PIL on a thread
pool (PIL releases the GIL while decoding) straight into a pinned uint8 slot (4 B / pixel),
draws every sample's augmentation on the host (``dataset.augment``, keyed by (seed, epoch,
index)), copies the slot to the device on its own stream and launches ``msu_augment_batch``
there; the consumer's stream waits on an event, so decode, upload and augmentation of the
next step overlap the current training step.  ``slots`` pinned slots rotate; a slot is reused
only after its upload has completed.

Data parallel: each step consumes ``batches_per_step * world_size`` consecutive sampler
batches; rank r takes the ``batches_per_step`` batches of slice r (the reference's sampler
yields batches of 2, so bs 8 per GPU = 4 sampler batches, each with its guaranteed fake).
"""
import queue
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
from torch.utils.data import ConcatDataset, Subset

from ..scripts.batch_data_loader_V2 import BatchPatternSampler
from . import augment
from .dataset import DataPrepartion, RandomGenerator, augment_batch


# ------------------------------------------------------------------ epoch plan (trainer.py:195-237)
def real_ratio_for_epoch(epoch_num, dynamic_loader):
    """``trainer.py:196-208``."""
    if not dynamic_loader:
        return 0.4
    if epoch_num < 9:
        return 0.1
    if epoch_num < 20:
        return 0.10 + 0.03 * (epoch_num - 8)
    if epoch_num < 30:
        return 0.4
    if epoch_num < 35:
        return 0.2
    return 0.4


def num_real_for(total_fake, total_real, real_ratio):
    """``trainer.py:210-215``: real images so that reals are ``real_ratio`` of the epoch, made
    even in total; more than available raises ValueError (the reference's message)."""
    num_real = int((total_fake / (1 - real_ratio)) * real_ratio)
    if ((num_real + total_fake) % 2) != 0:
        num_real = max(0, num_real - 1)
    if num_real > total_real:
        raise ValueError("More real images are reqzired than available: num_reall {num_real} num_total {total_real}")
    return num_real


def epoch_plan(db_fake, db_real, epoch_num, seed, dynamic_loader=False, batch_size=2):
    """The mixed dataset and batch sampler of one epoch (``trainer.py:195-237``): returns
    ``(db_mixed, batch_sampler, real_ratio, indices_real)``."""
    real_ratio = real_ratio_for_epoch(epoch_num, dynamic_loader)
    total_fake, total_real = len(db_fake), len(db_real)
    num_real = num_real_for(total_fake, total_real, real_ratio)
    g = torch.Generator().manual_seed(int(seed) + int(epoch_num))
    indices_real = torch.randperm(total_real, generator=g)[:num_real]
    db_mixed = ConcatDataset([db_fake, Subset(db_real, indices_real)])
    n_fake, n_real = len(db_fake), num_real
    sampler = BatchPatternSampler(fake_indices=list(range(n_fake)),
                                  real_indices=list(range(n_fake, n_fake + n_real)),
                                  num_batch=(n_fake + n_real) // 2, batch_size=batch_size,
                                  epoch=epoch_num + 1)
    return db_mixed, sampler, real_ratio, indices_real


# ------------------------------------------------------------------ index resolution
def resolve(ds, idx):
    """(base dataset with ``read_raw``, its index) behind Subset / ConcatDataset wrappers."""
    while True:
        if isinstance(ds, Subset):
            idx = int(ds.indices[idx])
            ds = ds.dataset
        elif isinstance(ds, ConcatDataset):
            if idx < 0:
                idx += len(ds)
            k = int(np.searchsorted(ds.cumulative_sizes, idx, side="right"))
            idx = idx - (ds.cumulative_sizes[k - 1] if k > 0 else 0)
            ds = ds.datasets[k]
        else:
            return ds, idx


def _base_transform(ds):
    while isinstance(ds, (Subset, ConcatDataset)):
        ds = ds.dataset if isinstance(ds, Subset) else ds.datasets[0]
    t = getattr(ds, "transform", None)
    for t_ in getattr(t, "transforms", [t]):  # torchvision-style Compose([RandomGenerator(...)])
        if isinstance(t_, (RandomGenerator, DataPrepartion)):
            return t_
    return None


class _Slot:
    def __init__(self, B, H, W, labels):
        self.img = torch.empty(B, H, W, 3, dtype=torch.uint8).pin_memory()
        self.lbl = torch.empty(B, H, W, dtype=torch.uint8).pin_memory() if labels else None
        self.ops = torch.empty(B, 2, dtype=torch.int32).pin_memory()
        self.luts = torch.empty(B, augment.N_LUT, 256, dtype=torch.uint8).pin_memory()
        self.uploaded = None  # event: the slot's H2D copies are done


class GpuBatchLoader:
    """Iterates device batches ``{'image': f32 [B, 3, H, W], 'label': f32 [B, H, W],
    'case_name': [...]}`` for a dataset of ``SegArtifact_dataset``s (possibly wrapped in
    Subset / ConcatDataset) and a batch sampler.

    ``transform``: a ``RandomGenerator`` / ``DataPrepartion`` (default: the dataset's own, else
    normalisation only); ``seed`` / ``epoch`` key the per-sample draws."""

    def __init__(self, dataset, batch_sampler, *, transform=None, device=None, num_threads=8, slots=3,
                 seed=1234, epoch=0, rank=0, world_size=1, batches_per_step=1, drop_last=True):
        self.dataset = dataset
        self.batch_sampler = batch_sampler
        self.transform = transform if transform is not None else _base_transform(dataset)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.num_threads = num_threads
        self.n_slots = max(2, int(slots))
        self.seed, self.epoch = seed, epoch
        self.rank, self.world_size = rank, world_size
        self.batches_per_step = batches_per_step
        self.drop_last = drop_last
        self._slots = None
        self._stream = None

    def set_epoch(self, epoch):
        self.epoch = int(epoch)
        if hasattr(self.batch_sampler, "set_epoch"):
            self.batch_sampler.set_epoch(epoch)

    # -------------------------------------------------------------- step index lists
    def steps(self):
        """Per-step index lists of this rank."""
        group = self.batches_per_step * self.world_size
        buf = []
        for batch in self.batch_sampler:
            buf.append(list(batch))
            if len(buf) == group:
                mine = buf[self.rank * self.batches_per_step:(self.rank + 1) * self.batches_per_step]
                yield [i for b in mine for i in b]
                buf = []
        if buf and not self.drop_last and len(buf) > self.rank * self.batches_per_step:
            mine = buf[self.rank * self.batches_per_step:(self.rank + 1) * self.batches_per_step]
            yield [i for b in mine for i in b]

    def __len__(self):
        n = len(self.batch_sampler) // (self.batches_per_step * self.world_size)
        return n

    # -------------------------------------------------------------- producer
    def _draw(self, idx):
        if isinstance(self.transform, RandomGenerator):
            return self.transform.draw(augment.sample_rng(self.seed, self.epoch, idx))
        return 0, 0, augment.identity_luts()

    def _produce(self, q, stop):
        pool = ThreadPoolExecutor(self.num_threads)
        try:
            k = 0
            for idx in self.steps():
                if stop.is_set():
                    break
                self._load_step(pool, q, k, idx)
                k += 1
        except BaseException as e:  # surfaced to the consumer
            q.put(e)
            return
        finally:
            pool.shutdown(wait=True)
        q.put(None)

    def _load_step(self, pool, q, k, idx):
        B = len(idx)
        refs = [resolve(self.dataset, i) for i in idx]
        first = refs[0][0].read_raw(refs[0][1]) if self._slots is None else None
        if self._slots is None:
            H, W = first[0].shape[:2]
            labels = first[1] is not None
            self._slots = [_Slot(B, H, W, labels) for _ in range(self.n_slots)]
            self._stream = torch.cuda.Stream(self.device)
        slot = self._slots[k % self.n_slots]
        if slot.uploaded is not None:
            slot.uploaded.synchronize()
        if B > slot.img.shape[0]:
            raise ValueError(f"step of {B} samples exceeds the slot size {slot.img.shape[0]}")
        img_np, lbl_np = slot.img.numpy(), None if slot.lbl is None else slot.lbl.numpy()

        def load(j):
            ds, i = refs[j]
            im, lb = first if (j == 0 and first is not None) else ds.read_raw(i)
            if self.transform is not None:
                self.transform.check(im)
            if im.shape != img_np.shape[1:]:
                raise ValueError(f"sample {idx[j]}: image {im.shape} differs from the batch's {img_np.shape[1:]}")
            img_np[j] = im
            if lbl_np is not None:
                lbl_np[j] = lb
            op, ks, luts = self._draw(idx[j])
            slot.ops[j, 0], slot.ops[j, 1] = op, ks
            slot.luts[j] = torch.from_numpy(luts)

        list(pool.map(load, range(B)))
        with torch.cuda.device(self.device), torch.cuda.stream(self._stream):
            img_d = slot.img[:B].to(self.device, non_blocking=True)
            lbl_d = None if slot.lbl is None else slot.lbl[:B].to(self.device, non_blocking=True)
            ops_d = slot.ops[:B].to(self.device, non_blocking=True)
            luts_d = slot.luts[:B].to(self.device, non_blocking=True)
            slot.uploaded = torch.cuda.Event()
            slot.uploaded.record(self._stream)
            x, y = augment_batch(img_d, lbl_d, ops_d, luts_d)
            done = torch.cuda.Event()
            done.record(self._stream)
        names = [ds.sample_list[i].strip('\n') for ds, i in refs]
        q.put((x, y, names, done))

    # -------------------------------------------------------------- consumer
    def __iter__(self):
        q = queue.Queue(maxsize=self.n_slots - 1)
        stop = threading.Event()
        th = threading.Thread(target=self._produce, args=(q, stop), daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                x, y, names, done = item
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(done)
                x.record_stream(cur)
                out = {'image': x, 'case_name': names}
                if y is not None:
                    y.record_stream(cur)
                    out['label'] = y
                yield out
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get(timeout=0.05)
                except queue.Empty:
                    pass
            th.join()
