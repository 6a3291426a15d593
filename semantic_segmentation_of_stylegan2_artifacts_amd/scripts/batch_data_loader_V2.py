"""``BatchPatternSampler``: every batch of two holds at least one fake image.

Drop-in for the reference's ``scripts/batch_data_loader_V2.py:9-95`` (same constructor, the
same ``ValueError`` rules, the same batches for the same epoch).  Each epoch:

* the fake and real index lists are shuffled by ``random.Random(epoch)`` (fake first, then
  real), and so is the batch *pattern* -- ``rest_fake`` entries "2" (fake + fake) and
  ``len(real)`` entries "1" (fake + real).  The pattern is an attribute shuffled in place, so
  a second pass over the same sampler starts from the previous pass's order, exactly as in
  the reference;
* batch ``b`` puts its guaranteed fake first when ``random.Random(epoch + b).random() < 0.5``.

Host-side index logic only; the GPU half of the input pipeline is ``dataset.loader``.
"""
import random
from typing import Iterator, List

from torch.utils.data import Sampler


class BatchPatternSampler(Sampler):
    def __init__(self, fake_indices, real_indices, num_batch, batch_size, epoch):
        self.fake_indices = list(fake_indices)
        self.real_indices = list(real_indices)
        n_fake, n_real = len(self.fake_indices), len(self.real_indices)
        if batch_size != 2:
            raise ValueError("batch_size must be 2 ")
        if n_fake == 0:
            raise ValueError("Need at least 1 fake index to guarantee 'at least one fake per batch'.")
        if n_real == 0:
            raise ValueError("Need at least 1 real index to guarantee 'at least one fake per batch'.")
        if n_fake + n_real != 2 * num_batch:
            raise ValueError("num fake + num real != batch_size * 2")
        if n_fake < num_batch:
            raise ValueError("num fake needs to be higher than the number of batches")
        self.epoch = epoch
        self.num_batch = num_batch
        self.rest_fake = n_fake - num_batch
        # 2: a second fake fills the batch; 1: a real one does
        self.pattern = [2] * self.rest_fake + [1] * n_real
        self.i_fake = 0
        self.i_real = 0

    def __len__(self) -> int:
        return self.num_batch

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __iter__(self) -> Iterator[List[int]]:
        shuffler = random.Random(self.epoch)
        fake, real = list(self.fake_indices), list(self.real_indices)
        for seq in (fake, real, self.pattern):
            shuffler.shuffle(seq)
        self.i_fake = self.i_real = 0
        for b in range(self.num_batch):
            fake_first = random.Random(self.epoch + b).random() < 0.5
            guaranteed = self._take_fake(fake) if fake_first else None
            second = self._take_real(real) if self.pattern[b] == 1 else self._take_fake(fake)
            if fake_first:
                yield [guaranteed, second]
            else:
                yield [second, self._take_fake(fake)]

    def _take_fake(self, fake):
        if self.i_fake >= len(fake):
            raise ValueError(f"length of trian fake data {len(fake)} exeded with i_fake: {self.i_fake}")
        self.i_fake += 1
        return fake[self.i_fake - 1]

    def _take_real(self, real):
        if self.i_real >= len(real):
            raise ValueError(f"length of train real data {len(real)} exeded with i_real: {self.i_real}")
        self.i_real += 1
        return real[self.i_real - 1]
