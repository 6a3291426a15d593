"""Generate ``tests/golden/batch_sampler.json`` by running the REFERENCE sampler.

Run in the survey/dev container only (needs ``/root/reference``; never on the GPU box):

    python tests/golden/gen_input_golden.py

Imports the reference's ``scripts/batch_data_loader_V2.py`` (its imports -- ``random``,
``torch.utils.data.Sampler``, ``typing``, ``numpy`` -- are all present) and records, for
several (fake, real, epoch) cases, the batches of two consecutive passes over one sampler
instance (the pattern list is shuffled in place, so the second pass differs) plus a
``set_epoch`` pass, and the ``ValueError`` messages of the constructor's checks.  Also
records ``torch.randperm`` real subsets of ``trainer.py:225-226`` for a few (seed, epoch)
pairs (the epoch plan's only library RNG).
"""
import importlib.util
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    spec = importlib.util.spec_from_file_location("ref_bdl", os.path.join(REF, "scripts", "batch_data_loader_V2.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cases = []
    for n_fake, n_real, epoch in [(3, 1, 1), (6, 4, 1), (6, 4, 2), (10, 2, 7), (9, 5, 13), (40, 24, 3),
                                  (800, 532, 1), (800, 532, 36)]:
        fake = list(range(n_fake))
        real = list(range(n_fake, n_fake + n_real))
        nb = (n_fake + n_real) // 2
        s = mod.BatchPatternSampler(fake, real, nb, 2, epoch)
        first = [list(b) for b in s]
        second = [list(b) for b in s]
        s.set_epoch(epoch + 5)
        third = [list(b) for b in s]
        cases.append(dict(n_fake=n_fake, n_real=n_real, epoch=epoch, len=len(s), passes=[first, second, third]))
    errors = []
    for args in [([0, 1], [2, 3], 2, 4, 1), ([], [0, 1], 1, 2, 1), ([0, 1], [], 1, 2, 1), ([0, 1, 2], [3], 3, 2, 1),
                 ([0], [1, 2, 3], 2, 2, 1)]:
        try:
            mod.BatchPatternSampler(*args)
            errors.append(dict(args=args, error=None))
        except ValueError as e:
            errors.append(dict(args=args, error=str(e)))
    perms = []
    for seed, epoch, total in [(120, 0, 532), (120, 11, 532), (1234, 3, 40)]:
        g = torch.Generator().manual_seed(seed + epoch)
        perms.append(dict(seed=seed, epoch=epoch, total=total, perm=torch.randperm(total, generator=g).tolist()))
    out = dict(source="reference scripts/batch_data_loader_V2.py (imported), trainer.py:225-226 randperm",
               cases=cases, errors=errors, randperm=perms)
    with open(os.path.join(HERE, "batch_sampler.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote batch_sampler.json", len(cases), "cases")


if __name__ == "__main__":
    main()
