"""CPU (gloo, world_size 2): the bucketed, backward-overlapped gradient all-reduce of
trainer.GradBucketer over flat gradient buffers gives exactly the gradient of the global
batch (sum over ranks), for any bucket size, and leaves every rank with identical
gradients -- the data-parallel semantics of the reference's nn.DataParallel
(trainer.py:96-97: loss = mean over the global batch, grads reduced)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import FlatGroup, GradBucketer, is_no_decay, cosine_lr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Shared(nn.Module):
    """A layer used twice per step, like MS-UNet's shared concat_back_dim[2/3]."""

    def __init__(self):
        super().__init__()
        self.inp = nn.Linear(16, 32)
        self.shared = nn.Linear(32, 32)
        self.norm = nn.LayerNorm(32)
        self.out = nn.Linear(32, 8)

    def forward(self, x):
        h = self.shared(torch.relu(self.inp(x)))
        h = self.shared(torch.relu(self.norm(h)))
        return self.out(h)


def _model():
    torch.manual_seed(0)
    return _Shared()


def _data(rank, n=6):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(n, 16, generator=g), torch.randn(n, 8, generator=g)


def _worker(rank, world, port, bucket_bytes, out, wire=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _model()
    named = list(m.named_parameters())
    decay = [(n, p) for n, p in named if not is_no_decay(n, p)][::-1]
    nodecay = [(n, p) for n, p in named if is_no_decay(n, p)][::-1]
    groups = [FlatGroup(decay, 0.01, "cpu"), FlatGroup(nodecay, 0.0, "cpu")]
    red = GradBucketer(groups, bucket_bytes, wire_dtype=wire)
    for step in range(3):  # step 0 learns the accumulation counts, later steps overlap
        x, y = _data(rank + 10 * step)
        loss = ((m(x) - y) ** 2).mean() / world  # each rank's share of the global mean
        loss.backward()
        red.finish()
        grads = torch.cat([p.grad.reshape(-1).clone() for g in groups for p in g.params])
        for g in groups:  # alignment gaps of the flat buffers stay zero
            used = torch.zeros(g.numel, dtype=torch.bool)
            for p, off in zip(g.params, g.offsets):
                used[off:off + p.numel()] = True
            assert not g.grad[~used].any()
        out[(rank, step)] = grads
        for g in groups:
            g.grad.zero_()
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes,wire", [(64, None), (1 << 20, None), (256, torch.bfloat16),
                                               (1 << 20, torch.float16)])
def test_bucketed_allreduce_equals_global_batch(bucket_bytes, wire):
    """wire: the 16-bit gradient all-reduce (BASELINE config 5 'fp16 grads'): the sum is
    taken over 16-bit casts of each rank's gradient, so it matches the global-batch gradient
    to 16-bit rounding; every rank still ends with bitwise-identical gradients."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), bucket_bytes, out, wire), nprocs=world, join=True)
    for step in range(3):
        m = _model()
        named = list(m.named_parameters())
        xs, ys = zip(*[_data(r + 10 * step) for r in range(world)])
        loss = ((m(torch.cat(xs)) - torch.cat(ys)) ** 2).mean()
        loss.backward()
        decay = [p for n, p in named if not is_no_decay(n, p)][::-1]
        nodecay = [p for n, p in named if is_no_decay(n, p)][::-1]
        ref = torch.cat([p.grad.reshape(-1) for p in decay + nodecay])
        g0, g1 = out[(0, step)], out[(1, step)]
        assert torch.equal(g0, g1), "ranks disagree"
        if wire is None:
            torch.testing.assert_close(g0, ref, rtol=1e-5, atol=1e-6)
        else:
            eps = 2.0 ** -8 if wire == torch.bfloat16 else 2.0 ** -11
            torch.testing.assert_close(g0, ref, rtol=3 * eps, atol=3 * eps * ref.abs().max().item())
            assert not torch.equal(g0, ref)  # the wire really is 16-bit


def _small_worker(rank, world, port, out, loss_scale, init_scale):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _model()
    named = list(m.named_parameters())
    groups = [FlatGroup(named[::-1], 0.0, "cpu")]
    red = GradBucketer(groups, 1 << 20, wire_dtype=torch.float16)
    if init_scale is not None:
        red.scale.fill_(init_scale)
        red.inv_scale.fill_(1.0 / init_scale)
    x, y = _data(0)  # the same batch on both ranks: the sum has no cancellation
    (((m(x) - y) ** 2).mean() * loss_scale / world).backward()
    red.finish()
    found = torch.zeros(1)
    found.fill_(float(not torch.isfinite(groups[0].grad).all()))
    red.update_scale(found)
    out[rank] = (groups[0].grad.clone(), float(found), float(red.scale))
    dist.destroy_process_group()


@pytest.mark.parametrize("loss_scale", [1e-4, 1e-6])
def test_fp16_wire_keeps_tiny_gradients(loss_scale):
    """the f16 wire scales the buckets (GradScaler-style, 2^16 to start) before the
    cast, so gradients of 1e-6 .. 1e-10 survive f16's 6e-8 underflow; unscaled they would
    flush to zero or lose most of their bits."""
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_small_worker, args=(world, _free_port(), out, loss_scale, None), nprocs=world, join=True)
    m = _model()
    named = list(m.named_parameters())
    x, y = _data(0)
    (((m(x) - y) ** 2).mean() * loss_scale).backward()
    ref = torch.cat([p.grad.reshape(-1) for _, p in named[::-1]])
    got = torch.cat([out[0][0][o:o + p.numel()] for p, o in
                     zip([p for _, p in named[::-1]], FlatGroup(named[::-1], 0.0, "cpu").offsets)])
    assert torch.equal(out[0][0], out[1][0])
    assert out[0][1] == 0.0 and out[0][2] == 2.0 ** 16  # no overflow, scale kept
    if loss_scale < 1e-5:  # the case needs the scale: many gradients below f16's underflow
        assert (ref.abs() < 6e-8).float().mean().item() > 0.05
    # f16 rounding of each rank's scaled share and of the sum; 1e-11 absolute floor
    # (unscaled, anything below 6e-8 would be lost)
    excess = ((got - ref).abs() - 4 * 2.0 ** -11 * ref.abs()).max().item()
    assert excess <= 1e-11, excess


def test_fp16_wire_overflow_is_flagged_and_backs_off():
    """A scale that overflows f16 in the sum: the gradients come back non-finite on every rank
    (the trainer's non-finite check then skips the step everywhere) and the scale halves."""
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_small_worker, args=(world, _free_port(), out, 1.0, 2.0 ** 40), nprocs=world, join=True)
    for r in range(world):
        assert out[r][1] == 1.0
        assert out[r][2] == 2.0 ** 39


def test_no_decay_rule_matches_reference():
    """trainer.py:137: 1-D params, '.bias' names and names containing 'norm' -> no decay."""
    p2 = torch.zeros(3, 3)
    p1 = torch.zeros(3)
    assert not is_no_decay("layers.0.blocks.0.attn.qkv.weight", p2)
    assert is_no_decay("layers.0.blocks.0.attn.qkv.bias", p1)
    assert is_no_decay("layers.0.blocks.0.norm1.weight", p1)
    assert is_no_decay("layers.0.blocks.0.attn.relative_position_bias_table", torch.zeros(169, 3)) is False
    assert is_no_decay("up.norm.weight", p1)


def test_cosine_schedule_matches_timm_semantics():
    """timm CosineLRScheduler(t_initial=60-20, warmup_t=20, warmup_prefix=True) per epoch."""
    base, wlr, mn = 1e-5, 1e-6, 1e-6
    assert cosine_lr(0, base, 20, 60, wlr, mn) == pytest.approx(wlr)
    assert cosine_lr(10, base, 20, 60, wlr, mn) == pytest.approx(wlr + 10 * (base - wlr) / 20)
    assert cosine_lr(20, base, 20, 60, wlr, mn) == pytest.approx(base)
    assert cosine_lr(40, base, 20, 60, wlr, mn) == pytest.approx(mn + 0.5 * (base - mn))
    assert cosine_lr(70, base, 20, 60, wlr, mn) == pytest.approx(mn)


def test_reseed_gives_each_rank_its_own_masks():
    """ranks must not share drop-path / attention-dropout randomness.  The model is
    built from the shared seed (same weights); reseed(seed, rank) then splits the streams."""
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import reseed
    from semantic_segmentation_of_stylegan2_artifacts_amd.network import model_parts
    draws = []
    for rank in (0, 1, 0):
        reseed(120, rank)
        scale = model_parts._drop_path_scale(0.5, True, 64, "cpu")
        draws.append((model_parts._next_seed(), torch.rand(4), scale.clone()))
    assert draws[0][0] == draws[2][0] and torch.equal(draws[0][1], draws[2][1])  # reproducible
    assert draws[0][0] != draws[1][0]
    assert not torch.equal(draws[0][1], draws[1][1])
    model_parts._SCALE_POOL.clear()
