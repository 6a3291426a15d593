"""Training step of ``trainer.py:295-336`` re-planned for MI355X data parallelism.

Reference step (per batch): autocast fp16 -> model -> DynamicLoss -> GradScaler backward ->
AdamW (two param groups, ``trainer.py:130-152``) -> ``loss.item()``; multi-GPU via
``nn.DataParallel`` (``trainer.py:96-97``; unusable for N_GPU > 1 because the batch
sampler requires batch_size == 2).

Here:
* one process per GPU (torchrun env), bf16 autocast (no loss scaling needed), no host
  synchronisation inside the step (the loss stays on the device);
* trainable parameters and their gradients live in two flat f32 buffers (weight-decay /
  no-decay, the reference's split rule) laid out in reverse registration order, so
  gradients become ready roughly front-to-back during backward;
* DP: the gradient buffers are cut into ~``bucket_mb`` buckets; when every parameter of a
  bucket has accumulated its gradient (post-accumulate hooks) the bucket is all-reduced
  (RCCL over xGMI, ``async_op``) while backward continues; the 1/world average is folded
  into the fused AdamW kernel; ``grad_wire_dtype`` (bf16 / f16) all-reduces 16-bit casts of
  the buckets instead (half the bytes; BASELINE config 5's "fp16 grads");
* AdamW = one fused HIP launch per group over the flat buffer, lr / step read from device
  memory, skipped (GradScaler semantics) when a gradient is non-finite;
* after four eager steps the device side of the step is captured into a HIP graph and
  replayed (``Trainer.step``) when the eager step is launch-bound: the host then issues one
  launch per step;
* parameters whose outputs the reference discards (dead central-decoder branches) never
  receive gradients there; they are excluded here, matching torch AdamW's skip of
  ``grad is None``.
"""
import math
import os
import threading
import time

import torch
import torch.distributed as dist

from . import ops, switches
from .loss import DynamicLoss
from .network import model_parts



def is_no_decay(name, param):
    """``trainer.py:137``: 1-D params, biases and anything with 'norm' in its name."""
    return param.ndim == 1 or name.endswith(".bias") or "norm" in name.lower()


def cosine_lr(epoch, base_lr, warmup_epochs, max_epochs, warmup_lr, min_lr, warmup_prefix=True):
    """timm CosineLRScheduler(t_initial=lr_epochs - warmup, warmup_prefix, cycle_limit=1),
    stepped per epoch as in ``trainer.py:155-169, :412`` (lr_epochs = max(60, max_epochs))."""
    lr_epochs = max(60, max_epochs)
    t_initial = lr_epochs - warmup_epochs
    if epoch < warmup_epochs:
        return warmup_lr + epoch * (base_lr - warmup_lr) / warmup_epochs
    t = epoch - warmup_epochs if warmup_prefix else epoch
    if t >= t_initial:
        return min_lr
    return min_lr + 0.5 * (base_lr - min_lr) * (1 + math.cos(math.pi * t / t_initial))


class FlatGroup:
    """Parameters (and grads) of one optimizer group re-homed into flat f32 buffers."""

    def __init__(self, named_params, weight_decay, device):
        self.names = [n for n, _ in named_params]
        self.params = [p for _, p in named_params]
        self.weight_decay = weight_decay
        # every parameter starts on a 64-B boundary (16-B vector kernels write gradients in
        # place); the gaps stay zero in data, grad and both moments
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + 15) // 16 * 16
        n = off
        self.numel = n
        self.count = sum(p.numel() for p in self.params)
        self.data = torch.zeros(n, device=device, dtype=torch.float32)
        self.grad = torch.zeros(n, device=device, dtype=torch.float32)
        self.exp_avg = torch.zeros_like(self.data)
        self.exp_avg_sq = torch.zeros_like(self.data)
        # bf16 shadow of the parameters, refreshed once per step: the Linear ops read it
        # instead of casting every weight at every call
        self.shadow = torch.empty(n, device=device, dtype=torch.bfloat16)
        for p, off in zip(self.params, self.offsets):
            k = p.numel()
            self.data[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.data[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            p._msu_shadow = self.shadow[off:off + k].view_as(p)
            p._msu_shadow_ver = -1  # not valid until the first refresh
            p._msu_direct = True  # backward kernels accumulate straight into p.grad
        # transposed bf16 shadow of the 2-D weights (Linear weights: both dims multiples of 8),
        # written by one batched transpose after each refresh: the input-gradient GEMMs read
        # W^T in the forward GEMM's layout instead of transposing per call (ops._shadow_t)
        tab, owners, toff, tiles = [], [], 0, 0
        for p, off in zip(self.params, self.offsets):
            if p.ndim == 2 and p.shape[0] % 8 == 0 and p.shape[1] % 8 == 0:
                N, K = p.shape
                tab.append((off, toff, N, K, tiles))
                owners.append(p)
                tiles += -(-N // 64) * -(-K // 64)
                toff += (N * K + 7) // 8 * 8
        self.tshadow = self.ttable = None
        self.ntiles = tiles
        if tab and torch.device(device).type == "cuda":
            self.tshadow = torch.empty(toff, device=device, dtype=torch.bfloat16)
            self.ttable = torch.tensor(tab, dtype=torch.int64).to(device)
            for (_, to, N, K, _), p in zip(tab, owners):
                p._msu_shadow_t = self.tshadow[to:to + N * K].view(K, N)

    def refresh_shadow(self):
        """Re-cast the bf16 shadow after the master weights changed (AdamW writes them through
        a raw pointer).  Each parameter records its version: an in-place write made through
        the parameter itself (load_state_dict, ``p.copy_``) bumps it and makes the Linear ops
        cast that weight again until the next refresh."""
        self.copy_shadow()
        self.mark_shadow()

    def copy_shadow(self):
        self.shadow.copy_(self.data)
        self.transpose_shadow()

    def transpose_shadow(self):
        """The transposed shadow of the 2-D weights from the (refreshed) shadow."""
        if self.tshadow is not None and ops._SHADOW_T:
            ops.transpose16_multi(self.shadow, self.tshadow, self.ttable, self.ntiles)

    def mark_shadow(self):
        """Host-only half of the refresh: the raw-pointer AdamW and the shadow copy do not
        bump parameter versions, so this can run while the GPU is still in backward."""
        for p in self.params:
            p._msu_shadow_ver = p._version


class GradBucketer:
    """Bucketed, backward-overlapped gradient all-reduce over flat gradient buffers.

    A bucket is all-reduced as soon as every accumulation into its parameters' gradients has
    happened.  Parameters used more than once per step (MS-UNet shares concat_back_dim[2/3]
    between the central and the main decoder, model_parts.py:792-824) receive several
    accumulations, so the number expected per bucket is measured on the first step (the
    graph is static), which all-reduces every bucket after backward; later steps overlap.
    """

    # GradScaler defaults (torch.amp.GradScaler): the fp16 wire's dynamic scale
    INIT_SCALE, GROWTH_FACTOR, BACKOFF_FACTOR, GROWTH_INTERVAL = 2.0 ** 16, 2.0, 0.5, 2000

    def __init__(self, groups, bucket_bytes, process_group=None, wire_dtype=None):
        self.pg = process_group
        # wire_dtype (bf16 / f16): each bucket is cast into a persistent 16-bit buffer, summed
        # over the ranks in that precision and cast back into the f32 gradients -- half the
        # xGMI bytes per step (BASELINE config 5: "fp16 grads"), at 16-bit rounding of the
        # per-rank gradients and of the ring's partial sums.  None: f32 all-reduce.
        self.wire_dtype = None if wire_dtype in (None, torch.float32) else wire_dtype
        self.wire = {}  # bucket index -> 16-bit buffer
        # f16 has 5 exponent bits: like the reference's GradScaler-scaled fp16 gradients
        # (trainer.py:182,314-316) the buckets are multiplied by a dynamic scale before the
        # cast (tiny gradients stay above f16's 6e-8 underflow) and divided by it on the way
        # back; a sum that overflows comes back inf, the trainer's non-finite check skips the
        # step on every rank and update_scale() halves the scale (x2 after 2000 clean steps).
        # bf16 keeps f32's exponent range: no scale.
        dev = groups[0].grad.device
        self.scale = self.inv_scale = self.growth_tracker = None
        if self.wire_dtype == torch.float16:
            self.scale = torch.full((1,), self.INIT_SCALE, device=dev, dtype=torch.float32)
            self.inv_scale = torch.full((1,), 1.0 / self.INIT_SCALE, device=dev, dtype=torch.float32)
            self.growth_tracker = torch.zeros(1, device=dev, dtype=torch.int32)
        # the collectives' own stream (one per device): each bucket's cast / all-reduce waits
        # there for both the main and the weight-gradient side stream, so neither stream's
        # later kernels queue behind a collective that blocks until every rank arrives
        self.comm = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self.buckets = []       # (group, start, end)
        self.param_bucket = {}  # id(param) -> bucket index
        for g in groups:
            start = 0
            count = 0
            for p, off in zip(g.params, g.offsets):
                end = off + p.numel()
                self.param_bucket[id(p)] = len(self.buckets)
                count += 1
                if (end - start) * 4 >= bucket_bytes:
                    self.buckets.append([g, start, end])
                    start, count = end, 0
            if count:
                self.buckets.append([g, start, g.numel])
        self.main_stream = None  # the stream the training step runs on (set per step)
        # set by the Trainer while it captures the step: every bucket is then issued by finish()
        # on the capturing thread.  Backward's hooks run on autograd's device thread, and a
        # collective issued there during a thread-local capture was at times handed to the
        # process group's watchdog as eager work; the watchdog's query of its event (recorded
        # in the capturing stream) then aborted the process (hipErrorCapturedEvent, r04f)
        self.capturing = False
        self.expected = None    # accumulations per bucket, learned on the first step
        self.pending = [0] * len(self.buckets)
        self.launched = [False] * len(self.buckets)
        self.works = []
        # (bucket, thread id, "hook" | "finish", capturing) of every launch of the current step;
        # ``last_launches`` keeps the previous step's (tests/test_capture_guard.py checks that a
        # capture issues every bucket from finish() on the capturing thread)
        self.launches = []
        self.last_launches = []
        self.handles = []
        for g in groups:
            for p in g.params:
                self.handles.append(p.register_post_accumulate_grad_hook(self._hook))

    def _reduce(self, b, g, s, e):
        """Issue bucket b's all-reduce on the current stream: (work, 16-bit buffer or None)."""
        if self.wire_dtype is None:
            return dist.all_reduce(g.grad[s:e], op=dist.ReduceOp.SUM, group=self.pg, async_op=True), None
        buf = self.wire.get(b)
        if buf is None:
            buf = self.wire[b] = torch.empty(e - s, device=g.grad.device, dtype=self.wire_dtype)
        if self.scale is not None:
            torch.mul(g.grad[s:e], self.scale, out=buf)
        else:
            buf.copy_(g.grad[s:e])
        return dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.pg, async_op=True), buf

    def _launch(self, b, via):
        g, s, e = self.buckets[b]
        self.launched[b] = True
        self.launches.append((b, threading.get_ident(), via, self.capturing))
        if self.comm is None:
            self.works.append((b,) + self._reduce(b, g, s, e))
            return
        # the bucket's gradients come from both streams: the comm stream catches up with the
        # work issued so far on the main stream (named explicitly: the hook may fire while
        # autograd runs a side-stream node) and on the weight-gradient side stream
        dev = g.grad.device
        main = self.main_stream if self.main_stream is not None else torch.cuda.current_stream(dev)
        if self.capturing or torch.cuda.is_current_stream_capturing():
            # under HIP-graph capture the collective is issued from the capturing main stream
            # (the graph runs it as a branch of its own anyway): a capture that also forked the
            # comm stream crashed hipStreamEndCapture on ROCm 7.2 (tests/test_gpu_rccl.py)
            side = ops.side_stream(dev)
            if side is not None:
                main.wait_stream(side)
            with torch.cuda.stream(main):
                self.works.append((b,) + self._reduce(b, g, s, e))
            return
        self.comm.wait_stream(main)
        side = ops.side_stream(dev)
        if side is not None:
            self.comm.wait_stream(side)
        with torch.cuda.stream(self.comm):
            self.works.append((b,) + self._reduce(b, g, s, e))

    def _hook(self, p):
        b = self.param_bucket[id(p)]
        self.pending[b] += 1
        if self.expected is not None and self.pending[b] == self.expected[b] and not self.capturing:
            self._launch(b, "hook")

    def _unwire(self, b, buf):
        g, s, e = self.buckets[b]
        if self.scale is not None:
            torch.mul(buf, self.inv_scale, out=g.grad[s:e])
        else:
            g.grad[s:e].copy_(buf)

    def finish(self):
        """Launch what backward did not, wait for every bucket's sum (the current stream waits
        for the comm stream: AdamW is ordered after the exchange without a host sync)."""
        if self.expected is None:
            self.expected = list(self.pending)
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b, "finish")
        if self.comm is None or self.capturing or torch.cuda.is_current_stream_capturing():
            for b, w, buf in self.works:  # (the current stream waits for each collective)
                w.wait()
                if buf is not None:
                    self._unwire(b, buf)
        else:
            with torch.cuda.stream(self.comm):
                for b, w, buf in self.works:
                    w.wait()  # the comm stream waits for the collective
                    if buf is not None:  # back into the f32 gradients, after the sum
                        self._unwire(b, buf)
            main = self.main_stream if self.main_stream is not None else torch.cuda.current_stream(self.comm.device)
            main.wait_stream(self.comm)
        self.works = []
        self.pending = [0] * len(self.buckets)
        self.launched = [False] * len(self.buckets)
        self.last_launches, self.launches = self.launches, []

    def reset(self):
        """Forget a step that did not finish (e.g. an aborted HIP-graph capture): no pending
        accumulation counts, no launched flags, no outstanding work handles."""
        self.works = []
        self.pending = [0] * len(self.buckets)
        self.launched = [False] * len(self.buckets)
        self.launches = []

    def update_scale(self, found_inf):
        """GradScaler's dynamic-scale rule for the f16 wire (no-op otherwise), on the device:
        found_inf (f32 [1], the step's non-finite flag) -> scale x0.5, else x2 after
        GROWTH_INTERVAL consecutive clean steps."""
        if self.scale is None:
            return
        torch._amp_update_scale_(self.scale, self.growth_tracker, found_inf, self.GROWTH_FACTOR,
                                 self.BACKOFF_FACTOR, self.GROWTH_INTERVAL)
        torch.reciprocal(self.scale, out=self.inv_scale)


def reseed(seed, rank=0):
    """Per-rank randomness for data parallelism: the model is built from the shared seed
    (identical initial weights on every rank), then every rank draws its own drop-path and
    dropout masks (torch CPU/HIP generators and the attention-dropout seed stream), so the
    global batch sees independent masks per sample, as the reference's single process does."""
    from .network import model_parts
    s = int(seed) + 1_000_003 * int(rank)
    torch.manual_seed(s)  # seeds the HIP generators of every device too
    model_parts.reseed(s)


def rccl_capture_blocker(process_group):
    """Why a HIP-graph capture of the step over ``process_group`` would be unsafe, or None.

    ProcessGroupNCCL's event cache (TORCH_NCCL_CUDA_EVENT_CACHE, on by default) hands a retired
    work's HIP events to new works; after a capture its watchdog thread can query an event last
    recorded inside the capture, HIP refuses the query (hipErrorCapturedEvent) and the watchdog
    terminates the process (round-3 record).  The variable must be 0 before the
    process group is created; gloo groups never capture (their collectives run on the host).
    ``process_group=None`` is the default (WORLD) group, as for the collectives themselves."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    try:
        backend = dist.get_backend(process_group)
    except (RuntimeError, ValueError):
        return None
    if backend == "nccl" and os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE", "1") != "0":
        return ("the RCCL process group was created with TORCH_NCCL_CUDA_EVENT_CACHE on; set "
                "TORCH_NCCL_CUDA_EVENT_CACHE=0 before init_process_group to capture the step")
    return None


class Trainer:
    def __init__(self, model, config, device, lr=None, amp_dtype=torch.bfloat16, bucket_mb=32,
                 world_size=1, process_group=None, rank=0, seed=None, skip_nonfinite=True, use_graph=None,
                 graph_warmup=4, grad_wire_dtype=None, always_reduce=False):
        self.model = model
        self.device = device
        self.amp_dtype = amp_dtype
        self.rank = rank
        if seed is not None:
            reseed(seed, rank)
        core = model.ms_unet if hasattr(model, "ms_unet") else model
        dead = set()
        if hasattr(core, "dead_modules"):
            for m in core.dead_modules():
                dead.update(id(p) for p in m.parameters())
        decay, no_decay = [], []
        for name, p in model.named_parameters():
            if not p.requires_grad or id(p) in dead:
                continue
            (no_decay if is_no_decay(name, p) else decay).append((name, p))
        # reverse registration order ~ gradient-ready order during backward
        self.groups = [FlatGroup(decay[::-1], config.TRAIN.WEIGHT_DECAY, device),
                       FlatGroup(no_decay[::-1], 0.0, device)]
        # the dead branches' parameters are never updated: one 16-bit shadow each for the run, so
        # their no-grad forwards (side stream) read it instead of casting every weight every step
        # (16 cast launches per step at Swin-T); a write through the parameter (load_state_dict)
        # bumps its version and the ops cast it again (ops._shadow)
        for m in (core.dead_modules() if hasattr(core, "dead_modules") else []):
            for p in m.parameters():
                if p.is_floating_point() and p.dim() >= 2 and p.device.type == "cuda":
                    p._msu_shadow = p.detach().to(amp_dtype)
                    p._msu_shadow_ver = p._version
        opt = config.TRAIN.OPTIMIZER
        self.betas = tuple(opt.BETAS)
        self.eps = float(opt.EPS)
        # device-resident step scalars {lr, step}: AdamW reads them on the GPU, so a skipped
        # (non-finite) step is not counted without a host sync, and the launch is replayable
        self.hyper = torch.zeros(2, device=device, dtype=torch.float64)
        self.lr = float(config.TRAIN.BASE_LR if lr is None else lr)
        # GradScaler semantics (trainer.py:182,315-316): a step whose gradients hold an inf /
        # NaN leaves parameters and moments untouched
        self.skip_nonfinite = skip_nonfinite
        self.found_inf = torch.zeros(1, device=device, dtype=torch.float32)
        self._one = torch.ones((), device=device, dtype=torch.float32)
        t = config.TRAIN
        self.loss_fn = DynamicLoss(alpha=t.TVERSKY_LOSS_ALPHA, beta=t.TVERSKY_LOSS_BETA,
                                   tversky_bce_mix=t.LOSS_TVERSKY_BCE_MIX)
        self.world_size = world_size
        self.step_count = 0
        self._applied_base = 0  # AdamW step count not taken by this trainer (loaded checkpoints)
        self._shadow_fresh = False
        self.inv_world = torch.full((1,), 1.0 / world_size, device=device, dtype=torch.float32)
        # always_reduce: the bucketed all-reduce even for one rank (a 1-rank RCCL group exercises
        # the product DP path on one GPU)
        self.reducer = (GradBucketer(self.groups, int(bucket_mb * (1 << 20)), process_group, grad_wire_dtype)
                        if world_size > 1 or always_reduce else None)
        # HIP-graph replay of the step (see step()).  use_graph: True / False, or None = the
        # MSU_GRAPH environment switch: "1" always, "0" never, "auto" (default) = capture only
        # when the eager step is launch-bound (host issue time >= GRAPH_HOST_FRACTION of the
        # GPU time, measured on the last warmup step): the replay removes the host from the
        # critical path, but costs ~1-2 % of GPU time where the host is not on it
        on_gpu = torch.device(device).type == "cuda"
        mode = use_graph if use_graph is not None else switches.get("MSU_GRAPH")
        mode = {True: "1", False: "0"}.get(mode, str(mode))
        self.graph_mode = mode if on_gpu else "0"
        if self.graph_mode != "0" and self.reducer is not None and dist.get_backend(process_group) != "nccl":
            self.graph_mode = "0"  # gloo collectives run on the host: not capturable
        blocker = rccl_capture_blocker(self.reducer.pg) if self.reducer is not None else None
        if self.graph_mode != "0" and blocker:
            # never capture into a process group whose watchdog can abort the process;
            # every rank sees the same environment, so every rank stays eager together
            import warnings
            warnings.warn(f"HIP-graph replay disabled: {blocker}")
            self.graph_mode = "0"
        if self.graph_mode == "auto" and world_size > 1:
            # a captured multi-rank step has only been replayed on a 1-rank RCCL group
            # (tests/test_gpu_rccl.py): replay under DP only when asked for (MSU_GRAPH=1)
            self.graph_mode = "0"
        self.use_graph = self.graph_mode != "0"
        self._probe = []  # [(host seconds, start event, end event)] of the auto-mode probe steps
        self.graph_warmup = graph_warmup
        self._graph = None
        self._graph_failed = False
        self.dev_seed = torch.zeros(1, device=device, dtype=torch.int64)
        if self.use_graph:
            model_parts.set_device_seed(self.dev_seed)

    @property
    def lr(self):
        return self._lr

    @lr.setter
    def lr(self, value):
        self._lr = float(value)
        self.hyper[0:1].fill_(self._lr)

    def optimizer_steps(self):
        """AdamW steps actually applied (skipped non-finite steps excluded); syncs."""
        return int(self.hyper[1].item())

    def skipped_steps(self):
        """Training steps whose update was skipped (non-finite gradients); syncs."""
        return self.step_count - (self.optimizer_steps() - self._applied_base)

    def _reference_param_order(self):
        """The parameter list of the reference optimizer (trainer.py:130-152): every trainable
        parameter in named_parameters() order, the decay group first -- dead-branch
        parameters included (they are in the reference's groups, they just never get grads)."""
        decay, no_decay = [], []
        for name, p in self.model.named_parameters():
            if p.requires_grad:
                (no_decay if is_no_decay(name, p) else decay).append(p)
        return decay, no_decay

    def optimizer_state_dict(self):
        """This trainer's AdamW state in ``torch.optim.AdamW.state_dict()`` format, parameter
        indices in the reference's group order (what trainer.py:408 saves)."""
        decay, no_decay = self._reference_param_order()
        where = {}
        for g in self.groups:
            for p, off in zip(g.params, g.offsets):
                where[id(p)] = (g, off)
        step = torch.tensor(float(self.optimizer_steps()))
        state = {}
        for i, p in enumerate(decay + no_decay):
            if id(p) not in where:
                continue
            g, off = where[id(p)]
            n = p.numel()
            state[i] = {"step": step.clone(),
                        "exp_avg": g.exp_avg[off:off + n].view_as(p).detach().cpu().clone(),
                        "exp_avg_sq": g.exp_avg_sq[off:off + n].view_as(p).detach().cpu().clone()}
        common = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "amsgrad": False, "foreach": None,
                  "maximize": False, "capturable": False, "differentiable": False, "fused": None}
        groups = [dict(common, weight_decay=self.groups[0].weight_decay, params=list(range(len(decay)))),
                  dict(common, weight_decay=0.0, params=list(range(len(decay), len(decay) + len(no_decay))))]
        return {"state": state, "param_groups": groups}

    def load_optimizer_state_dict(self, sd):
        """Inverse of optimizer_state_dict (e.g. from a reference ``epoch_<n>.pth``)."""
        decay, no_decay = self._reference_param_order()
        where = {}
        for g in self.groups:
            for p, off in zip(g.params, g.offsets):
                where[id(p)] = (g, off)
        steps = set()
        with torch.no_grad():
            for i, p in enumerate(decay + no_decay):
                st = sd["state"].get(i, sd["state"].get(str(i)))
                if st is None or id(p) not in where:
                    continue
                g, off = where[id(p)]
                n = p.numel()
                g.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1))
                g.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(float(st["step"]))
        if len(steps) > 1:
            raise ValueError(f"per-parameter AdamW steps differ: {sorted(steps)}")
        if steps:
            st = steps.pop()
            self._applied_base += int(st) - self.optimizer_steps()
            self.hyper[1:2].fill_(st)
        self.lr = sd["param_groups"][0]["lr"]

    def num_params(self):
        return sum(g.count for g in self.groups)

    def set_epoch(self, epoch, config):
        t = config.TRAIN
        self.lr = cosine_lr(epoch, t.BASE_LR, t.WARMUP_EPOCHS, t.MAX_EPOCHS, t.WARMUP_LR, t.MIN_LR,
                            t.LR_SCHEDULER.WARMUP_PREFIX)

    def forward_loss(self, images, labels):
        with torch.autocast("cuda", dtype=self.amp_dtype, enabled=self.amp_dtype != torch.float32):
            out = self.model(images)
            return self.loss_fn(out, labels)

    def step(self, images, labels):
        """One training step; returns the (device) loss of this rank's batch.

        After ``graph_warmup`` eager steps (lazy library / kernel-attribute initialisation,
        the all-reduce accumulation counts of step 0), the whole device side of the step --
        forward, DynamicLoss, backward with its side-stream work, the bucketed all-reduce,
        the non-finite check, AdamW, the gradient reset and the bf16 shadow refresh -- is
        captured once into a HIP graph and replayed: one launch per step instead of ~1300.
        Inputs are copied into the graph's static buffers; dropout keeps drawing fresh masks
        (device-side seed counter, drop-path pools redrawn inside the graph)."""
        if not self.model.training:  # Module.train() walks all ~400 modules: ~1 ms of host time
            self.model.train()
        if self.graph_mode == "auto" and self.step_count >= self.graph_warmup and self._graph is None:
            self._decide_graph()
        if self.use_graph and self.step_count >= self.graph_warmup:
            if self._graph is not None and self.loss_fn is not self._graph_loss_fn:
                self.invalidate_graph()  # the captured step holds the old loss module
            if self._graph is None and not self._graph_failed:
                self._capture(images, labels)
            if self._graph is not None:
                return self._replay(images, labels)
        return self._eager_step(images, labels)

    # ------------------------------------------------------------------ eager / captured body
    def _device_step(self, images, labels):
        """Everything the step enqueues on the GPU (the body that is captured)."""
        if self.use_graph:
            self.dev_seed.add_(1)  # new attention-dropout masks per step / replay
            model_parts.refresh_drop_pools()
        ops.set_grad_ready_callback(self.reducer._hook if self.reducer is not None else None)
        if self.reducer is not None and torch.device(self.device).type == "cuda":
            self.reducer.main_stream = torch.cuda.current_stream(self.device)
        # the DynamicLoss forward (msu_dynloss_fwd3) zeroes the non-finite flag for this step; a
        # loss_fn swapped for something else leaves it to the fill below
        ops.set_step_flag(self.found_inf)
        try:
            loss = self.forward_loss(images, labels)
            self._flag_reset_by_loss = ops.step_flag_reset()
        finally:
            ops.set_step_flag(None)
        loss.backward(self._one)  # a persistent seed: no ones_like fill per step
        if self.reducer is not None:
            self.reducer.finish()
        ops.join_side_streams()  # weight gradients issued on the side stream
        inv = self.inv_world if self.world_size > 1 else None
        bf16 = self.amp_dtype == torch.bfloat16
        if bf16:
            # the bf16 shadow's parameter versions are marked now, while the GPU still has
            # backward work queued, not after the last launch of the step (it left the GPU idle
            # there); the shadow itself is refreshed after AdamW below
            for g in self.groups:
                g.mark_shadow()
        found = None
        wire_scaled = self.reducer is not None and self.reducer.scale is not None
        if self.skip_nonfinite or wire_scaled:
            # after the all-reduce: an inf on any rank reaches every rank's sum, so all ranks
            # skip together (an f16-wire overflow included: it must never reach AdamW)
            found = self.found_inf
            if not self._flag_reset_by_loss:
                found.zero_()
            ops.nonfinite_(self.groups[0].grad, found, self.groups[1].grad)
            if wire_scaled:
                self.reducer.update_scale(found)
        ops.step_advance_(self.hyper, found)
        for g in self.groups:
            # the gradient reset and (bf16) the shadow refresh ride in AdamW's pass: no fill and
            # no re-read of the parameters for the cast (a skipped step leaves the shadow as is
            # and zeroes the gradient too)
            ops.adamw_dev_(g.data, g.grad, g.exp_avg, g.exp_avg_sq, self.hyper, self.betas[0], self.betas[1],
                           self.eps, g.weight_decay, inv_scale=inv, found_inf=found,
                           shadow=g.shadow if bf16 else None, zero_grad=True)
            if bf16:  # keeps evaluation between steps on the updated weights
                g.transpose_shadow()
        return loss.detach()

    GRAPH_HOST_FRACTION = 0.9

    def _decide_graph(self):
        """auto mode: graph replay iff the probed eager step was launch-bound."""
        if not self._probe:
            self.use_graph = False
            return
        # the probe step with the shorter GPU time: a step that stalled on a one-off (allocator
        # growth, a lazy library load: the host waits on the GPU there) reads host ~ GPU
        self._probe[-1][2].synchronize()
        timed = [(e0.elapsed_time(e1) * 1e-3, host_s) for host_s, e0, e1 in self._probe]
        gpu_s, host_s = min(timed)
        self.graph_probe = {"host_ms": round(host_s * 1e3, 3), "gpu_ms": round(gpu_s * 1e3, 3)}
        self.use_graph = host_s >= self.GRAPH_HOST_FRACTION * gpu_s
        self.graph_mode = "1" if self.use_graph else "0"

    def _eager_step(self, images, labels):
        if self.amp_dtype == torch.bfloat16 and not self._shadow_fresh:
            for g in self.groups:
                g.refresh_shadow()
        self._shadow_fresh = False
        probe = self.graph_mode == "auto" and self.graph_warmup - 2 <= self.step_count <= self.graph_warmup - 1
        if probe:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            t0 = time.perf_counter()
        loss = self._device_step(images, labels)
        if probe:
            host = time.perf_counter() - t0
            e1.record()
            self._probe.append((host, e0, e1))
        self.step_count += 1
        # the next step's refresh is skipped; a write through a parameter in between bumps its
        # version and the Linear ops cast that weight themselves (ops._shadow)
        self._shadow_fresh = self.amp_dtype == torch.bfloat16
        return loss

    def _param_versions(self):
        return sum(p._version for g in self.groups for p in g.params)

    def _capture(self, images, labels):
        """Capture _device_step into a HIP graph (nothing executes during capture)."""
        blocker = rccl_capture_blocker(self.reducer.pg) if self.reducer is not None else None
        if blocker:  # use_graph forced on after construction: refuse instead of aborting later
            raise RuntimeError(f"cannot capture the training step: {blocker}")
        if self.amp_dtype == torch.bfloat16 and not self._shadow_fresh:
            for g in self.groups:
                g.refresh_shadow()
        self._sx = images.detach().clone()
        self._sy = labels.detach().clone()
        torch.cuda.synchronize(self.device)
        if self.reducer is not None and dist.is_initialized():
            # the process group's watchdog thread polls its eager works' events every ~100 ms;
            # one it has not retired yet, queried while the capture below holds the RCCL stream,
            # can fail with hipErrorCapturedEvent and terminate the process (seen once in the
            # r06ah suite, in a process's third capture).  The warmup's works are complete
            # (synchronize above): give the watchdog a few polls to drop them first
            time.sleep(0.3)
        graph = torch.cuda.CUDAGraph()
        # The captured step is single-stream: with the weight-gradient / dead-branch side
        # stream forked into the capture, the ROCm 7.2 graph executor's parallel branches gave
        # run-to-run different gradients (tests/test_gpu_graph.py, tools/determinism_check.py;
        # deterministic again with DEBUG_HIP_FORCE_GRAPH_QUEUES=1).  Replay is only chosen
        # when the step is launch-bound, where the side-stream overlap matters least.
        # MSU_GRAPH_SIDE=1 keeps the side stream (A/B switch).
        side_prev = ops._side_enabled
        if switches.get("MSU_GRAPH_SIDE") != "1":
            ops._side_enabled = False
        try:
            # thread_local: the process group's watchdog thread keeps querying its events while
            # this thread captures; in the default "global" mode such a query from another
            # thread fails the capture (hipErrorStreamCaptureUnsupported, tests/test_gpu_rccl.py)
            if self.reducer is not None:
                self.reducer.capturing = True
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                loss = self._device_step(self._sx, self._sy)
        except Exception as e:  # noqa: BLE001 -- any capture failure: stay eager, loudly
            if self.reducer is not None:
                self.reducer.capturing = False
            ops._side_enabled = side_prev
            # the aborted capture left accumulation counts, launched flags and captured work
            # handles in the reducer: a later eager step must start from a clean bucket state
            if self.reducer is not None:
                self.reducer.reset()
            ops._side_keep.clear()
            self._sx = self._sy = None
            torch.cuda.synchronize(self.device)
            if self.world_size > 1:
                # one rank silently falling back to eager while the others replay would
                # desynchronise the collectives: fail on every rank instead
                raise RuntimeError(f"HIP graph capture of the data-parallel training step failed: {e!r}") from e
            import warnings
            warnings.warn(f"HIP graph capture of the training step failed ({e!r}); continuing eagerly")
            self._graph_failed = True
            return
        if self.reducer is not None:
            self.reducer.capturing = False
            # (bucket, thread, "hook" | "finish", capturing) of the captured collectives: every one
            # from finish() on this thread (tests/test_gpu_rccl.py checks it)
            self.capture_launches = list(self.reducer.last_launches)
        ops._side_enabled = side_prev
        self._graph = graph
        self._graph_loss_fn = self.loss_fn
        self._sloss = loss
        self._versions = self._param_versions()

    def _replay(self, images, labels):
        if images.shape != self._sx.shape or labels.shape != self._sy.shape or \
                images.dtype != self._sx.dtype or labels.dtype != self._sy.dtype:
            # the graph is specialised to the captured batch: anything else (a short last
            # batch, another resolution) runs eagerly instead of broadcasting into the buffers
            return self._eager_step(images, labels)
        v = self._param_versions()
        if v != self._versions:
            # a write through a parameter (load_state_dict, p.copy_) since the last step: the
            # captured forward reads the bf16 shadow, so re-derive it before replaying
            if self.amp_dtype == torch.bfloat16:
                for g in self.groups:
                    g.refresh_shadow()
            self._versions = v
        self._sx.copy_(images)
        self._sy.copy_(labels)
        self._graph.replay()
        self.step_count += 1
        return self._sloss.clone()

    def invalidate_graph(self):
        """Drop the captured step; the next step captures again.  The replay repeats the
        captured kernels with the captured Python decisions: call this after changing the
        model's structure, its train/eval-dependent settings or frozen parameters (a new
        loss_fn and writes through parameters are detected by step() itself)."""
        self._graph = None
        self._graph_failed = False
