"""The MS-UNet hot-path operators, registered as ``torch.library`` custom ops.

Every operator is ``torch.ops.msunet.<name>``: a schema, a CUDA (HIP) kernel that launches
hand-written gfx950 kernels from ``libmsunet_hip.so`` through the C-ABI
(``include/msunet_hip.h``) on the current HIP stream, a fake (meta) kernel for shape
propagation, and an autograd formula attached with ``torch.library.register_autograd``.
There is no CPU / eager fallback: a CPU tensor has no kernel (the dispatcher raises) and a
missing library raises ``_lib.HipLibraryError``.

Activations are float32 (parity mode), bfloat16 (training mode) or float16 (the reference's
``torch.amp.autocast('cuda', dtype=torch.float16)`` step, trainer.py:308), chosen by the
autocast state of the caller; statistics, parameters and parameter gradients are float32.

The public functions below (``layer_norm``, ``linear``, ``window_attention`` ...) are what the
modules in ``network/`` call.  They cast the activation to the autocast dtype and invoke the
registered op.  (A plain ``autograd.Function`` route around the dispatcher measured equal on
the GPU-bound 1024^2 step, r02c 50.50 vs 50.57 ms: gone.)
"""
import ctypes
import functools

import torch

from . import _lib, switches

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
_LOW = (torch.bfloat16, torch.float16)


# ----------------------------------------------------------------------------- helpers
def _dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported activation dtype {t.dtype} (float32 / bfloat16 / float16)") from None


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("msunet HIP ops need tensors on a HIP device (no CPU fallback)")


def _p(t):
    return None if t is None else t.data_ptr()


_raw_stream = torch._C._cuda_getCurrentRawStream


def _s(t):
    """hipStream_t (as int) of the current stream on t's device.  The raw getter skips the
    Python Stream object torch.cuda.current_stream builds: a few us per launch of host time,
    which is what bounds the short stage-2/3 kernels."""
    return _raw_stream(t.get_device())


def act_dtype(device_type="cuda"):
    """Activation dtype for the current context: autocast dtype if enabled, else float32."""
    if torch.is_autocast_enabled(device_type):
        return torch.get_autocast_dtype(device_type)
    return torch.float32


def _f32(t):
    return t if (t.dtype == torch.float32 and t.is_contiguous()) else t.float().contiguous()


def _as(t, dtype):
    t = t if t.dtype == dtype else t.to(dtype)
    return t.contiguous()


# ----------------------------------------------------------------------------- registration
_LIB = torch.library.Library("msunet", "DEF")
_OPS = {}


def _define(name, schema, impl, fake, setup=None, backward=None):
    """Register ``torch.ops.msunet.<name>``: CUDA kernel, fake kernel, autograd formula."""
    _LIB.define(name + schema)
    _LIB.impl(name, impl, "CUDA")
    torch.library.register_fake("msunet::" + name, fake, lib=_LIB)
    if backward is not None:
        torch.library.register_autograd("msunet::" + name, backward, setup_context=setup, lib=_LIB)
    op = _OPS[name] = getattr(torch.ops.msunet, name).default
    return op


def registered_ops():
    """Names of the torch.ops.msunet operators."""
    return sorted(_OPS)


# ----------------------------------------------------------------------------- direct grads
# A trainer that keeps parameters and gradients in flat buffers (trainer.FlatGroup) marks
# its parameters ``_msu_direct``: the backward kernels then add straight into the
# preallocated ``.grad`` views (no temporary + AccumulateGrad add per parameter) and report
# each parameter to ``_grad_ready`` (the bucketed all-reduce) themselves.
_grad_ready = None


def set_grad_ready_callback(fn):
    global _grad_ready
    _grad_ready = fn


# Linear weight gradients that accumulate straight into .grad run on a side stream: nothing
# later in backward reads them, so they overlap the input-gradient chain (which is often
# latency-bound at stages 1-3) instead of sitting on it.  The trainer joins the side stream
# before the optimizer (join_side_streams) and the bucketed all-reduce is issued from it.
_side_enabled = switches.on("MSU_WGRAD_SIDE")
_side_streams = {}
# per-use switches of the side stream (tools/graph_side_probe.py bisects the forked capture)
_side_wgrad = True      # Linear weight gradients
_side_attn_tail = True  # attention relative-table / qkv-bias reductions


def side_stream(device):
    """The weight-gradient side stream of a device, or None when disabled (also while a
    single-stream HIP graph capture has switched it off) / never used."""
    device = torch.device(device)
    if device.type != "cuda" or not _side_enabled or not _side_streams:
        return None
    return _side_streams.get(device.index if device.index is not None else torch.cuda.current_device())


def _side_stream_for(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _side_streams.get(idx)
    if st is None:
        # lowest priority: when both streams have work queued, the dispatcher serves the
        # main (critical-path) stream's workgroups first
        # (low / equal priority measured equal, r02c; a high-priority main stream -0.4 %)
        st = _side_streams[idx] = torch.cuda.Stream(device=idx, priority=1)
    return st


def join_side_streams():
    """Current stream(s) wait for every weight-gradient side stream."""
    for idx, st in _side_streams.items():
        torch.cuda.current_stream(idx).wait_stream(st)


_join_queued = False


def _guard_side_write(p, ev):
    """p.grad was just updated on the side stream (event ev).  If autograd later accumulates
    another gradient into p on the main stream (e.g. the qkv bias: its Linear adds db here,
    the attention op returns the padded tokens' share), that AccumulateGrad must wait for it:
    a tensor hook on p makes the current stream wait for the last such event first."""
    p = getattr(p, "_msu_param", p)  # a param_view: guard its parameter
    p._msu_side_event = ev
    _side_event_params.append(p)
    if not getattr(p, "_msu_side_hooked", False):
        def hook(grad, p=p):
            # called with None when the backward that owns p returned no gradient (direct
            # accumulation): nothing will be added, nothing to wait for
            e = getattr(p, "_msu_side_event", None)
            if grad is not None and e is not None:
                torch.cuda.current_stream(p.device).wait_event(e)
            return grad
        p.register_hook(hook)
        p._msu_side_hooked = True


# Tensors a side-stream kernel is still reading.  record_stream only keeps their memory from
# being reused; it does not stop autograd from accumulating into them IN PLACE: a gradient
# returned for two inputs (the add-LN backward hands the same `da` to the residual and to the
# branch) is "stealable" by autograd's InputBuffer once its use count drops to one, and the
# main stream would then add into it while a side-stream weight gradient still reads it.  One
# extra reference per tensor, held until the end-of-backward join, keeps it out of reach.
_side_keep = []
# parameters whose _msu_side_event was set in this backward: cleared at its end, so no later
# wait (a hook, _linbwd) orders on an event of an earlier step or from outside a capture
_side_event_params = []


# Residual-gradient handoff.  A Swin block whose input x is a plain tensor (a stage's first
# block) feeds x to two ops: norm1's LayerNorm and norm2's residual-add LayerNorm (x + attn).
# Autograd would sum the two gradients of x with an ATen add (14 launches per Swin-T step, 50 M
# elements each at stage 0).  Both ops carry the same handoff key instead: norm2's backward --
# which always runs first (attn(norm1(x)) feeds norm2) -- parks its gradient of x here and
# returns none for it, and norm1's backward pops it and adds it inside the LayerNorm backward
# kernel (the add-mode residual-gradient input).  Cleared at the end of every backward.
# The same key extends to a stage input's other readers (MSUNetSys.forward_features: the skip
# fusions' skip halves and the central decoders' PatchExpand Linears, model_parts.py:775-829):
# their backwards, which run before the stage's first block, park their input gradients too
# (up to three per key: msu_layernorm_bwd3's dres / dres2 / dres3).  A reader whose backward
# comes after the adder's (key closed) returns its gradient to autograd as usual, so the sum
# is right in any order.
_RES_HANDOFF = switches.on("MSU_RES_HANDOFF")
_res_handoff = {}  # key -> parked gradients of the keyed tensor, in park order
_res_closed = set()  # keys whose adder (the plain LayerNorm) ran in this backward
_res_keys = iter(range(1, 1 << 62))
res_handoff_calls = 0  # LayerNorm backwards that took parked gradients (tests)
res_parked = 0  # gradients parked (tests)
res_dropped = 0  # parked gradients no adder took (its tensor's gradient was not needed; tests)


def residual_handoff_key():
    """A fresh key pairing a plain layer_norm with the other readers of its input (the
    add_layer_norm over it; skip fusions / Linears given the same key), or 0 (no pairing:
    autograd sums the gradients)."""
    return next(_res_keys) if (_RES_HANDOFF and torch.is_grad_enabled()) else 0


def _park(key, g):
    """A reader's gradient of the keyed tensor, handed to the adder; False when there is no key
    or the adder already ran (the caller returns g to autograd)."""
    global res_parked
    if not key or key in _res_closed:
        return False
    _res_handoff.setdefault(key, []).append(g)
    res_parked += 1
    _join_at_end_of_backward()  # clears the mailbox at the end of this backward
    return True


def _take(key):
    """The adder's side: the parked gradients of key (and the key closed)."""
    if not key:
        return []
    _res_closed.add(key)
    _join_at_end_of_backward()
    return _res_handoff.pop(key, [])


def _end_of_backward():
    global _join_queued, res_dropped
    _join_queued = False
    _flush_ln()
    res_dropped += sum(len(v) for v in _res_handoff.values())
    _res_handoff.clear()
    _res_closed.clear()
    join_side_streams()
    _side_keep.clear()  # the main stream now waits for every side-stream read
    for p in _side_event_params:
        p._msu_side_event = None
    _side_event_params.clear()


def _join_at_end_of_backward():
    """Once per backward pass: when it ends, the main stream waits for the side stream, so
    .grad read after ``backward()`` returns is complete (overlap stays inside backward)."""
    global _join_queued
    if not _join_queued:
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
        _join_queued = True


def _direct(*params):
    return all(p is not None and getattr(p, "_msu_direct", False) and p.grad is not None for p in params)


def _notify(*params):
    if _grad_ready is not None:
        for p in params:
            if p is not None:
                _grad_ready(getattr(p, "_msu_param", p))


def param_view(param, shape):
    """A reshaped view of a parameter that the ops treat as the parameter itself: a trainer-
    direct parameter's view carries the viewed .grad (backward kernels add into it), the viewed
    16-bit shadow and the owner (notified to the gradient bucketer, side-stream guards).  E.g.
    PatchEmbed's [C, Cin, p, p] conv weight as the [C, Cin*p*p] Linear weight of its im2col GEMM."""
    v = param.view(shape)
    if _direct(param):
        v.grad = param.grad.view(shape)
        v._msu_direct = True
        v._msu_param = param
        sh = getattr(param, "_msu_shadow", None)
        if sh is not None:
            v._msu_shadow = sh.view(shape)
            v._msu_shadow_ver = getattr(param, "_msu_shadow_ver", -1)
    return v


def _ln_grads(ctx, C, device):
    """(dgamma, dbeta, accumulate, direct) buffers for a LayerNorm backward; (None, None, ...)
    with direct parameters under MSU_LN_DEFER: the kernel writes only its partial rows, summed
    into .grad later by _ln_finish's batch."""
    w, b = ctx.affine
    ctx.ln_deferred = False
    if _direct(w, b):
        if _LN_DEFER and C % 4 == 0 and w.grad.data_ptr() % 16 == 0 and b.grad.data_ptr() % 16 == 0:
            ctx.ln_deferred = True  # (16-B rows and outputs: msu_colsum_batch's float4 sums)
            return None, None, 1, True
        return w.grad, b.grad, 1, True
    dw, db = torch.empty(2, C, device=device, dtype=torch.float32)  # contiguous: one reduction
    return dw, db, 0, False


# Deferred LayerNorm parameter gradients (MSU_LN_DEFER): a LayerNorm backward with trainer-
# direct gamma / beta writes its [nparts][2C] partial rows and ends there; the partials of the
# LayerNorms of one width (a stage) are summed into .grad by one msu_colsum_batch launch when the
# width changes, and the rest at the end of backward.  Each kernel's in-kernel tail reduction
# (last-arriving blocks summing ~1 MB of partials, 8-15 us at the end of every launch, r06ac)
# leaves its critical path; the parameters are notified to the gradient bucketer after the batch.
_LN_DEFER = switches.on("MSU_LN_DEFER")
_ln_pending = []  # (part, nparts, C, gamma, beta)
ln_batches = 0  # batched reductions launched (tests)


def _flush_ln():
    """Sum the pending LayerNorm partials into their parameters' .grad (one launch per 48 rows
    of segments), then notify the parameters."""
    global ln_batches
    if not _ln_pending:
        return
    parts, strides, nps, ns, outs = [], [], [], [], []
    for part, n, C, w, b in _ln_pending:
        for off, g in ((0, w.grad), (C, b.grad)):
            parts.append(part.data_ptr() + 4 * off)
            strides.append(2 * C)
            nps.append(n)
            ns.append(C)
            outs.append(g.data_ptr())
    k = len(parts)
    P = ctypes.c_void_p * k
    _lib.call("msu_colsum_batch", k, P(*parts), (ctypes.c_long * k)(*strides), (ctypes.c_int * k)(*nps),
              (ctypes.c_int * k)(*ns), P(*outs), 1, _s(_ln_pending[0][0]))
    ln_batches += 1
    pend = list(_ln_pending)
    _ln_pending.clear()
    for _, _, _, w, b in pend:
        _notify(w, b)


def _ln_finish(ctx, part, n, C):
    """After a LayerNorm backward with direct parameters: register its partials (deferred) or
    notify (reduced in the kernel)."""
    w, b = ctx.affine
    if not ctx.ln_deferred:
        _notify(w, b)
        return
    if _ln_pending and _ln_pending[-1][2] != C:
        _flush_ln()
    _ln_pending.append((part, n, C, w, b))
    _join_at_end_of_backward()


def _ln_parts(rows, C, device):
    n = _lib.lib().msu_ln_part_blocks(rows, C)
    return n, torch.empty(n * 3 * C, device=device, dtype=torch.float32)


IN_PLAIN, IN_ADD, IN_MERGE, IN_D2S2 = 0, 1, 2, 3


def _stats(x, rows):
    return (torch.empty(rows, device=x.device, dtype=torch.float32),
            torch.empty(rows, device=x.device, dtype=torch.float32))


# ----------------------------------------------------------------------------- LayerNorm
def _ln_impl(x, w, b, eps, handoff=0):
    _need_cuda(x)
    x = x.contiguous()
    C = x.shape[-1]
    rows = x.numel() // C
    y = torch.empty_like(x)
    mean, rstd = _stats(x, rows)
    _lib.call("msu_layernorm_fwd", _dt(x), IN_PLAIN, _p(x), None, None, 1, None, _p(w), _p(b),
              _p(y), _p(mean), _p(rstd), rows, C, 0, 0, 0, eps, _s(x))
    return y, mean, rstd


def _ln_fake(x, w, b, eps, handoff=0):
    rows = x.numel() // x.shape[-1]
    return torch.empty_like(x), x.new_empty(rows, dtype=torch.float32), x.new_empty(rows, dtype=torch.float32)


def _ln_setup(ctx, inputs, output):
    x, w, b = inputs[:3]  # layer_norm (+ handoff), merge_layer_norm, d2s_layer_norm
    ctx.save_for_backward(x.contiguous(), w, output[1], output[2])
    ctx.affine = (w, b)
    ctx.handoff = inputs[4] if len(inputs) > 4 else 0
    ctx.set_materialize_grads(False)


def _ln_backward(ctx, dy, _dm, _dr):
    global res_handoff_calls
    x, w, mean, rstd = ctx.saved_tensors
    res = _take(ctx.handoff)  # the other readers' gradients of x (the paired add-LN's first)
    if dy is None:
        return (functools.reduce(torch.add, res) if res else None), None, None, None, None
    dy = _as(dy, x.dtype)
    C = x.shape[-1]
    rows = x.numel() // C
    dx = torch.empty_like(x)
    dw, db, acc, direct = _ln_grads(ctx, C, x.device)
    n, part = _ln_parts(rows, C, x.device)
    if res:
        # the add-mode backward: dx = LN'(dy) + res (+ res2 + res3) in one pass, one rounding
        # (no branch output: scale null; a fourth reader's gradient, not on the model's path, is
        # folded in by an add first)
        res = [_as(r, x.dtype).contiguous() for r in res]
        if len(res) > 3:
            res = res[:2] + [functools.reduce(torch.add, res[2:])]
        res_handoff_calls += 1
        r2 = res[1] if len(res) > 1 else None
        r3 = res[2] if len(res) > 2 else None
        _lib.call("msu_layernorm_bwd3", _dt(x), IN_ADD, _p(dy), _p(x), _p(res[0]), _p(r2), _p(r3), _p(w),
                  _p(mean), _p(rstd), _p(dx), None, None, rows // x.shape[0], _p(part), n, _p(dw), _p(db), rows, C,
                  0, 0, 0, acc, _s(x))
    else:
        _lib.call("msu_layernorm_bwd", _dt(x), IN_PLAIN, _p(dy), _p(x), None, _p(w), _p(mean), _p(rstd),
                  _p(dx), None, None, 1, _p(part), n, _p(dw), _p(db), rows, C, 0, 0, 0, acc, _s(x))
    if direct:
        _ln_finish(ctx, part, n, C)
        return dx, None, None, None, None
    return dx, dw, db, None, None


_layer_norm = _define("layer_norm",
                      "(Tensor x, Tensor weight, Tensor bias, float eps, int handoff=0) -> (Tensor, Tensor, Tensor)",
                      _ln_impl, _ln_fake, _ln_setup, _ln_backward)


def layer_norm(x, weight, bias, eps=1e-5, handoff=0):
    """nn.LayerNorm(C) over the last dim; x keeps its (autocast) dtype.  handoff: a
    ``residual_handoff_key()`` shared with the add_layer_norm that also reads x (its gradient of
    x is added inside this op's backward kernel)."""
    return _layer_norm(_as(x, act_dtype()), _f32(weight), _f32(bias), float(eps), int(handoff))[0]


def _add_ln_impl(a, branch, scale, w, b, eps, handoff=0):
    """s = a + scale[sample] * branch ; y = LN(s)."""
    _need_cuda(a, branch)
    a, branch = a.contiguous(), branch.contiguous()
    C = a.shape[-1]
    rows = a.numel() // C
    rps = rows // a.shape[0]
    s = torch.empty_like(a)
    y = torch.empty_like(a)
    mean, rstd = _stats(a, rows)
    _lib.call("msu_layernorm_fwd", _dt(a), IN_ADD, _p(a), _p(branch), _p(scale), rps, _p(s), _p(w),
              _p(b), _p(y), _p(mean), _p(rstd), rows, C, 0, 0, 0, eps, _s(a))
    return s, y, mean, rstd


def _add_ln_fake(a, branch, scale, w, b, eps, handoff=0):
    rows = a.numel() // a.shape[-1]
    return (torch.empty_like(a), torch.empty_like(a), a.new_empty(rows, dtype=torch.float32),
            a.new_empty(rows, dtype=torch.float32))


def _add_ln_setup(ctx, inputs, output):
    a, branch, scale, w, b, eps, handoff = inputs
    s, y, mean, rstd = output
    ctx.save_for_backward(s, w, mean, rstd, scale)
    ctx.rps = (a.numel() // a.shape[-1]) // a.shape[0]
    ctx.affine = (w, b)
    ctx.handoff = handoff
    ctx.set_materialize_grads(False)


def _add_ln_backward(ctx, ds, dy, _dm, _dr):
    s, w, mean, rstd, scale = ctx.saved_tensors
    C = s.shape[-1]
    rows = s.numel() // C
    if dy is None:
        dy = torch.zeros_like(s)
    dy = _as(dy, s.dtype)
    ds = None if ds is None else _as(ds, s.dtype)
    da = torch.empty_like(s)
    dbr = torch.empty_like(s) if scale is not None else None
    dw, dbb, acc, direct = _ln_grads(ctx, C, s.device)
    n, part = _ln_parts(rows, C, s.device)
    _lib.call("msu_layernorm_bwd", _dt(s), IN_ADD, _p(dy), _p(s), _p(ds), _p(w), _p(mean), _p(rstd),
              _p(da), _p(dbr), _p(scale), ctx.rps, _p(part), n, _p(dw), _p(dbb), rows, C, 0, 0, 0, acc, _s(s))
    if direct:
        _ln_finish(ctx, part, n, C)
        dw = dbb = None
    dbr = dbr if dbr is not None else da
    if _park(ctx.handoff, da):
        # a's other reader is the paired plain LayerNorm, whose backward runs later and adds da
        # in its kernel: autograd sees no gradient for a here
        return None, dbr, None, dw, dbb, None, None
    return da, dbr, None, dw, dbb, None, None


_add_layer_norm = _define(
    "add_layer_norm",
    "(Tensor a, Tensor branch, Tensor? scale, Tensor weight, Tensor bias, float eps, int handoff=0)"
    " -> (Tensor, Tensor, Tensor, Tensor)",
    _add_ln_impl, _add_ln_fake, _add_ln_setup, _add_ln_backward)


def add_layer_norm(a, branch, scale, weight, bias, eps=1e-5, handoff=0):
    """(s, LN(s)) with s = a + scale[sample] * branch (torchvision block residual with
    StochasticDepth 'row', fused with the next norm).  handoff: the key of the plain layer_norm
    that also reads ``a`` (see ``residual_handoff_key``)."""
    dt = act_dtype()
    sc = None if scale is None else _f32(scale)
    s, y, _, _ = _add_layer_norm(_as(a, dt), _as(branch, dt), sc, _f32(weight), _f32(bias), float(eps),
                                 int(handoff))
    return s, y


def _merge_ln_impl(x, w, b, eps):
    _need_cuda(x)
    x = x.contiguous()
    B, H, W, C = x.shape
    rows = B * (H // 2) * (W // 2)
    y = torch.empty(B, rows // B, 4 * C, device=x.device, dtype=x.dtype)
    mean, rstd = _stats(x, rows)
    _lib.call("msu_layernorm_fwd", _dt(x), IN_MERGE, _p(x), None, None, 1, None, _p(w), _p(b),
              _p(y), _p(mean), _p(rstd), rows, 4 * C, H, W, C, eps, _s(x))
    return y, mean, rstd


def _merge_ln_fake(x, w, b, eps):
    B, H, W, C = x.shape
    rows = B * (H // 2) * (W // 2)
    return (x.new_empty(B, rows // B, 4 * C), x.new_empty(rows, dtype=torch.float32),
            x.new_empty(rows, dtype=torch.float32))


def _merge_ln_backward(ctx, dy, _dm, _dr):
    x, w, mean, rstd = ctx.saved_tensors
    if dy is None:
        return None, None, None, None
    B, H, W, C = x.shape
    rows = B * (H // 2) * (W // 2)
    dy = _as(dy, x.dtype)
    dx = torch.empty_like(x)
    dw, db, acc, direct = _ln_grads(ctx, 4 * C, x.device)
    n, part = _ln_parts(rows, 4 * C, x.device)
    _lib.call("msu_layernorm_bwd", _dt(x), IN_MERGE, _p(dy), _p(x), None, _p(w), _p(mean), _p(rstd),
              _p(dx), None, None, 1, _p(part), n, _p(dw), _p(db), rows, 4 * C, H, W, C, acc, _s(x))
    if direct:
        _ln_finish(ctx, part, n, 4 * C)
        return dx, None, None, None
    return dx, dw, db, None


_merge_layer_norm = _define("merge_layer_norm",
                            "(Tensor x, Tensor weight, Tensor bias, float eps) -> (Tensor, Tensor, Tensor)",
                            _merge_ln_impl, _merge_ln_fake, _ln_setup, _merge_ln_backward)


def merge_layer_norm(x, weight, bias, eps=1e-5):
    """PatchMerging gather (x0,x1,x2,x3 order) + LayerNorm(4C): [B,H,W,C] -> [B,HW/4,4C]."""
    return _merge_layer_norm(_as(x, act_dtype()), _f32(weight), _f32(bias), float(eps))[0]


def _d2s_ln_impl(x, w, b, eps):
    _need_cuda(x)
    x = x.contiguous()
    B, H, W, C4 = x.shape
    c = C4 // 4
    rows = B * 4 * H * W
    y = torch.empty(B, 4 * H * W, c, device=x.device, dtype=x.dtype)
    mean, rstd = _stats(x, rows)
    _lib.call("msu_layernorm_fwd", _dt(x), IN_D2S2, _p(x), None, None, 1, None, _p(w), _p(b),
              _p(y), _p(mean), _p(rstd), rows, c, H, W, 0, eps, _s(x))
    return y, mean, rstd


def _d2s_ln_fake(x, w, b, eps):
    B, H, W, C4 = x.shape
    rows = B * 4 * H * W
    return (x.new_empty(B, 4 * H * W, C4 // 4), x.new_empty(rows, dtype=torch.float32),
            x.new_empty(rows, dtype=torch.float32))


def _d2s_ln_backward(ctx, dy, _dm, _dr):
    x, w, mean, rstd = ctx.saved_tensors
    if dy is None:
        return None, None, None, None
    B, H, W, C4 = x.shape
    c = C4 // 4
    rows = B * 4 * H * W
    dy = _as(dy, x.dtype)
    dx = torch.empty_like(x)
    dw, db, acc, direct = _ln_grads(ctx, c, x.device)
    n, part = _ln_parts(rows, c, x.device)
    _lib.call("msu_layernorm_bwd", _dt(x), IN_D2S2, _p(dy), _p(x), None, _p(w), _p(mean), _p(rstd),
              _p(dx), None, None, 1, _p(part), n, _p(dw), _p(db), rows, c, H, W, 0, acc, _s(x))
    if direct:
        _ln_finish(ctx, part, n, c)
        return dx, None, None, None
    return dx, dw, db, None


_d2s_layer_norm = _define("d2s_layer_norm",
                          "(Tensor x, Tensor weight, Tensor bias, float eps) -> (Tensor, Tensor, Tensor)",
                          _d2s_ln_impl, _d2s_ln_fake, _ln_setup, _d2s_ln_backward)


def d2s_layer_norm(x, weight, bias, eps=1e-5):
    """PatchExpand rearrange 'b h w (p1 p2 c) -> b (h p1) (w p2) c' (p=2) + LayerNorm(c)."""
    return _d2s_layer_norm(_as(x, act_dtype()), _f32(weight), _f32(bias), float(eps))[0]


# ----------------------------------------------------------------------------- attention
# dropout keep bits stored by the forward for the backward (False: the backward re-hashes the
# mask from the seed, as the f32 parity kernels always do; bit-identical, equal speed since the
# xorshift streams, r02c -- the stored form is the default, the re-hash stays for the tests)
_ATTN_KEEP = True

_ATTN_AUX = switches.on("MSU_ATTN_AUX")


def _attn_fwd_ws(dt, C, nh):
    """msu_win_attn_fwd_workspace restated (window_attention_mfma.hip aux_floats): the 16-bit
    forward's aux region -- relative-bias image nh x 4096 f32, the 16-bit qkv-bias row, a zero
    row; f32 kernels 1.  Python-side so fake kernels propagate shapes without the library
    (tests/test_capi.py checks it against the library over a grid of shapes)."""
    return nh * 4096 + (6 * C + 1) // 2 + 4 if dt in _LOW else 1


def _nwin(B, H, W):
    return B * (-(-H // 7)) * (-(-W // 7))


def _attn_bwd_ws(dt, B, H, W, C, nh):
    """msu_win_attn_bwd_workspace restated: 16-bit -- aux region + per-block partials of the
    relative-table gradient (169 x nh) and the qkv-bias gradient (3C), over head_blocks(nwin,
    1024 / nh) blocks (a multiple of 8); f32 -- min(2048 / nh, nwin) blocks of nh x 49^2 + 3C
    partials and one nh x 49^2 image."""
    nwin = _nwin(B, H, W)
    if dt in _LOW:
        cap = max(8, (1024 // nh) // 8 * 8)
        parts = (min(nwin, cap) + 7) // 8 * 8
        return _attn_fwd_ws(dt, C, nh) + parts * nh * 169 + parts * 3 * C
    nblk = max(1, min(2048 // nh, nwin))
    return nblk * nh * 49 * 49 + nh * 49 * 49 + nblk * 3 * C


def _attn_keep_words(dt, B, H, W, nh):
    """msu_win_attn_keep_words restated: 128 keep-bit words per window x head (16-bit kernels)."""
    return _nwin(B, H, W) * nh * 128 if dt in _LOW else 0


def _attn_ws_numel(dt, B, H, W, C, nh):
    """Workspace floats of a 16-bit attention forward that its backward reuses: the forward's aux
    region (relative-bias image, bias / zero rows) stays valid for the backward, which then skips
    its own aux launch (msu_win_attn_bwd2 with table = null); f32: the forward's only."""
    n = _attn_fwd_ws(dt, C, nh)
    if dt in _LOW and _ATTN_AUX:
        n = max(n, _attn_bwd_ws(dt, B, H, W, C, nh))
    return n


def _attn_impl(qkv, qkv_bias, table, num_heads, shift, p_drop, seed, seed_dev):
    _need_cuda(qkv)
    qkv = qkv.contiguous()
    B, H, W, C3 = qkv.shape
    C = C3 // 3
    out = torch.empty(B, H, W, C, device=qkv.device, dtype=qkv.dtype)
    ws = torch.empty(_attn_ws_numel(qkv.dtype, B, H, W, C, num_heads), device=qkv.device, dtype=torch.float32)
    # the dropout keep bits, written by the forward for the backward (16-bit dtypes)
    keep = torch.empty(_attn_keep_words(qkv.dtype, B, H, W, num_heads) if p_drop > 0 and _ATTN_KEEP else 0,
                       device=qkv.device, dtype=torch.int32)
    _lib.call("msu_win_attn_fwd", _dt(qkv), _p(qkv), _p(qkv_bias), _p(table), _p(out), _p(ws), B, H, W,
              C, num_heads, shift, float(p_drop), seed, _p(seed_dev), _p(keep) if keep.numel() else None,
              _s(qkv))
    return out, keep, ws


def _attn_fake(qkv, qkv_bias, table, num_heads, shift, p_drop, seed, seed_dev):
    B, H, W, C3 = qkv.shape
    kw = _attn_keep_words(qkv.dtype, B, H, W, num_heads) if (p_drop > 0 and _ATTN_KEEP) else 0
    return (qkv.new_empty(B, H, W, C3 // 3), qkv.new_empty(kw, dtype=torch.int32),
            qkv.new_empty(_attn_ws_numel(qkv.dtype, B, H, W, C3 // 3, num_heads), dtype=torch.float32))


def _attn_setup(ctx, inputs, output):
    qkv, qkv_bias, table, num_heads, shift, p_drop, seed, seed_dev = inputs
    keep = output[1]
    ctx.mark_non_differentiable(keep, output[2])
    ctx.aux_ws = output[2]
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(qkv.contiguous(), qkv_bias, table, seed_dev, keep)
    # the parameter itself when it reached us uncast (trainer flat buffers: direct .grad)
    ctx.bias_param = qkv_bias if isinstance(qkv_bias, torch.nn.Parameter) else None
    ctx.table_param = table if isinstance(table, torch.nn.Parameter) else None
    ctx.cfg = (num_heads, shift, float(p_drop), seed)


def _attn_backward(ctx, dout, _dkeep, _dws=None):
    qkv, qkv_bias, table, seed_dev, keep = ctx.saved_tensors
    if dout is None:
        return None, None, None, None, None, None, None, None
    kp = _p(keep) if keep.numel() else None
    nh, shift, p_drop, seed = ctx.cfg
    B, H, W, C3 = qkv.shape
    C = C3 // 3
    dout = _as(dout, qkv.dtype)
    need = _attn_bwd_ws(qkv.dtype, B, H, W, C, nh)
    ws = getattr(ctx, "aux_ws", None)
    if ws is not None and _ATTN_AUX and qkv.dtype in _LOW and ws.numel() >= need:
        tbl = None  # the forward's aux region is still in ws: no second aux launch
    else:
        ws = torch.empty(need, device=qkv.device, dtype=torch.float32)
        tbl = _p(table)
    dqkv = torch.empty_like(qkv)
    bp, tp = ctx.bias_param, ctx.table_param
    if bp is not None and tp is not None and _side_enabled and _side_attn_tail and _direct(bp, tp):
        # parameter-gradient tail on the side stream: the relative-table / qkv-bias
        # reductions and their .grad adds.  The qkv bias's .grad has a second writer, its
        # Linear's db: on the side stream too when that Linear runs the two-kernel backward
        # (one stream, program order), or on the main stream in the one-pass backward
        # (_linbwd, stage 0), which runs later in this backward and first makes the main
        # stream wait on the event recorded below (bias._msu_side_event)
        # (the fork is a fresh torch event per call: a HIP graph capture of the step turns
        # every record / wait pair into its own edge)
        main = torch.cuda.current_stream(qkv.device)
        side = _side_stream_for(qkv.device)
        _lib.call("msu_win_attn_bwd2", _dt(qkv), _p(qkv), _p(qkv_bias), tbl, _p(dout), _p(dqkv),
                  None, None, _p(ws), B, H, W, C, nh, shift, p_drop, seed, _p(seed_dev), kp,
                  main.cuda_stream, -1)
        side.wait_stream(main)
        ws.record_stream(side)
        _side_keep.append(ws)
        with torch.cuda.stream(side):
            # the reductions add straight into .grad (no .grad adds behind them)
            _lib.call("msu_win_attn_bwd_tail2", _dt(qkv), _p(ws), _p(tp.grad), _p(bp.grad), B, H, W, C, nh, 1,
                      side.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(side)
        _guard_side_write(bp, ev)
        _guard_side_write(tp, ev)
        _join_at_end_of_backward()
        _notify(bp, tp)
        return dqkv, None, None, None, None, None, None, None
    dtable = torch.empty_like(table)
    dbias = torch.empty(3 * C, device=qkv.device, dtype=torch.float32)
    _lib.call("msu_win_attn_bwd", _dt(qkv), _p(qkv), _p(qkv_bias), tbl, _p(dout), _p(dqkv),
              _p(dtable), _p(dbias), _p(ws), B, H, W, C, nh, shift, p_drop, seed, _p(seed_dev), kp, _s(qkv))
    return dqkv, dbias, dtable, None, None, None, None, None


_window_attention = _define(
    "window_attention",
    "(Tensor qkv, Tensor qkv_bias, Tensor table, int num_heads, int shift, float p_drop, int seed, Tensor? seed_dev)"
    " -> (Tensor, Tensor, Tensor)",
    _attn_impl, _attn_fake, _attn_setup, _attn_backward)


def window_attention(qkv, qkv_bias, table, num_heads, shift, p_drop=0.0, seed=0, seed_dev=None):
    """torchvision shifted_window_attention core between the qkv and proj Linears.
    qkv: [B, H, W, 3C] (unpadded tokens) -> [B, H, W, C].  Dropout masks hash (seed, window,
    head, i, j); seed_dev: optional device int64 [1] mixed into the seed (per-step counter of a
    replayed HIP graph)."""
    C3 = qkv.shape[-1]
    if C3 % 3 or (C3 // 3) != num_heads * 32:
        raise ValueError(f"head_dim must be 32 (C={C3 // 3}, heads={num_heads})")
    return _window_attention(_as(qkv, act_dtype()), _f32(qkv_bias), _f32(table), int(num_heads),
                             int(shift), float(p_drop), int(seed) & ((1 << 63) - 1), seed_dev)[0]


# ----------------------------------------------------------------------------- fused qkv + attention
# Stage-0 fused unit (csrc/window_attention_mfma.hip attn_qkv_fwd_mfma): the qkv Linear and the
# window attention in one kernel, qkv never read back (in inference never written).  The backward
# is the existing ones in sequence: the proj Linear's, the attention backward (dqkv, relative
# table, padded-token bias share), then the qkv Linear's (one-pass msu_linear_bwd at stage 0).
# The kernel is the window-per-workgroup one with proj inside (msu_win_attn_qkv_fwd2);
# MSU_ATTN_QKV=0: the unfused qkv Linear + window_attention + proj path.  (A head-stationary
# form with independent waves, proj a separate Linear, was slower: r04d 165.6 / 165.8 vs 166.4 /
# 166.5 img/s, gone.)
_ATTN_QKV = switches.on("MSU_ATTN_QKV")
fused_qkv_calls = 0  # fused-unit launches (tests assert which path a forward took)


class _Ctx:
    """A stand-in autograd ctx for calling an op's backward function from another op's."""

    def __init__(self, saved, **kw):
        self.saved_tensors = saved
        self.__dict__.update(kw)


def _attn_qkv_impl(x, weight, bias, table, proj_weight, proj_bias, num_heads, shift, p_drop, seed, seed_dev,
                   store):
    """(y, o, qkv, keep): y = proj(o) when proj_weight is given (else y = o and o is empty),
    o = attention(x W^T + b); o / qkv are kept (written) only when ``store`` (training)."""
    global fused_qkv_calls
    _need_cuda(x)
    x = x.contiguous()
    B, H, W, C = x.shape
    dt = x.dtype
    w = _shadow(weight, dt)
    proj = proj_weight is not None
    wp = _shadow(proj_weight, dt) if proj else None
    y = torch.empty(B, H, W, C, device=x.device, dtype=dt)
    o = torch.empty(B, H, W, C, device=x.device, dtype=dt) if (proj and store) else x.new_empty(0)
    qkv = torch.empty(B, H, W, 3 * C, device=x.device, dtype=dt) if store else x.new_empty(0)
    ws = torch.empty(_attn_ws_numel(dt, B, H, W, C, num_heads) if store else _attn_fwd_ws(dt, C, num_heads),
                     device=x.device, dtype=torch.float32)
    keep = torch.empty(_attn_keep_words(dt, B, H, W, num_heads) if p_drop > 0 and _ATTN_KEEP else 0,
                       device=x.device, dtype=torch.int32)
    fused_qkv_calls += 1
    _lib.call("msu_win_attn_qkv_fwd2", _dt(x), _p(x), _p(w), _p(bias), _p(table), _p(wp),
              _p(proj_bias) if proj else None, _p(y), _p(o) if o.numel() else None, _p(qkv) if store else None,
              _p(keep) if keep.numel() else None, _p(ws), B, H, W, C, num_heads, shift, float(p_drop), seed,
              _p(seed_dev), _s(x))
    return y, o, qkv, keep, ws


def _attn_qkv_fake(x, weight, bias, table, proj_weight, proj_bias, num_heads, shift, p_drop, seed, seed_dev, store):
    B, H, W, C = x.shape
    kw = _attn_keep_words(x.dtype, B, H, W, num_heads) if (p_drop > 0 and _ATTN_KEEP) else 0
    nws = _attn_ws_numel(x.dtype, B, H, W, C, num_heads) if store else _attn_fwd_ws(x.dtype, C, num_heads)
    return (x.new_empty(B, H, W, C),
            x.new_empty(B, H, W, C) if (proj_weight is not None and store) else x.new_empty(0),
            x.new_empty(B, H, W, 3 * C) if store else x.new_empty(0), x.new_empty(kw, dtype=torch.int32),
            x.new_empty(nws, dtype=torch.float32))


def _attn_qkv_setup(ctx, inputs, output):
    x, weight, bias, table, proj_weight, proj_bias, num_heads, shift, p_drop, seed, seed_dev, store = inputs
    _, o, qkv, keep, ws = output
    ctx.mark_non_differentiable(o, qkv, keep, ws)
    ctx.aux_ws = ws
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(x.contiguous(), o, qkv, bias, table, seed_dev, keep)
    ctx.params = (weight, bias, proj_weight, proj_bias)
    ctx.bias_param = bias if isinstance(bias, torch.nn.Parameter) else None
    ctx.table_param = table if isinstance(table, torch.nn.Parameter) else None
    ctx.cfg = (num_heads, shift, float(p_drop), seed)


def _attn_qkv_backward(ctx, dy, _do, _dqkv, _dkeep, _dws=None):
    x, o, qkv, bias, table, seed_dev, keep = ctx.saved_tensors
    if dy is None:
        return (None,) * 12
    if qkv.numel() == 0:
        raise RuntimeError("window_attention_qkv: backward through a forward that did not keep qkv (store=False)")
    weight, _, wp, bp = ctx.params
    dwp = dbp = None
    if wp is not None:
        # proj Linear first: do = dy . W_proj, dW_proj / db_proj from (dy, o)
        pctx = _Ctx((o,), params=(wp, bp), needs_input_grad=(True, ctx.needs_input_grad[4], ctx.needs_input_grad[5]))
        dout, dwp, dbp = _linear_grads(pctx, dy)
    else:
        dout = dy
    actx = _Ctx((qkv, bias, table, seed_dev, keep), cfg=ctx.cfg, bias_param=ctx.bias_param,
                table_param=ctx.table_param, aux_ws=ctx.aux_ws)
    dqkv, dbias_pad, dtable = _attn_backward(actx, dout, None)[:3]
    lctx = _Ctx((x,), params=(weight, bias),
                needs_input_grad=(ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]))
    dx, dw, db = _linear_grads(lctx, dqkv)
    if db is not None and dbias_pad is not None:
        db = db + dbias_pad
    elif dbias_pad is not None:
        db = dbias_pad
    return dx, dw, db, dtable, dwp, dbp, None, None, None, None, None, None


_window_attention_qkv = _define(
    "window_attention_qkv",
    "(Tensor x, Tensor weight, Tensor bias, Tensor table, Tensor? proj_weight, Tensor? proj_bias, int num_heads,"
    " int shift, float p_drop, int seed, Tensor? seed_dev, bool store) -> (Tensor, Tensor, Tensor, Tensor, Tensor)",
    _attn_qkv_impl, _attn_qkv_fake, _attn_qkv_setup, _attn_qkv_backward)


def window_attention_qkv_fusable(x, num_heads, bias):
    """Whether the fused stage-0 unit takes this block: 16-bit, C = 96 with 3 heads, a qkv bias."""
    if not _ATTN_QKV or bias is None or not x.is_cuda or act_dtype() not in _LOW:
        return False
    C = x.shape[-1]
    return bool(_lib.lib().msu_win_attn_qkv_supported(C, num_heads))


def window_attention_qkv(x, weight, bias, table, num_heads, shift, p_drop=0.0, seed=0, seed_dev=None,
                         proj_weight=None, proj_bias=None):
    """window_attention(linear(x, weight, bias), bias, table, ...) with the qkv Linear fused in
    (and the proj Linear, ``linear(., proj_weight, proj_bias)``, when given): x [B, H, W, C] (LN1
    output) -> [B, H, W, C]."""
    dt = act_dtype()
    x = _as(x, dt)
    proj = proj_weight is not None
    if proj and proj_bias is None:
        raise ValueError("the fused proj needs its bias")
    params = [weight, bias, table] + ([proj_weight, proj_bias] if proj else [])
    store = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
    # _f32 hands an f32 contiguous Parameter through as the same object (direct .grad in the
    # backward), and converts anything else: the kernel reads the biases and the table as f32
    return _window_attention_qkv(x, weight, _f32(bias), _f32(table),
                                 proj_weight if proj else None, _f32(proj_bias) if proj else None,
                                 int(num_heads), int(shift), float(p_drop), int(seed) & ((1 << 63) - 1), seed_dev,
                                 bool(store))[0]


# ----------------------------------------------------------------------------- token GEMM
TOK_PLAIN, TOK_GELU_DUAL, TOK_GELU_GRAD = 0, 1, 2
_tok_cache = {}


def tok_supported(M, N, K):
    """Whether the HIP token GEMM (csrc/gemm_tok.h) covers this 16-bit Linear shape."""
    key = (int(M), int(N), int(K))
    r = _tok_cache.get(key)
    if r is None:
        r = _tok_cache[key] = bool(_lib.lib().msu_tok_gemm_supported(*key))
    return r


def tok_supported_epi(M, N, K, epi):
    """``tok_supported`` for one epilogue (TOK_GELU_* plans cap the column chunk at 192)."""
    key = (int(M), int(N), int(K), int(epi))
    r = _tok_cache.get(key)
    if r is None:
        r = _tok_cache[key] = bool(_lib.lib().msu_tok_gemm_supported_epi(*key))
    return r




def tok_gemm(a, w, bias=None, epi=TOK_PLAIN, h=None, a2=None, gelu_only=False):
    """16-bit Y = epi(A . W^T + bias) on the token GEMM kernel.  a: [..., K1] (+ a2: [..., K-K1]),
    w: [N, K] (a's dtype), bias: [N] f32.  Returns Y (and GELU(Y) for TOK_GELU_DUAL).
    gelu_only (TOK_GELU_DUAL): one buffer for both outputs -- the kernel's GELU store follows
    its pre-activation store to the same address, so the returned pair is (GELU(Y), GELU(Y))
    and the L2 merges the two writes of each line (no-grad MLPs: nobody needs Y)."""
    N, K = w.shape
    K1 = a.shape[-1]
    M = a.numel() // K1
    a = a.contiguous()
    y = torch.empty(*a.shape[:-1], N, device=a.device, dtype=a.dtype)
    y2 = (y if gelu_only else torch.empty_like(y)) if epi == TOK_GELU_DUAL else None
    _lib.call("msu_tok_gemm", _dt(a), _p(a), _p(None if a2 is None else a2.contiguous()),
              K1 if a2 is not None else 0, _p(w), _p(bias), _p(y), _p(y2), _p(h), M, N, K, epi, _s(a))
    return (y, y2) if epi == TOK_GELU_DUAL else y


def nt_supported(M, N, K):
    """Whether the tiled NT GEMM (csrc/gemm_nt.hip) covers this 16-bit Linear shape."""
    key = ("nt", int(M), int(N), int(K))
    r = _tok_cache.get(key)
    if r is None:
        r = _tok_cache[key] = bool(_lib.lib().msu_nt_gemm_supported(*key[1:]))
    return r


def nt_gemm(a, w, bias=None, epi=TOK_PLAIN, h=None, gelu_only=False):
    """16-bit Y = epi(A . W^T + bias) on the tiled NT GEMM (tok_gemm's epilogues and gelu_only)."""
    N, K = w.shape
    M = a.numel() // K
    a = a.contiguous()
    y = torch.empty(*a.shape[:-1], N, device=a.device, dtype=a.dtype)
    y2 = (y if gelu_only else torch.empty_like(y)) if epi == TOK_GELU_DUAL else None
    _lib.call("msu_nt_gemm", _dt(a), _p(a), _p(w), _p(bias), _p(y), _p(y2), _p(h), M, N, K, epi, _s(a))
    return (y, y2) if epi == TOK_GELU_DUAL else y


def nt_gemm_kn(a, wk, epi=TOK_PLAIN, h=None):
    """16-bit Y = epi(A . Wk) on the tiled NT GEMM with Wk [K, N] read in place (no bias)."""
    K, N = wk.shape
    M = a.numel() // K
    a = a.contiguous()
    y = torch.empty(*a.shape[:-1], N, device=a.device, dtype=a.dtype)
    _lib.call("msu_nt_gemm_kn", _dt(a), _p(a), _p(wk), None, _p(y), None, _p(h), M, N, K, epi, _s(a))
    return y


def _wt(w):
    """[N, K] 16-bit weight -> contiguous W^T [K, N] for the input-gradient GEMM."""
    return w.t().contiguous()


def _gemm_dx(dy, w, epi=TOK_PLAIN, h=None, param=None):
    """16-bit epi(dy . w): the input gradient of y = x . w^T (w [N, K]) on the routed GEMM.  W^T
    comes from the trainer's transposed shadow of ``param`` when it has one (both GEMMs then run
    their forward layout); otherwise the NT route reads w in place (KN variant) and the token
    GEMM takes a per-call W^T copy."""
    N, K = w.shape
    M = dy.numel() // N
    wt = _shadow_t(param, w.dtype)
    if gemm_route(M, K, N, epi) == "nt" and wt is None:
        return nt_gemm_kn(dy, w, epi, h)
    return _gemm(dy, _wt(w) if wt is None else wt, None, epi, h)


def _gelu16(h):
    """GELU(h) in h's 16-bit format on the current stream (msu_gelu_fwd: the fused epilogues'
    arithmetic and rounding)."""
    g = torch.empty_like(h)
    _lib.call("msu_gelu_fwd", _dt(h), _p(h), _p(g), h.numel(), _s(h))
    return g


def _wgrad(dy, x, weight, bias, M, N, K, x_gelu_of=None, side_ok=True):
    """Linear weight/bias gradients on msu_linear_wgrad; (None, None) when accumulated
    straight into the trainer's flat .grad views.  x None: x = GELU(x_gelu_of), derived on the
    stream the weight gradient runs on.  side_ok False: on the main stream even with direct
    parameters (a Linear whose input needs no gradient -- PatchEmbed's, the last node of backward:
    nothing is left on the main stream to overlap it, and behind the side stream's queue it would
    only delay the end-of-backward join)."""
    L = _lib.lib()
    if _direct(weight) and (bias is None or _direct(bias)):
        if _side_enabled and _side_wgrad and side_ok:
            src = x if x is not None else x_gelu_of
            main = torch.cuda.current_stream(src.device)
            side = _side_stream_for(src.device)
            side.wait_stream(main)  # dy and x are ready
            with torch.cuda.stream(side):
                if x is None:
                    x = _gelu16(x_gelu_of)  # allocated on the side stream, used there only
                ws = torch.empty(L.msu_wgrad_workspace(M, N, K), device=x.device, dtype=torch.float32)
                _lib.call("msu_linear_wgrad", _dt(x), _p(dy), _p(x), _p(weight.grad),
                          _p(None if bias is None else bias.grad), _p(ws), M, N, K, 1, side.cuda_stream)
            dy.record_stream(side)  # their memory is not reused by the main stream meanwhile
            src.record_stream(side)
            _side_keep.append(dy)  # ... nor accumulated into in place (see _side_keep)
            _side_keep.append(src)
            ev = torch.cuda.Event()
            ev.record(side)
            _guard_side_write(weight, ev)
            if bias is not None:
                _guard_side_write(bias, ev)
            _join_at_end_of_backward()
        else:
            if x is None:
                x = _gelu16(x_gelu_of)
            ws = torch.empty(L.msu_wgrad_workspace(M, N, K), device=x.device, dtype=torch.float32)
            _lib.call("msu_linear_wgrad", _dt(x), _p(dy), _p(x), _p(weight.grad),
                      _p(None if bias is None else bias.grad), _p(ws), M, N, K, 1, _s(x))
        _notify(weight, bias)
        return None, None
    if x is None:
        x = _gelu16(x_gelu_of)
    ws = torch.empty(L.msu_wgrad_workspace(M, N, K), device=x.device, dtype=torch.float32)
    dw = torch.empty(N, K, device=x.device, dtype=torch.float32)
    db = torch.empty(N, device=x.device, dtype=torch.float32) if bias is not None else None
    _lib.call("msu_linear_wgrad", _dt(x), _p(dy), _p(x), _p(dw), _p(db), _p(ws), M, N, K, 0, _s(x))
    return dw, db


def _shadow(param, dt):
    """16-bit copy of an f32 master parameter: the trainer's per-step shadow buffer when it
    keeps one (``_msu_shadow``, the trainer's compute dtype), else a cast."""
    sh = getattr(param, "_msu_shadow", None)
    if sh is not None and sh.dtype == dt and getattr(param, "_msu_shadow_ver", -1) == param._version:
        return sh
    return param.to(dt)


# the trainer's transposed weight shadow for the input-gradient GEMMs (r03i: +2.1 %); False (the
# tests' second arm): W^T read in place by the NT GEMM's KN variant / copied per call for the
# token GEMM, as under fp16 autocast over the bf16 shadow
_SHADOW_T = True


def _shadow_t(param, dt):
    """The trainer's transposed 16-bit shadow W^T [K, N] of a Linear weight W [N, K], refreshed
    with the shadow (None when there is none or it is stale)."""
    if param is None or not _SHADOW_T:
        return None
    sh = getattr(param, "_msu_shadow_t", None)
    if sh is not None and sh.dtype == dt and getattr(param, "_msu_shadow_ver", -1) == param._version:
        return sh
    return None


def transpose16_multi(src, dst, table, ntiles):
    """dst segments = transposes of src segments (table rows {src off, dst off, N, K, first tile})."""
    _lib.call("msu_transpose16_multi", _p(src), _p(dst), _p(table), int(table.shape[0]), int(ntiles), _s(src))


# GEMM routing of the 16-bit Linears (forward and input gradient): the token GEMM (weight in
# LDS, tokens streamed) for the HBM-bound stage-0 shapes and the narrow-K stage-1 shapes, the
# persistent tiled NT GEMM (csrc/gemm_nt.hip) for the wide-weight stage 1-3 shapes -- every
# Linear of the step runs on a hand-written kernel.  A/B switches (MSU_GEMM_ROUTE): "lib" =
# the library GEMM (hipBLASLt) wherever the epilogue allows it, "ntmlp" = the NT GEMM only for
# the GELU-epilogue MLP GEMMs (library elsewhere), "nt" = the NT GEMM before the narrow-K token
# GEMM plans.
_ROUTE_FORCE = switches.get("MSU_GEMM_ROUTE")


def gemm_route(M, N, K, epi=TOK_PLAIN):
    """'tok' | 'nt' | 'lib' for a 16-bit Y = epi(A[M,K] . W[N,K]^T + b) (input gradients: W^T)."""
    key = ("route", int(M), int(N), int(K), int(epi))
    r = _tok_cache.get(key)
    if r is None:
        tok = tok_supported_epi(M, N, K, epi)
        if _ROUTE_FORCE == "lib" and epi == TOK_PLAIN:
            r = "lib"
        elif tok and (M >= 262144 or (epi == TOK_PLAIN and N * K <= 576 * 192 and N >= 3 * K)):
            r = "tok"
        elif _ROUTE_FORCE == "nt" and nt_supported(M, N, K):
            r = "nt"
        elif tok and (N * K <= 576 * 192 or (epi != TOK_PLAIN and M >= 131072)):
            r = "tok"
        elif _ROUTE_FORCE in ("", "ntlib") and nt_supported(M, N, K):
            r = "nt"
        elif _ROUTE_FORCE == "ntmlp" and epi != TOK_PLAIN and nt_supported(M, N, K):
            r = "nt"
        else:
            r = "lib"
        _tok_cache[key] = r
    return r


def _gemm(a, w, bias=None, epi=TOK_PLAIN, h=None, gelu_only=False):
    """16-bit epi(a . w^T + bias) on the routed GEMM (bias: f32 [N] or None)."""
    N, K = w.shape
    M = a.numel() // K
    r = gemm_route(M, N, K, epi)
    if r == "tok":
        return tok_gemm(a, w, bias, epi, h, gelu_only=gelu_only)
    if r == "nt":
        return nt_gemm(a, w, bias, epi, h, gelu_only=gelu_only)
    if epi != TOK_PLAIN:
        raise RuntimeError(f"no HIP GEMM covers the epilogue {epi} at M={M} N={N} K={K}")
    with torch.autocast("cuda", enabled=False):
        return torch.nn.functional.linear(a, w, None if bias is None else bias.to(a.dtype))


def _mm(a, w, bias=None):
    """16-bit a . w^T (+ bias) on the routed GEMM."""
    return _gemm(a, w, bias)


# ----------------------------------------------------------------------------- Linear
def _linear_impl(x, weight, bias, handoff=0):
    """Y = x . W^T + b in x's dtype; the f32 master weight / bias are cast inside the op so
    that the parameter gradients are the f32 ones of the weight-gradient kernel."""
    _need_cuda(x)
    dt = x.dtype
    w = _shadow(weight, dt)
    N, K = w.shape
    M = x.numel() // K
    if dt in _LOW and gemm_route(M, N, K) != "lib":
        return _gemm(x, w, None if bias is None else _f32(bias))
    b = None if bias is None else _shadow(bias, dt)
    with torch.autocast("cuda", enabled=False):
        return torch.nn.functional.linear(x, w, b)


def _linear_fake(x, weight, bias, handoff=0):
    return x.new_empty(*x.shape[:-1], weight.shape[0])


def _linear_setup(ctx, inputs, output):
    x, weight, bias = inputs[:3]
    ctx.save_for_backward(x)
    ctx.params = (weight, bias)
    ctx.handoff = inputs[3] if len(inputs) > 3 else 0


# One-pass Linear backward (csrc/gemm_linbwd.hip) for the stage-0 block Linears: dX, dW and db
# from one read of dY on the main stream, instead of the input-gradient GEMM plus a side-stream
# weight gradient that reads dY again.  A/B switch MSU_LINBWD=0: the two-kernel path.
_LINBWD = switches.on("MSU_LINBWD")
_LINBWD_MIN_M = 65536


linbwd_calls = 0  # one-pass backward launches (tests assert which path a backward took)


def _linbwd(dy, x, weight, bias, M, N, K, h=None, gelu_x=False):
    """dX = dy . W (* GELU'(h)) with dW / db accumulated into the trainer's .grad in the same
    pass; None when the shape, dtype or parameters are not covered (caller: two-kernel path).
    W^T is the trainer's transposed shadow when it has one in x's dtype, else a per-call
    transpose of the 16-bit weight (fp16 autocast over a bf16 shadow, or _SHADOW_T off)."""
    global linbwd_calls
    if not _LINBWD or x.dtype not in _LOW or M < _LINBWD_MIN_M:
        return None
    if not _direct(weight) or (bias is not None and not _direct(bias)):
        return None
    L = _lib.lib()
    if not L.msu_linear_bwd_supported(M, K, N):
        return None
    wt = _shadow_t(weight, x.dtype)
    if wt is None:
        wt = _wt(_shadow(weight, x.dtype))
    if bias is not None:
        # the qkv bias also receives the attention's padded-token share on the side stream
        # (msu_win_attn_bwd_tail, issued earlier in this backward): add after it
        ev = getattr(bias, "_msu_side_event", None)
        if ev is not None:
            torch.cuda.current_stream(x.device).wait_event(ev)
    dx = torch.empty(*dy.shape[:-1], K, device=dy.device, dtype=dy.dtype)
    ws = torch.empty(L.msu_linear_bwd_workspace(M, K, N), device=x.device, dtype=torch.float32)
    # gelu_x: x is H and the kernel stages GELU(H) as the input (msu_linear_bwd with X = null)
    _lib.call("msu_linear_bwd", _dt(x), _p(dy), _p(None if gelu_x else x.contiguous()), _p(wt), _p(h), _p(dx),
              _p(weight.grad),
              _p(None if bias is None else bias.grad), _p(ws), M, K, N, 1, _s(x))
    linbwd_calls += 1
    _notify(weight, bias)
    return dx


def _linear_grads(ctx, dy):
    """(dx, dW, db) of a Linear; dx is None when it went to x's keyed LayerNorm (ctx.handoff,
    absent on the hand-made contexts of the fused units' backwards)."""
    (x,) = ctx.saved_tensors
    weight, bias = ctx.params
    key = getattr(ctx, "handoff", 0)
    w = _shadow(weight, x.dtype)
    dy = _as(dy, x.dtype)
    N, K = w.shape
    M = dy.numel() // N
    if ctx.needs_input_grad[0]:
        dx = _linbwd(dy.contiguous(), x, weight, bias, M, N, K)
        if dx is not None:
            return (None if _park(key, dx) else dx), None, None
    dx = None
    if ctx.needs_input_grad[0]:
        if x.dtype in _LOW and gemm_route(M, K, N) != "lib":
            dx = _gemm_dx(dy, w, param=weight)
        else:
            with torch.autocast("cuda", enabled=False):
                dx = dy.matmul(w)
    if dx is not None and _park(key, dx):
        dx = None  # x's gradient goes to its keyed LayerNorm's backward kernel
    if not (ctx.needs_input_grad[1] or (bias is not None and ctx.needs_input_grad[2])):
        return dx, None, None  # frozen weight and bias: no weight-gradient work at all
    dw, db = _wgrad(dy, x, weight, bias, M, N, K, side_ok=ctx.needs_input_grad[0])
    return dx, dw, db


def _linear_backward(ctx, dy):
    return (*_linear_grads(ctx, dy), None)


_linear = _define("linear", "(Tensor x, Tensor weight, Tensor? bias, int handoff=0) -> Tensor",
                  _linear_impl, _linear_fake, _linear_setup, _linear_backward)


def linear(x, weight, bias=None, handoff=0):
    """nn.functional.linear with the HIP weight-gradient kernel (activation dtype per autocast);
    16-bit forward / input-gradient GEMMs on the token GEMM where it covers the shape.
    handoff: a ``residual_handoff_key()`` of x (its gradient is added in the keyed LayerNorm's
    backward kernel)."""
    _need_cuda(x)
    dt = act_dtype()
    x = _as(x, dt)
    N, K = weight.shape
    if K % 8 or N % 8:
        return torch.nn.functional.linear(x, weight.to(dt), None if bias is None else bias.to(dt))
    return _linear(x, weight, bias, int(handoff))


# ----------------------------------------------------------------------------- skip fusion
def nt_gemm_cat(x, skip, w, bias):
    """16-bit Y = [x | skip] . W^T + bias on the NT GEMM (x's width a multiple of 64)."""
    N, K = w.shape
    K1 = x.shape[-1]
    M = x.numel() // K1
    x, skip = x.contiguous(), skip.contiguous()
    y = torch.empty(*x.shape[:-1], N, device=x.device, dtype=x.dtype)
    _lib.call("msu_nt_gemm_cat", _dt(x), _p(x), _p(skip), K1, _p(w), _p(bias), _p(y), M, N, K, _s(x))
    return y


def _cat_route(M, N, K, C1):
    """The GEMM that takes a skip fusion without the concatenated copy, or None."""
    r = gemm_route(M, N, K)
    if r == "tok" and C1 % 8 == 0:
        return "tok"
    if r == "nt" and C1 % 64 == 0:
        return "nt"
    return None


def _linear_cat_impl(x, skip, weight, bias, handoff=0):
    W = _shadow(weight, x.dtype)
    N, K = W.shape
    C1 = x.shape[-1]
    if _cat_route(x.numel() // C1, N, K, C1) == "nt":
        return nt_gemm_cat(x, skip, W, _f32(bias))
    return tok_gemm(x, W, _f32(bias), a2=skip)


def _linear_cat_fake(x, skip, weight, bias, handoff=0):
    return x.new_empty(*x.shape[:-1], weight.shape[0])


def _linear_cat_setup(ctx, inputs, output):
    x, skip, weight, bias = inputs[:4]
    ctx.save_for_backward(x, skip)
    ctx.params = (weight, bias)
    ctx.handoff = inputs[4] if len(inputs) > 4 else 0


def _wgrad_into(dy, x, dw, db, M, N, K, acc):
    """msu_linear_wgrad of one input half: dw [N, K] may be a column slice of a wider [N, Kt]
    gradient (row stride Kt, the kernel's ldw); acc = 1 adds into it."""
    L = _lib.lib()
    ws = torch.empty(L.msu_wgrad_workspace(M, N, K), device=x.device, dtype=torch.float32)
    _lib.call("msu_linear_wgrad_ld", _dt(x), _p(dy), _p(x), _p(dw), dw.stride(0), _p(db), _p(ws), M, N, K, acc,
              _s(x))




def _linear_cat_backward(ctx, dy):
    x, skip = ctx.saved_tensors
    weight, bias = ctx.params
    W = _shadow(weight, x.dtype)
    dy = _as(dy, x.dtype)
    N = W.shape[0]
    C1, C2 = x.shape[-1], skip.shape[-1]
    M = dy.numel() // N
    outs = []
    wt = _shadow_t(weight, W.dtype)  # W^T [K, N]: the halves are row ranges, no copies
    for lo, hi in ((0, C1), (C1, C1 + C2)):
        outs.append(_gemm(dy, W[:, lo:hi].t().contiguous() if wt is None else wt[lo:hi]))
    if _park(ctx.handoff, outs[1]):
        outs[1] = None  # the skip's gradient goes to its keyed LayerNorm's backward kernel
    # weight gradient per half straight into the column slices of dW (bias with the first):
    # the trainer's flat .grad (accumulate) or a fresh [N, C1 + C2] gradient
    direct = _direct(weight, bias)
    if direct and _side_enabled and _side_wgrad:
        # on the weight-gradient side stream like every other Linear's (the shared skip-fusion
        # Linears -- concat_back_dim[2 / 3] serve the central decoders too -- then have all
        # their .grad writers on one stream, in program order)
        main = torch.cuda.current_stream(x.device)
        side = _side_stream_for(x.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            _wgrad_into(dy, x, weight.grad[:, :C1], bias.grad, M, N, C1, 1)
            _wgrad_into(dy, skip, weight.grad[:, C1:], None, M, N, C2, 1)
        for t in (dy, x, skip):
            t.record_stream(side)
            _side_keep.append(t)
        ev = torch.cuda.Event()
        ev.record(side)
        _guard_side_write(weight, ev)
        _guard_side_write(bias, ev)
        _join_at_end_of_backward()
        _notify(weight, bias)
        return outs[0], outs[1], None, None, None
    if direct:
        dw, db, acc = weight.grad, bias.grad, 1
    else:
        dw = torch.empty(N, C1 + C2, device=x.device, dtype=torch.float32)
        db = torch.empty(N, device=x.device, dtype=torch.float32)
        acc = 0
    _wgrad_into(dy, x, dw[:, :C1], db, M, N, C1, acc)
    _wgrad_into(dy, skip, dw[:, C1:], None, M, N, C2, acc)
    if direct:
        _notify(weight, bias)
        return outs[0], outs[1], None, None, None
    return outs[0], outs[1], dw, db, None


_linear_cat = _define("linear_cat", "(Tensor x, Tensor skip, Tensor weight, Tensor bias, int handoff=0) -> Tensor",
                      _linear_cat_impl, _linear_cat_fake, _linear_cat_setup, _linear_cat_backward)


def linear_cat(x, skip, weight, bias, handoff=0):
    """``F.linear(torch.cat([x, skip], -1), weight, bias)`` (skip fusion, model_parts.py:792-794,
    :804-806, :823-824); x / skip: [..., C1] / [..., C2] with equal leading dims.  16-bit: the
    concatenation is folded into the A loads of the routed GEMM (token GEMM or NT GEMM: no
    concatenated copy) and split back out of the input gradient (two GEMMs over W's halves).
    handoff: the skip's ``residual_handoff_key()`` (its gradient is added in the keyed
    LayerNorm's backward kernel)."""
    _need_cuda(x)
    dt = act_dtype()
    x, skip = _as(x, dt), _as(skip, dt)
    N, K = weight.shape
    C1, C2 = x.shape[-1], skip.shape[-1]
    M = x.numel() // C1
    if dt in _LOW and bias is not None and C1 + C2 == K and _cat_route(M, N, K, C1) is not None:
        return _linear_cat(x, skip, weight, bias, int(handoff))
    return linear(torch.cat([x, skip], -1), weight, bias)


# ----------------------------------------------------------------------------- fused MLP
def mlp_fusable(x, fc1_weight, fc2_weight):
    """torchvision MLP (mlp.0 -> GELU -> mlp.3) fusable in 16-bit: the two GELU-epilogue GEMMs
    (mlp.0 forward, mlp.3 input gradient: both [M,C] x [C,Hd]) have a HIP GEMM (token GEMM
    or tiled NT GEMM), the other two run on whichever GEMM is routed for their shape."""
    if act_dtype() not in _LOW:
        return False
    Hd, C = fc1_weight.shape
    M = x.numel() // C
    if fc2_weight.shape != (C, Hd):
        return False
    return (gemm_route(M, Hd, C, TOK_GELU_DUAL) != "lib" and
            gemm_route(M, Hd, C, TOK_GELU_GRAD) != "lib")


# MSU_MLP_INFER=0 / MSU_MLP_TRAIN=0: the no-grad / training stage-0 MLPs on the token-GEMM pair
# (A/B switches)
_MLP_INFER = switches.on("MSU_MLP_INFER")
_MLP_TRAIN = switches.on("MSU_MLP_TRAIN")
mlp_infer_calls = 0  # fused MLP launches without H (tests assert which path a no-grad forward took)
mlp_train_calls = 0  # fused MLP launches storing H


# the (C, hidden) shapes the fused MLP kernels are built for: msu_mlp_fused_supported restated
# (stage 0: csrc/mlp_fused.hip, weights resident in LDS; stage 1: csrc/mlp_s1.hip, weights streamed
# through an LDS ring; tests/test_capi.py checks the two agree), so fake kernels need no library
MLP_KERNEL_SHAPES = ((96, 384), (192, 768))
# MSU_MLP_S1=0: the stage-1 MLPs on the GEMM pair (A/B switch)
_MLP_S1 = switches.on("MSU_MLP_S1")
MLP_FUSED_SHAPES = MLP_KERNEL_SHAPES if _MLP_S1 else MLP_KERNEL_SHAPES[:1]


def _mlp_fused_ok(C, Hd):
    return (int(C), int(Hd)) in MLP_FUSED_SHAPES


def _mlp_impl(x, w1, b1, w2, b2, keep):
    """y = mlp.3(GELU(mlp.0(x))) (torchvision ops.misc.MLP without dropout): mlp.0's epilogue
    stores H and GELU(H) (returned for backward); mlp.3's input gradient applies GELU'(H) in
    its epilogue.  keep = False (no backward will run: the reference's discarded branches,
    inference): H is not kept -- the GELU store overwrites it in one buffer -- and H / G come
    back empty."""
    global mlp_infer_calls, mlp_train_calls
    _need_cuda(x)
    W1 = _shadow(w1, x.dtype)
    W2 = _shadow(w2, x.dtype)
    Hd, C = W1.shape
    fused = _mlp_fused_route(x, w1, keep)
    if fused:
        # one kernel, the hidden activation on chip (csrc/mlp_fused.hip); training keeps H only
        # (the backward re-derives GELU(H)).  Operands 16-B aligned (weight shadows are views
        # into one flat buffer).
        x = x.contiguous()
        B1, B2 = _f32(b1), _f32(b2)
        if all(t.data_ptr() % 16 == 0 for t in (x, W1, W2, B1, B2)) and W1.is_contiguous() and W2.is_contiguous():
            y = torch.empty(*x.shape[:-1], C, device=x.device, dtype=x.dtype)
            h = torch.empty(*x.shape[:-1], Hd, device=x.device, dtype=x.dtype) if keep else None
            if keep:
                mlp_train_calls += 1
            else:
                mlp_infer_calls += 1
            _lib.call("msu_mlp_fused_fwd", _dt(x), _p(x), _p(W1), _p(B1), _p(W2), _p(B2), _p(y), _p(h),
                      x.numel() // C, C, Hd, _s(x))
            return y, (h if keep else x.new_empty(0)), x.new_empty(0)
    h, g = _gemm(x, W1, _f32(b1), TOK_GELU_DUAL, gelu_only=not keep)
    y = _gemm(g, W2, _f32(b2))
    if not keep:
        return y, x.new_empty(0), x.new_empty(0)
    # the fused route's output contract (G empty: the backward re-derives it) also when an
    # unaligned operand sent the call to the GEMM pair -- the fake kernel can't see alignment
    return y, h, (x.new_empty(0) if fused else g)


def _mlp_fused_route(x, w1, keep):
    """Whether an mlp call takes the fused kernel's output contract: H kept, G empty (training)."""
    Hd, C = w1.shape
    return bool((_MLP_TRAIN if keep else _MLP_INFER) and x.dtype in _LOW and _mlp_fused_ok(C, Hd))


def _mlp_fake(x, w1, b1, w2, b2, keep):
    hid = x.new_empty(*x.shape[:-1], w1.shape[0]) if keep else x.new_empty(0)
    g = x.new_empty(0) if (not keep or _mlp_fused_route(x, w1, keep)) else torch.empty_like(hid)
    return x.new_empty(*x.shape[:-1], w2.shape[0]), hid, g


def _mlp_setup(ctx, inputs, output):
    x, w1, b1, w2, b2, keep = inputs
    y, h, g = output
    ctx.save_for_backward(x, h, g)
    ctx.params = (w1, b1, w2, b2)
    ctx.mark_non_differentiable(h, g)
    ctx.set_materialize_grads(False)


def _mlp_backward(ctx, dy, _dh, _dg):
    x, h, g = ctx.saved_tensors
    if dy is None:
        return None, None, None, None, None, None
    if h.numel() == 0:
        raise RuntimeError("mlp: backward through a forward that did not keep its activations (keep=False)")
    w1, b1, w2, b2 = ctx.params
    W1 = _shadow(w1, x.dtype)
    W2 = _shadow(w2, x.dtype)
    dy = _as(dy, x.dtype)
    Hd, C = W1.shape
    M = x.numel() // C
    dy = dy.contiguous()
    if g.numel() == 0:  # fused forward: H only; mlp.3's pass re-derives GELU(H) while staging
        dh = _linbwd(dy, h, w2, b2, M, C, Hd, h=h, gelu_x=True)
    else:
        dh = _linbwd(dy, g, w2, b2, M, C, Hd, h=h)  # mlp.3 in one pass (dh through GELU')
    if dh is None:
        # two kernels: the weight gradient reads GELU(H) -- after a fused forward it is derived
        # from H (in H's 16-bit format) where that weight gradient runs, the side stream
        dw2, db2 = _wgrad(dy, g if g.numel() else None, w2, b2, M, C, Hd, x_gelu_of=h)
        dh = _gemm_dx(dy, W2, TOK_GELU_GRAD, h=h, param=w2)
    else:
        dw2 = db2 = None
    dx = _linbwd(dh, x, w1, b1, M, Hd, C) if ctx.needs_input_grad[0] else None  # mlp.0 in one pass
    if dx is None:
        dw1, db1 = _wgrad(dh, x, w1, b1, M, Hd, C)
        dx = _gemm_dx(dh, W1, param=w1) if ctx.needs_input_grad[0] else None
    else:
        dw1 = db1 = None
    return dx, dw1, db1, dw2, db2, None


_mlp = _define("mlp", "(Tensor x, Tensor w1, Tensor b1, Tensor w2, Tensor b2, bool keep) -> (Tensor, Tensor, Tensor)",
               _mlp_impl, _mlp_fake, _mlp_setup, _mlp_backward)


_MLP_LN = switches.on("MSU_MLP_LN")
add_ln_mlp_calls = 0


def add_layer_norm_mlp(a, branch, scale, ln_weight, ln_bias, eps, fc1_weight, fc1_bias, fc2_weight, fc2_bias):
    """No-grad (s, mlp(LN(s))) with s = a + scale[sample] * branch in one kernel
    (csrc/mlp_fused.hip), or None when not covered (autograd on, widths, dtype, alignment)."""
    global add_ln_mlp_calls
    dt = act_dtype()
    if torch.is_grad_enabled() or not (_MLP_LN and _MLP_INFER) or dt not in _LOW or not a.is_cuda:
        return None
    C = a.shape[-1]
    Hd = fc1_weight.shape[0]
    if fc1_bias is None or fc2_bias is None or (C, Hd) != MLP_FUSED_SHAPES[0] or fc2_weight.shape != (C, Hd):
        return None
    a, branch = _as(a, dt), _as(branch, dt)
    W1, W2 = _shadow(fc1_weight, dt), _shadow(fc2_weight, dt)
    B1, B2, G, Bt = _f32(fc1_bias), _f32(fc2_bias), _f32(ln_weight), _f32(ln_bias)
    sc = None if scale is None else _f32(scale)
    ts = [a, branch, W1, W2, B1, B2, G, Bt]
    if not all(t.data_ptr() % 16 == 0 for t in ts) or not (W1.is_contiguous() and W2.is_contiguous()):
        return None
    rows = a.numel() // C
    s = torch.empty_like(a)
    y = torch.empty_like(a)
    add_ln_mlp_calls += 1
    _lib.call("msu_add_ln_mlp_fwd", _dt(a), _p(a), _p(branch), _p(sc), rows // a.shape[0], _p(G), _p(Bt),
              float(eps), _p(W1), _p(B1), _p(W2), _p(B2), _p(s), _p(y), rows, C, Hd, _s(a))
    return s, y


def mlp(x, fc1_weight, fc1_bias, fc2_weight, fc2_bias):
    """Fused torchvision MLP forward/backward (16-bit; see ``mlp_fusable``)."""
    _need_cuda(x)
    keep = torch.is_grad_enabled() and any(t.requires_grad for t in (x, fc1_weight, fc1_bias, fc2_weight, fc2_bias))
    return _mlp(_as(x, act_dtype()), fc1_weight, fc1_bias, fc2_weight, fc2_bias, bool(keep))[0]


# ----------------------------------------------------------------------------- residual
def _residual_impl(x, br, scale):
    """x + br * scale[sample] in one pass (StochasticDepth 'row' scale)."""
    _need_cuda(x, br)
    x, br = x.contiguous(), br.contiguous()
    out = torch.empty_like(x)
    _lib.call("msu_residual", _dt(x), _p(x), _p(br), _p(scale), _p(out), x.numel(), x[0].numel(), _s(x))
    return out


def _residual_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[2])


def _residual_backward(ctx, dy):
    """dx = dy, dbr = dy * scale[sample]."""
    (scale,) = ctx.saved_tensors
    dy = dy.contiguous()
    dbr = torch.empty_like(dy)
    _lib.call("msu_residual", _dt(dy), None, _p(dy), _p(scale), _p(dbr), dy.numel(), dy[0].numel(), _s(dy))
    return dy, dbr, None


_residual = _define("residual", "(Tensor x, Tensor br, Tensor scale) -> Tensor",
                    _residual_impl, lambda x, br, scale: torch.empty_like(x), _residual_setup, _residual_backward)


def residual_add(x, br, scale):
    """``x + br * scale.view(B, 1, ...)`` (per-sample scale; plain add when scale is None)."""
    dt = act_dtype()
    if scale is None:
        return x + br.to(x.dtype)
    return _residual(_as(x, dt), _as(br, dt), _f32(scale))


# ----------------------------------------------------------------------------- GELU
def _gelu_impl(x):
    _need_cuda(x)
    x = x.contiguous()
    y = torch.empty_like(x)
    _lib.call("msu_gelu_fwd", _dt(x), _p(x), _p(y), x.numel(), _s(x))
    return y


def _gelu_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0].contiguous())


def _gelu_backward(ctx, dy):
    (x,) = ctx.saved_tensors
    dy = _as(dy, x.dtype)
    dx = torch.empty_like(x)
    _lib.call("msu_gelu_bwd", _dt(x), _p(x), _p(dy), _p(dx), x.numel(), _s(x))
    return dx


_gelu = _define("gelu", "(Tensor x) -> Tensor", _gelu_impl, lambda x: torch.empty_like(x), _gelu_setup,
                _gelu_backward)


def gelu(x):
    """Exact (erf) GELU, nn.GELU()."""
    return _gelu(_as(x, act_dtype()))


# ----------------------------------------------------------------------------- head
def _head_impl(z, gamma, beta, w, eps):
    _need_cuda(z)
    z = z.contiguous()
    B, H, W, C = z.shape
    rows = B * H * W
    logit = torch.empty(B, 1, H, W, device=z.device, dtype=torch.float32)
    mean, rstd = _stats(z, rows)
    _lib.call("msu_head_fwd", _dt(z), _p(z), _p(gamma), _p(beta), _p(w), _p(logit), _p(mean),
              _p(rstd), rows, C, eps, _s(z))
    return logit, mean, rstd


def _head_fake(z, gamma, beta, w, eps):
    B, H, W, C = z.shape
    rows = B * H * W
    return (z.new_empty(B, 1, H, W, dtype=torch.float32), z.new_empty(rows, dtype=torch.float32),
            z.new_empty(rows, dtype=torch.float32))


def _head_setup(ctx, inputs, output):
    z, gamma, beta, w, eps = inputs
    ctx.save_for_backward(z.contiguous(), gamma, beta, w, output[1], output[2])
    ctx.params = (gamma, beta, w)
    ctx.set_materialize_grads(False)


def _head_backward(ctx, dlogit, _dm, _dr):
    z, gamma, beta, w, mean, rstd = ctx.saved_tensors
    if dlogit is None:
        return None, None, None, None, None
    B, H, W, C = z.shape
    rows = B * H * W
    dlogit = _f32(dlogit)
    dz = torch.empty_like(z)
    # trainer-direct gamma / beta / output weight: summed straight into their .grad
    direct = _direct(*ctx.params)
    if direct:
        dg, db, dw = (p.grad for p in ctx.params)
    else:
        dg, db, dw = torch.empty(3, C, device=z.device, dtype=torch.float32)  # contiguous: one reduction
    n, part = _ln_parts(rows, C, z.device)
    _lib.call("msu_head_bwd2", _dt(z), _p(dlogit), _p(z), _p(gamma), _p(beta), _p(w), _p(mean),
              _p(rstd), _p(dz), _p(part), n, _p(dg), _p(db), _p(dw), rows, C, int(direct), _s(z))
    if direct:
        _notify(*ctx.params)
        return dz, None, None, None, None
    return dz, dg, db, dw.view(w.shape), None


_head = _define("head_norm_output",
                "(Tensor z, Tensor gamma, Tensor beta, Tensor w, float eps) -> (Tensor, Tensor, Tensor)",
                _head_impl, _head_fake, _head_setup, _head_backward)


def head_norm_output(z, gamma, beta, out_weight, eps=1e-5):
    """FinalPatchExpand_X4_V2.norm + bias-free 1x1 output conv (num_classes == 1).
    z: [B, H, W, C] -> f32 logits [B, 1, H, W]."""
    if out_weight.shape[0] != 1:
        raise ValueError("fused head supports num_classes == 1")
    # the [1, C, 1, 1] conv weight itself (contiguous: the kernel reads C floats), so a trainer-
    # direct parameter's .grad is reachable from the backward
    w = _f32(out_weight).contiguous()
    return _head(_as(z, act_dtype()), _f32(gamma), _f32(beta), w, float(eps))[0]


# ----------------------------------------------------------------------------- conv 3x3
# persistent workgroups of the refine-conv weight gradient (one 139 KB / 12-wave workgroup per
# CU; 192 / 128 measured slower beside the refine dgrads, r04ac; fewer of them held back to the
# stage-2 LayerNorm backward, neutral / slower: r06k, r06t, removed)
_CONV_WGRAD_BLOCKS = int(switches.get("MSU_CONV_WGRAD_BLOCKS"))


def _conv_wgrad(a, dz, mode, B, H, W, Cin, Cout, into=None):
    """(dW, db) of the refine conv; ``into`` = (weight, bias): added to their .grad instead."""
    L = _lib.lib()
    nchunk = _CONV_WGRAD_BLOCKS
    ws = torch.empty(L.msu_conv3x3_wgrad_workspace(nchunk, Cin, Cout, 0, 0), device=a.device, dtype=torch.float32)
    if into is None:
        dw = torch.empty(Cout, Cin, 3, 3, device=a.device, dtype=torch.float32)
        db = torch.empty(Cout, device=a.device, dtype=torch.float32)
    else:
        dw, db = into[0].grad, into[1].grad
    _lib.call("msu_conv3x3_wgrad2", _dt(a), mode, _p(a), _p(dz), _p(dw), _p(db), _p(ws), nchunk,
              B, H, W, Cin, Cout, 0 if into is None else 1, _s(a))
    return dw, db


# A/B switch MSU_CONV_SIDE=0: the refine convs' weight gradients on the main stream.  (Holding
# them back to the next side-stream fork measured equal, r04z: gone.)
_CONV_SIDE = switches.on("MSU_CONV_SIDE")


def _conv_wgrad_param(a, dz, mode, B, H, W, Cin, Cout, weight, bias):
    """The refine conv's (dW, db) as autograd gradients, or (None, None) when they went straight
    into the trainer's .grad on the weight-gradient side stream (nothing in backward reads
    them: off the activation-gradient chain, 2 x 1.3 ms per step on the main stream before)."""
    if not (_CONV_SIDE and _side_enabled and _direct(weight, bias)):
        return _conv_wgrad(a, dz, mode, B, H, W, Cin, Cout)
    main = torch.cuda.current_stream(a.device)
    side = _side_stream_for(a.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        _conv_wgrad(a, dz, mode, B, H, W, Cin, Cout, into=(weight, bias))
    for t in (a, dz):
        t.record_stream(side)
        _side_keep.append(t)
    ev = torch.cuda.Event()
    ev.record(side)
    _guard_side_write(weight, ev)
    _guard_side_write(bias, ev)
    _notify(weight, bias)
    _join_at_end_of_backward()
    return None, None


def _conv_weight(weight, dt, flip):
    """The refine conv's weight in the conv kernels' layout (msu_conv3x3_weight; one launch in
    place of the flip / permute / pad / cast chain of ATen kernels): flip 0 -> [9][Cout][Cin32],
    flip 1 -> [9][Cin][Cout32]."""
    Cout, Cin = weight.shape[0], weight.shape[1]
    P = ((Cout if flip else Cin) + 31) // 32 * 32
    out = torch.empty(9, Cin if flip else Cout, P, device=weight.device, dtype=dt)
    w = weight.contiguous()
    _lib.call("msu_conv3x3_weight", _dt(out), _p(w), _p(out), Cout, Cin, int(flip), _s(w))
    return out


def _refine_impl(x, weight, bias, d2s, H, W):
    """z = conv3x3(GELU(map(x)), W) + b, NHWC; map = identity or the 4x4 depth-to-space of
    FinalPatchExpand_X4_V2 (x: [B, H/4, W/4, 16*Cin])."""
    _need_cuda(x)
    x = x.contiguous()
    Cout, Cin = weight.shape[0], weight.shape[1]
    B = x.shape[0]
    dt = x.dtype
    wt = _conv_weight(weight, dt, 0)
    z = torch.empty(B, H, W, Cout, device=x.device, dtype=dt)
    _lib.call("msu_conv3x3_fwd", _dt(x), 1 | (2 if d2s else 0), _p(x), _p(wt), _p(bias), _p(z),
              B, H, W, Cin, Cout, _s(x))
    return z


def _refine_setup(ctx, inputs, output):
    x, weight, bias, d2s, H, W = inputs
    ctx.save_for_backward(x.contiguous(), weight)
    ctx.params = (weight, bias)
    ctx.cfg = (d2s, H, W)


def _refine_backward(ctx, dz):
    x, weight = ctx.saved_tensors
    d2s, H, W = ctx.cfg
    Cout, Cin = weight.shape[0], weight.shape[1]
    B = x.shape[0]
    dz = _as(dz, x.dtype)
    mode = 1 | (2 if d2s else 0)
    dx = None
    if ctx.needs_input_grad[0]:
        wf = _conv_weight(weight, x.dtype, 1)
        dx = torch.empty_like(x)
        _lib.call("msu_conv3x3_dgrad", _dt(x), mode, _p(dz), _p(wf), _p(x), _p(dx), B, H, W, Cin, Cout, _s(x))
    dw, db = _conv_wgrad_param(x, dz, mode, B, H, W, Cin, Cout, *ctx.params)
    return dx, dw, db, None, None, None


_refine_conv = _define(
    "refine_conv", "(Tensor x, Tensor weight, Tensor bias, bool d2s, int H, int W) -> Tensor",
    _refine_impl, lambda x, weight, bias, d2s, H, W: x.new_empty(x.shape[0], H, W, weight.shape[0]),
    _refine_setup, _refine_backward)


def refine_conv(x, weight, bias, d2s, out_hw):
    H, W = out_hw
    return _refine_conv(_as(x, act_dtype()), _f32(weight), _f32(bias), bool(d2s), int(H), int(W))


def _refine_act_impl(x, a, weight, bias, d2s, H, W, dual):
    """z = conv3x3(a, W) + b with a = GELU(map(x)) already materialised by the producer (x: the
    differentiable pre-activation, a: its activation, non-differentiable).  The conv loads a as
    is; the input gradient applies GELU'(x) in the dgrad epilogue, the weight gradient reads
    a.  dual: the second output is GELU(z) from the same epilogue (the next refine conv's
    input); otherwise an empty placeholder."""
    _need_cuda(x, a)
    a = a.contiguous()
    Cout, Cin = weight.shape[0], weight.shape[1]
    B = a.shape[0]
    dt = a.dtype
    wt = _conv_weight(weight, dt, 0)
    z = torch.empty(B, H, W, Cout, device=a.device, dtype=dt)
    z2 = torch.empty_like(z) if dual else z.new_empty(0)
    _lib.call("msu_conv3x3_fwd2", _dt(a), 2 if d2s else 0, _p(a), _p(wt), _p(bias), _p(z), _p(z2) if dual else None,
              B, H, W, Cin, Cout, _s(a))
    return z, z2


def _refine_act_fake(x, a, weight, bias, d2s, H, W, dual):
    z = a.new_empty(a.shape[0], H, W, weight.shape[0])
    return z, (torch.empty_like(z) if dual else z.new_empty(0))


def _refine_act_setup(ctx, inputs, output):
    x, a, weight, bias, d2s, H, W, dual = inputs
    ctx.save_for_backward(x, a.contiguous(), weight)
    ctx.params = (weight, bias)
    ctx.cfg = (d2s, H, W)
    ctx.mark_non_differentiable(output[1])
    ctx.set_materialize_grads(False)  # no zero-filled gradient for GELU(z)


def _refine_act_backward(ctx, dz, _dz2):
    x, a, weight = ctx.saved_tensors
    d2s, H, W = ctx.cfg
    if dz is None:
        return (None,) * 8
    Cout, Cin = weight.shape[0], weight.shape[1]
    B = a.shape[0]
    dz = _as(dz, a.dtype)
    dx = None
    if ctx.needs_input_grad[0]:
        wf = _conv_weight(weight, a.dtype, 1)
        dx = torch.empty_like(x)
        _lib.call("msu_conv3x3_dgrad", _dt(a), 1 | (2 if d2s else 0), _p(dz), _p(wf), _p(x), _p(dx),
                  B, H, W, Cin, Cout, _s(a))
    dw, db = _conv_wgrad_param(a, dz, 2 if d2s else 0, B, H, W, Cin, Cout, *ctx.params)
    return dx, None, dw, db, None, None, None, None


_refine_conv_act = _define(
    "refine_conv_act",
    "(Tensor x, Tensor a, Tensor weight, Tensor bias, bool d2s, int H, int W, bool dual) -> (Tensor, Tensor)",
    _refine_act_impl, _refine_act_fake, _refine_act_setup, _refine_act_backward)


def refine_conv_act(x, a, weight, bias, d2s, out_hw, dual=False):
    """``conv(GELU(map(x)))`` of FinalPatchExpand_X4_V2 with a = GELU(x) supplied by the
    producer's epilogue; returns z (and GELU(z), non-differentiable, when dual)."""
    dt = act_dtype()
    H, W = out_hw
    z, z2 = _refine_conv_act(_as(x, dt), _as(a, dt), _f32(weight), _f32(bias), bool(d2s), int(H), int(W),
                             bool(dual))
    return (z, z2) if dual else z


_zero_bias_cache = {}


def _zero_bias(N, device):
    """A persistent f32 zero vector (the GELU-dual epilogue needs a bias; the expand Linear has
    none): filled once, not per call.  Inside a graph capture the fill would only be recorded,
    so a capture that finds none takes a fresh (captured) one instead of caching it."""
    key = (N, str(device))
    z = _zero_bias_cache.get(key)
    if z is None:
        z = torch.zeros(N, device=device, dtype=torch.float32)
        if not torch.cuda.is_current_stream_capturing():
            _zero_bias_cache[key] = z
    return z


def _linear_gelu_impl(x, weight):
    """y = x . W^T (no bias) and the non-differentiable GELU(y) from the same epilogue
    (FinalPatchExpand_X4_V2.expand -> act, model_parts.py:458-460); the activation gradient is
    applied by the consumer (refine_conv_act's dgrad epilogue)."""
    _need_cuda(x)
    dt = x.dtype
    w = _shadow(weight, dt)
    N, K = w.shape
    M = x.numel() // K
    if dt in _LOW and gemm_route(M, N, K, TOK_GELU_DUAL) != "lib":
        return _gemm(x, w, _zero_bias(N, x.device), TOK_GELU_DUAL)
    with torch.autocast("cuda", enabled=False):
        y = torch.nn.functional.linear(x, w)
    g = torch.empty_like(y)
    _lib.call("msu_gelu_fwd", _dt(y), _p(y), _p(g), y.numel(), _s(y))
    return y, g


def _linear_gelu_fake(x, weight):
    y = x.new_empty(*x.shape[:-1], weight.shape[0])
    return y, torch.empty_like(y)


def _linear_gelu_setup(ctx, inputs, output):
    x, weight = inputs
    ctx.save_for_backward(x)
    ctx.params = (weight,)
    ctx.mark_non_differentiable(output[1])
    ctx.set_materialize_grads(False)  # no zero-filled gradient for GELU(y)


def _linear_gelu_backward(ctx, dy, _dg):
    (x,) = ctx.saved_tensors
    (weight,) = ctx.params
    if dy is None:
        return None, None
    w = _shadow(weight, x.dtype)
    dy = _as(dy, x.dtype)
    N, K = w.shape
    M = dy.numel() // N
    dx = None
    if ctx.needs_input_grad[0]:
        if x.dtype in _LOW and gemm_route(M, K, N) != "lib":
            dx = _gemm_dx(dy, w, param=weight)
        else:
            with torch.autocast("cuda", enabled=False):
                dx = dy.matmul(w)
    dw, _ = _wgrad(dy, x, weight, None, M, N, K)
    return dx, dw


_linear_gelu = _define("linear_gelu", "(Tensor x, Tensor weight) -> (Tensor, Tensor)",
                       _linear_gelu_impl, _linear_gelu_fake, _linear_gelu_setup, _linear_gelu_backward)


def linear_gelu(x, weight):
    """(x . W^T, GELU(x . W^T)): the second output is not differentiable."""
    _need_cuda(x)
    return _linear_gelu(_as(x, act_dtype()), weight)


# ----------------------------------------------------------------------------- patch embed
def _patchify_impl(img, patch, dtype_code):
    _need_cuda(img)
    img = _f32(img)
    B, Cin, H, W = img.shape
    dtype = {v: k for k, v in _DT.items()}[dtype_code]
    out = torch.empty(B * (H // patch) * (W // patch), Cin * patch * patch, device=img.device, dtype=dtype)
    _lib.call("msu_patchify", dtype_code, _p(img), _p(out), B, Cin, H, W, patch, _s(img))
    return out


def _patchify_fake(img, patch, dtype_code):
    B, Cin, H, W = img.shape
    dtype = {v: k for k, v in _DT.items()}[dtype_code]
    return img.new_empty(B * (H // patch) * (W // patch), Cin * patch * patch, dtype=dtype)


_patchify = _define("patchify", "(Tensor img, int patch, int dtype) -> Tensor", _patchify_impl, _patchify_fake)


def patchify(img, patch, dtype):
    """[B, Cin, H, W] f32 image -> [B*(H/p)*(W/p), Cin*p*p] im2col rows (no grad)."""
    _need_cuda(img)
    return _patchify(img, int(patch), _DT[dtype])


# ----------------------------------------------------------------------------- loss
# A one-float f32 flag the loss forward zeroes every step (the trainer's non-finite flag: the
# check after backward then only sets it, and no fill launch resets it).  None: nothing.
_step_flag = [None, False]  # [flag, reset by a loss launch since it was registered]


def set_step_flag(flag):
    """Register (or clear, None) the trainer's non-finite flag for the DynamicLoss forward to
    reset each step."""
    _step_flag[0] = flag
    _step_flag[1] = False


def step_flag_reset():
    """Whether a DynamicLoss launch reset the registered flag since it was registered."""
    return _step_flag[1]


def _dynloss_impl(logits, target, alpha, beta, mix):
    _need_cuda(logits, target)
    logits = logits.contiguous()
    target = _f32(target)
    B = logits.shape[0]
    N = logits[0].numel()
    L = _lib.lib()
    nblk = L.msu_dynloss_nblk(N)
    part = torch.empty(B * nblk * 12, device=logits.device, dtype=torch.float32)
    # the loss is a 0-dim output of its own (no select after the op: its backward would fill and
    # copy); coef [4B] plus the binarised flag in its last float
    out = torch.empty((), device=logits.device, dtype=torch.float32)
    coef = torch.empty(B * 4 + 1, device=logits.device, dtype=torch.float32)
    zero = _step_flag[0] if _step_flag[0] is not None and _step_flag[0].device == logits.device else None
    if zero is not None:
        _step_flag[1] = True
    _lib.call("msu_dynloss_fwd3", _dt(logits), _p(logits), _p(target), B, N, alpha, beta, mix,
              _p(part), nblk, _p(out), coef.data_ptr() + 16 * B, _p(coef), _p(zero), _s(logits))
    return out, coef


def _dynloss_fake(logits, target, alpha, beta, mix):
    return logits.new_empty((), dtype=torch.float32), logits.new_empty(logits.shape[0] * 4 + 1, dtype=torch.float32)


def _dynloss_setup(ctx, inputs, output):
    logits, target, alpha, beta, mix = inputs
    out, coef = output
    ctx.save_for_backward(logits.contiguous(), _f32(target), coef, out)
    ctx.cfg = (alpha, beta, mix)
    ctx.mark_non_differentiable(coef)
    ctx.set_materialize_grads(False)


def _dynloss_backward(ctx, g, _gc):
    logits, target, coef, out = ctx.saved_tensors
    alpha, beta, mix = ctx.cfg
    if g is None:
        return None, None, None, None, None
    B = logits.shape[0]
    N = logits[0].numel()
    g = _f32(g.reshape(1))
    dl = torch.empty(logits.shape, device=logits.device, dtype=torch.float32)
    _lib.call("msu_dynloss_bwd2", _dt(logits), _p(logits), _p(target), _p(coef), coef.data_ptr() + 16 * B,
              _p(g), B, N, alpha, beta, mix, _p(dl), _s(logits))
    return dl.to(logits.dtype), None, None, None, None


_dynamic_loss = _define(
    "dynamic_loss", "(Tensor logits, Tensor target, float alpha, float beta, float mix) -> (Tensor, Tensor)",
    _dynloss_impl, _dynloss_fake, _dynloss_setup, _dynloss_backward)


def dynamic_loss(logits, target, alpha, beta, mix):
    if target.dim() == 3:
        target = target.unsqueeze(1)
    if logits.shape[0] != target.shape[0]:
        raise ValueError(f"Batchsize from ouptut {logits.shape[0]} not equal to batchsize target {target.shape[0]}")
    if logits.shape[1:] != target.shape[1:]:
        raise ValueError(f"target shape {tuple(target.shape)} does not match output {tuple(logits.shape)}")
    if logits.dtype not in _DT:
        logits = logits.float()
    return _dynamic_loss(logits, target, float(alpha), float(beta), float(mix))[0]


# ----------------------------------------------------------------------------- optimizer
def adamw_(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step,
           inv_scale=None, found_inf=None):
    """In-place torch.optim.AdamW update over flat f32 buffers (one launch)."""
    _need_cuda(param)
    _lib.call("msu_adamw", _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), param.numel(), lr, beta1,
              beta2, eps, weight_decay, int(step), _p(inv_scale), _p(found_inf), _s(param))


def nonfinite_(x, flag, x2=None):
    """flag[0] = 1 if x (or x2) holds an inf / NaN (flag is zeroed by the caller)."""
    if x2 is None:
        _lib.call("msu_nonfinite", _p(x), x.numel(), _p(flag), _s(x))
    else:
        _lib.call("msu_nonfinite2", _p(x), x.numel(), _p(x2), x2.numel(), _p(flag), _s(x))


def adamw_dev_(param, grad, exp_avg, exp_avg_sq, hyper, beta1, beta2, eps, weight_decay, inv_scale=None,
               found_inf=None, shadow=None, zero_grad=False):
    """AdamW over flat f32 buffers with lr and step read from the device tensor
    ``hyper = [lr, step]`` (f64); no update at all when found_inf[0] != 0.  shadow: a 16-bit
    buffer of param's length receiving the updated values (the trainer's bf16 shadow);
    zero_grad: grad is zeroed in the same pass (also on a skipped step)."""
    _need_cuda(param)
    if shadow is None and not zero_grad:
        _lib.call("msu_adamw_dev", _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), param.numel(), _p(hyper),
                  beta1, beta2, eps, weight_decay, _p(inv_scale), _p(found_inf), _s(param))
        return
    if shadow is not None and (shadow.numel() != param.numel() or shadow.dtype not in _LOW):
        raise ValueError("adamw_dev_: the shadow must be a 16-bit buffer of the parameters' length")
    _lib.call("msu_adamw_dev2", _p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), param.numel(), _p(hyper),
              beta1, beta2, eps, weight_decay, _p(inv_scale), _p(found_inf), _p(shadow),
              _DT[shadow.dtype] if shadow is not None else 0, int(bool(zero_grad)), _s(param))


def step_advance_(hyper, found_inf=None):
    """hyper[1] += 1 unless found_inf[0] != 0 (a skipped step is not counted)."""
    _lib.call("msu_step_advance", _p(hyper), _p(found_inf), _s(hyper))
