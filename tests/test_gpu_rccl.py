"""GPU: the data-parallel product path over RCCL (torch.distributed backend "nccl").

A one-rank RCCL process group on one MI355X drives the real ``Trainer`` with the bucketed
gradient all-reduce forced on (``always_reduce``): every bucket's all-reduce is issued on the
bucketer's own comm stream while backward runs (after waiting for the main and the
weight-gradient side stream), ``finish()`` orders AdamW after the sums, all without a host
sync.  This is the replacement of the reference's ``nn.DataParallel`` (trainer.py:96-97) and
the code the 8-GPU scaling run executes; with one rank the sum is the identity, so:

* eager steps with the RCCL bucketer are bitwise identical to eager steps without it;
* the HIP-graph-captured step (the all-reduces captured into the graph) replays to the eager
  result (same tolerance as tests/test_gpu_graph.py);
* the f16 gradient wire (BASELINE config 5) with its dynamic scale stays within f16 rounding
  of the f32 step.

The scenarios run in one spawned child process (``rccl_runs``) with
``TORCH_NCCL_CUDA_EVENT_CACHE=0``: with the event cache, a later capture in the same process
could hand the watchdog thread an event recorded in the capture, and its query terminated the
process (r03j: the whole pytest run; r03p: the child, log attached to the failure).
"""
import os
import socket
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu

import cases  # noqa: E402
from oracle.msunet import make_cfg  # noqa: E402

DEV = "cuda"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(pg, graph, reduce, wire=None, steps=5, bucket_mb=1.0, lr=1e-3):
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config, ops
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    m = MSUNetSys(img_size=cfg["img_size"], embed_dim=cfg["embed_dim"], depths=cfg["depths"],
                  num_heads=cfg["num_heads"], drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0)
    m.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
    m = m.to(DEV).train()
    x, t = cases.model_inputs(cfg, 2, spec["seed"])
    x, t = x.to(DEV), t.to(DEV)
    tr = Trainer(m, load_config(None, "swin_t", **{"TRAIN.BASE_LR": lr}), DEV, use_graph=graph,
                 graph_warmup=2, process_group=pg, always_reduce=reduce, bucket_mb=bucket_mb,
                 grad_wire_dtype=wire)
    losses = []
    for i in range(steps):
        xi, ti = (x, t) if i % 2 == 0 else (x.flip(-1), t.flip(-1))
        losses.append(tr.step(xi, ti).item())
    torch.cuda.synchronize()
    ops.set_grad_ready_callback(None)
    info = {"captured": tr._graph is not None, "skipped": tr.skipped_steps(),
            "buckets": len(tr.reducer.buckets) if tr.reducer is not None else 0,
            "comm": tr.reducer.comm is not None if tr.reducer is not None else None,
            # (bucket, thread, "hook" | "finish", capturing) of the captured collectives, and
            # the thread that captured (all from finish() on the capturing thread)
            "capture_launches": getattr(tr, "capture_launches", None),
            "thread": threading.get_ident()}
    _KEEP.append(tr)  # see _child
    return losses, [torch.cat([g.data, g.exp_avg, g.exp_avg_sq]) for g in tr.groups], info


_KEEP = []


def _scenarios():
    """(name, kwargs of _run) in the order the child process runs them."""
    return [("no_dp", dict(graph=False, reduce=False, dp=False)),
            ("eager64k", dict(graph=False, reduce=True, bucket_mb=1 / 16)),
            ("eager_lr0", dict(graph=False, reduce=True, bucket_mb=1 / 4, lr=0.0)),
            ("graph_lr0", dict(graph=True, reduce=True, bucket_mb=1 / 4, lr=0.0)),
            ("graph_a", dict(graph=True, reduce=True, bucket_mb=1 / 4, side=False)),
            ("graph_b", dict(graph=True, reduce=True, bucket_mb=1 / 4, side=False)),
            ("f32", dict(graph=False, reduce=True)),
            ("f16", dict(graph=False, reduce=True, wire=torch.float16))]


def _child(rank, port, outdir):
    """All scenarios in one fresh process with one 1-rank RCCL group (spawned by the fixture:
    the state the rest of the GPU suite leaves in the test process -- captured graphs, side
    streams, allocator pools -- stays out of these captures; an abort here fails these tests
    instead of ending the whole suite)."""
    import torch.distributed as dist
    # the child's stdout / stderr (RCCL / HIP / c10d messages included) go to a log the fixture
    # attaches to a failure
    fd = os.open(os.path.join(outdir, "child.log"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    os.dup2(fd, 1)
    os.dup2(fd, 2)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # ProcessGroupNCCL's event cache hands a retired work's HIP events to new works: an event
    # recorded inside a capture could then be queried by the watchdog thread for an eager work
    # ("operation not permitted on an event last recorded in a capturing stream", which
    # terminates the process -- seen at the second capture of a process, r03o / r03p).
    # Fresh events per work, as the Trainer documents for captured steps over RCCL.
    os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    pg = dist.group.WORLD
    # the stage-0 block Linears take the one-pass backward (msu_linear_bwd, main stream, dW / db
    # straight into the flat .grad) as they do at the bench's size: the bucketer's readiness
    # counts and stream edges cover it too
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    assert ops._LINBWD
    ops._LINBWD_MIN_M = 1
    for name, kw in _scenarios():
        kw = dict(kw)
        dp = kw.pop("dp", True)
        # the determinism pair runs its eager warmup steps without the side stream (see
        # tests/test_gpu_graph.py::test_graph_replay_is_deterministic)
        from semantic_segmentation_of_stylegan2_artifacts_amd import ops
        ops._side_enabled = kw.pop("side", True)
        losses, states, info = _run(pg if dp else None, **kw)
        ops._side_enabled = True
        torch.save({"losses": losses, "states": [t.cpu() for t in states], "info": info},
                   os.path.join(outdir, f"{name}.pt"))
        torch.cuda.synchronize()
    # every Trainer (and its captured graph) stays alive until the group is destroyed (_KEEP)
    torch.cuda.synchronize()
    dist.destroy_process_group()
    _KEEP.clear()


@pytest.fixture(scope="module")
def rccl_runs(tmp_path_factory):
    import torch.multiprocessing as mp
    out = tmp_path_factory.mktemp("rccl")
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_child, args=(0, _free_port(), str(out)))
    p.start()
    p.join(600)
    if p.is_alive():
        p.kill()
        p.join()
    res = {}
    for name, _ in _scenarios():
        f = os.path.join(out, f"{name}.pt")
        if os.path.exists(f):
            res[name] = torch.load(f, weights_only=True)
    res["_exitcode"] = p.exitcode
    log = os.path.join(out, "child.log")
    res["_log"] = open(log).read()[-3000:] if os.path.exists(log) else ""
    return res


def _get(runs, name):
    assert name in runs, (f"RCCL child process ended (exit code {runs['_exitcode']}) before scenario {name}; "
                          f"its log ends:\n{runs['_log']}")
    r = runs[name]
    return r["losses"], r["states"], r["info"]


def test_rccl_bucketer_eager_equals_no_dp(rccl_runs):
    l0, s0, _ = _get(rccl_runs, "no_dp")
    l1, s1, info = _get(rccl_runs, "eager64k")  # 64 KB buckets
    assert info["buckets"] > 40 and info["comm"] and info["skipped"] == 0
    assert l0 == l1
    for a, b in zip(s0, s1):
        assert torch.equal(a, b)


def test_rccl_bucketer_graph_replay_equals_eager(rccl_runs):
    """lr = 0 as in tests/test_gpu_graph.py: every step computes the same gradient, so the
    AdamW moments of 2 eager steps + 3 replays equal those of 5 eager steps.  (With lr > 0 the
    single-stream replay's different f32 summation order of side- and main-stream gradient
    shares moves near-zero gradients by an ulp, which AdamW's g / sqrt(v) turns into
    lr-sized parameter differences: not a property of the all-reduce.)"""
    le, se, _ = _get(rccl_runs, "eager_lr0")
    lg, sg, info = _get(rccl_runs, "graph_lr0")
    assert info["buckets"] > 10
    assert info["captured"], "the step with RCCL all-reduces was not captured"
    log = info["capture_launches"]
    assert sorted(b for b, *_ in log) == list(range(info["buckets"]))
    assert all(via == "finish" and tid == info["thread"] and cap for _, tid, via, cap in log), log
    assert lg == pytest.approx(le, rel=1e-6, abs=1e-7), (le, lg)
    for a, b in zip(se, sg):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-9)


def test_rccl_bucketer_graph_replay_is_deterministic(rccl_runs):
    """Two captures of the step with its RCCL all-reduces replay bitwise identically (lr > 0)."""
    la, sa, ia = _get(rccl_runs, "graph_a")
    lb, sb, ib = _get(rccl_runs, "graph_b")
    assert ia["captured"] and ib["captured"]
    assert la == lb
    for a, b in zip(sa, sb):
        assert torch.equal(a, b)


def test_rccl_fp16_wire_matches_f32_step(rccl_runs):
    """config 5's f16 gradient wire, scaled: one rank's sum is its own f16-rounded (scaled)
    gradient, so the step matches the f32 step to f16 rounding and no step is skipped."""
    lf, sf, _ = _get(rccl_runs, "f32")
    lh, sh, info = _get(rccl_runs, "f16")
    assert info["skipped"] == 0
    assert lh[0] == lf[0]  # same weights before the first update
    assert lh == pytest.approx(lf, rel=1e-3)
    # parameters after 5 AdamW steps (lr 1e-3): f16 rounding of the gradients perturbs the
    # normalised update by at most a few 2^-11 of lr per step
    for a, b in zip(sf, sh):
        n = a.numel() // 3
        assert (a[:n] - b[:n]).abs().max().item() < 5 * 1e-3
