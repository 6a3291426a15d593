"""GPU: the HIP-graph replay of the training step (Trainer.step after its warmup steps).

* Replaying the captured step is the eager step: same losses and, after five steps (three
  of them replays), the same parameters and AdamW moments as a trainer that never captures
  (bf16 training mode, dropout off, same batches).
* Randomness stays live under replay: with attention dropout and stochastic depth on, two
  replays on the same batch and unchanged weights (lr = 0) give different losses -- the
  device seed counter and the redrawn drop-path pools are part of the graph -- while with
  every drop rate at zero they are bitwise equal.
* A write through a parameter between steps (load_state_dict) is seen by the next replay.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

import cases  # noqa: E402
from oracle.msunet import make_cfg  # noqa: E402

DEV = "cuda"


def _model(drop_path=0.0, attn_drop=0.0):
    from semantic_segmentation_of_stylegan2_artifacts_amd.network.model_parts import MSUNetSys
    spec = cases.model_cases()["swinT224"]
    cfg = make_cfg(**spec["cfg"])
    m = MSUNetSys(img_size=cfg["img_size"], embed_dim=cfg["embed_dim"], depths=cfg["depths"],
                  num_heads=cfg["num_heads"], drop_rate=0.0, attn_drop_rate=attn_drop, drop_path_rate=drop_path)
    m.load_state_dict(cases.model_params(cfg, spec["seed"]), strict=True)
    x, t = cases.model_inputs(cfg, 2, spec["seed"])
    return m.to(DEV).train(), x.to(DEV), t.to(DEV)


def _conf(lr):
    from semantic_segmentation_of_stylegan2_artifacts_amd import load_config
    return load_config(None, "swin_t", **{"TRAIN.BASE_LR": lr})


def _run(graph, lr, steps=5):
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    model, x, t = _model()
    tr = Trainer(model, _conf(lr), DEV, use_graph=graph, graph_warmup=2)
    losses = []
    for i in range(steps):
        xi, ti = (x, t) if i % 2 == 0 else (x.flip(-1), t.flip(-1))
        losses.append(tr.step(xi, ti).item())
    torch.cuda.synchronize()
    assert (tr._graph is not None) == graph
    return losses, [torch.cat([g.data, g.exp_avg, g.exp_avg_sq]) for g in tr.groups], tr.optimizer_steps()


def test_graph_replay_is_deterministic():
    """Two independent captures replay to bitwise-identical losses, parameters and moments.

    The two eager warmup steps run with the side stream off: with both the weight gradients and
    the attention parameter tail on the side stream, about one eager run in ten differs from
    the others at f32 rounding level in the encoder's gradients (tools/determinism_matrix.py
    parts, profiles/r03u_determinism.txt; the captured step itself is single-stream)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    prev = ops._side_enabled
    ops._side_enabled = False
    try:
        a, b = _run(True, 1e-3), _run(True, 1e-3)
    finally:
        ops._side_enabled = prev
    assert a[0] == b[0]
    for u, v in zip(a[1], b[1]):
        assert torch.equal(u, v)


def test_graph_replay_computes_the_eager_step():
    """With lr = 0 the weights stay put, so every step computes the same gradient: the AdamW
    moments accumulated over 2 eager steps + 3 replays equal those of 5 eager steps, the
    losses agree step by step (the replay runs the same kernels; only independent work may be
    scheduled in another order, so f32 sums of side-stream and main-stream shares may round
    differently)."""
    le, se, ne = _run(False, 0.0)
    lg, sg, ng = _run(True, 0.0)
    assert ne == ng == 5
    assert lg == pytest.approx(le, rel=1e-6, abs=1e-7), (le, lg)
    for a, b in zip(se, sg):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("drop", [False, True])
def test_graph_replay_draws_new_dropout_masks(drop):
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    model, x, t = _model(drop_path=0.2 if drop else 0.0, attn_drop=0.1 if drop else 0.0)
    tr = Trainer(model, _conf(0.0), DEV, use_graph=True, graph_warmup=2)
    for _ in range(2):
        tr.step(x, t)
    l1 = tr.step(x, t).item()  # capture + first replay
    l2 = tr.step(x, t).item()
    l3 = tr.step(x, t).item()
    assert tr._graph is not None
    if drop:
        assert l1 != l2 and l2 != l3, (l1, l2, l3)
    else:
        assert l1 == l2 == l3, (l1, l2, l3)


def test_graph_replay_sees_parameter_writes():
    from semantic_segmentation_of_stylegan2_artifacts_amd.trainer import Trainer
    model, x, t = _model()
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    tr = Trainer(model, _conf(0.0), DEV, use_graph=True, graph_warmup=2)
    for _ in range(3):
        base = tr.step(x, t).item()
    with torch.no_grad():
        model.output.weight.mul_(3.0)  # a write through a parameter
    changed = tr.step(x, t).item()
    assert changed != base
    model.load_state_dict(sd)  # back: the replay must see this write too
    again = tr.step(x, t).item()
    assert again == pytest.approx(base, rel=1e-6, abs=1e-7)


@pytest.mark.xfail(strict=False, reason="open: with the side stream on, about 1 eager run in 9 differed at f32 "
                                        "rounding level in encoder gradients (profiles/r03u_determinism.txt, DESIGN 4b)")
def test_eager_side_stream_step_is_deterministic():
    """The DEFAULT eager configuration (weight gradients and the attention parameter tail on the
    side stream): four independent runs of three steps at lr 0 give bitwise-identical AdamW
    moments.  Kept next to the side-stream-off test above so that a regression or a fix of the
    open rounding-level difference shows up (xfail, non-strict)."""
    from semantic_segmentation_of_stylegan2_artifacts_amd import ops
    assert ops._side_enabled
    runs = [_run(False, 0.0, steps=3) for _ in range(4)]
    for r in runs[1:]:
        for u, v in zip(runs[0][1], r[1]):
            assert torch.equal(u, v)
