"""CPU: the Trainer never captures a step into an RCCL process group whose event cache is on
(VERDICT r3 weak 7a): ``rccl_capture_blocker`` names the reason, the constructor then keeps the
step eager on every rank, and a capture forced later raises instead of letting c10d's watchdog
abort the process (hipErrorCapturedEvent)."""
import torch.distributed as dist

from semantic_segmentation_of_stylegan2_artifacts_amd import trainer as T


class _PG:
    def __init__(self, backend):
        self.backend = backend


def _fake_backend(monkeypatch):
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_backend", lambda pg=None: pg.backend)


def test_blocker_nccl_with_event_cache(monkeypatch):
    _fake_backend(monkeypatch)
    monkeypatch.delenv("TORCH_NCCL_CUDA_EVENT_CACHE", raising=False)
    why = T.rccl_capture_blocker(_PG("nccl"))
    assert why and "TORCH_NCCL_CUDA_EVENT_CACHE=0" in why
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "1")
    assert T.rccl_capture_blocker(_PG("nccl"))


def test_no_blocker_when_cache_off_or_gloo_or_no_group(monkeypatch):
    _fake_backend(monkeypatch)
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    assert T.rccl_capture_blocker(_PG("nccl")) is None
    monkeypatch.delenv("TORCH_NCCL_CUDA_EVENT_CACHE", raising=False)
    assert T.rccl_capture_blocker(_PG("gloo")) is None
    monkeypatch.setattr(dist, "is_initialized", lambda: False)
    assert T.rccl_capture_blocker(None) is None  # no process group at all


def test_forced_capture_raises(monkeypatch):
    _fake_backend(monkeypatch)
    monkeypatch.delenv("TORCH_NCCL_CUDA_EVENT_CACHE", raising=False)

    class _Reducer:
        pg = _PG("nccl")

    tr = T.Trainer.__new__(T.Trainer)
    tr.reducer = _Reducer()
    tr.amp_dtype = None
    try:
        tr._capture(None, None)
    except RuntimeError as e:
        assert "TORCH_NCCL_CUDA_EVENT_CACHE" in str(e)
    else:
        raise AssertionError("capture over an RCCL group with the event cache on did not raise")


def test_blocker_resolves_default_group(monkeypatch):
    """process_group=None means the default (WORLD) group once torch.distributed is initialised
    (ADVICE r4): an RCCL default group with the event cache on blocks the capture."""
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_backend", lambda pg=None: "nccl" if pg is None else pg.backend)
    monkeypatch.delenv("TORCH_NCCL_CUDA_EVENT_CACHE", raising=False)
    assert T.rccl_capture_blocker(None)
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    assert T.rccl_capture_blocker(None) is None


def test_capture_launches_every_bucket_from_finish_on_the_capturing_thread():
    """The r04f abort: autograd runs backward on its own device thread, and a bucket
    collective issued from a post-accumulate-grad hook there during a thread-local capture was
    handed to c10d's watchdog as eager work.  Invariant: while ``capturing`` is set, no hook
    launches a bucket; finish(), called on the capturing thread, launches all of them.  The
    backward runs on a second thread here, as autograd's device thread does for GPU tensors."""
    import socket
    import threading

    import torch
    import torch.nn as nn

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        m = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 32), nn.ReLU(), nn.Linear(32, 8))
        named = list(m.named_parameters())
        groups = [T.FlatGroup([(n, p) for n, p in named if p.ndim > 1][::-1], 0.01, "cpu"),
                  T.FlatGroup([(n, p) for n, p in named if p.ndim == 1][::-1], 0.0, "cpu")]
        red = T.GradBucketer(groups, 64)  # 64 B: a bucket per parameter
        x = torch.randn(4, 16)

        def backward():
            m(x).square().mean().backward()

        me = threading.get_ident()
        for step, capturing in enumerate([False, False, True, False]):
            red.capturing = capturing
            t = threading.Thread(target=backward)
            t.start()
            t.join()
            red.finish()
            red.capturing = False
            log = red.last_launches
            assert sorted(b for b, *_ in log) == list(range(len(red.buckets)))
            if capturing:
                assert all(via == "finish" and tid == me and cap for _, tid, via, cap in log), log
            elif step > 0:  # step 0 learns the accumulation counts: everything from finish()
                hooks = [tid for _, tid, via, _ in log if via == "hook"]
                assert hooks and all(tid != me for tid in hooks), log
            for g in groups:
                g.grad.zero_()
    finally:
        dist.destroy_process_group()
