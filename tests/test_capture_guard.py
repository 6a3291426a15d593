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
    assert T.rccl_capture_blocker(None) is None


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
