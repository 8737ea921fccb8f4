"""Observability + fault injection: Prometheus counters from the Infer loop, stage timers,
UNAVAILABLE mapping, injected faults surface as per-request errors (stream continues)."""
import pytest

from lumen_amd.proto import ml_service as pb
from lumen_amd.runtime import metrics
from lumen_amd.services.base import BaseInferenceService


class _Svc(BaseInferenceService):
    SERVICE_NAME = "test-svc"

    def __init__(self):
        super().__init__()
        self.registry.register_task("echo", lambda p, m, meta: (p, "text/plain", {}), "echo")
        self.registry.register_task("down", self._down, "unavailable")

    def _down(self, p, m, meta):
        class BackendNotInitializedError(Exception):
            pass

        raise BackendNotInitializedError("not ready")


def test_metrics_and_errors(monkeypatch):
    s = _Svc()
    reqs = [pb.InferRequest(correlation_id="a", task="echo", payload=b"x"),
            pb.InferRequest(correlation_id="b", task="down", payload=b"x")]
    out = list(s.Infer(iter(reqs), None))
    assert out[0].result == b"x" and out[1].error.code == pb.ERROR_CODE_UNAVAILABLE
    text = metrics.exposition().decode()
    assert 'lumen_requests_total{service="test-svc",status="ok",task="echo"}' in text
    monkeypatch.setenv("LUMEN_FAULT", "infer:1.0")
    out = list(s.Infer(iter([pb.InferRequest(correlation_id="c", task="echo", payload=b"y"),
                             pb.InferRequest(correlation_id="d", task="echo", payload=b"z")]), None))
    assert [r.error.code for r in out] == [pb.ERROR_CODE_INTERNAL] * 2 and "injected" in out[0].error.message


def test_stage_timer():
    t = metrics.StageTimer("unit", gpu=False)
    with t.stage("decode"):
        sum(range(1000))
    with t.stage("forward"):
        pass
    m = t.meta()
    assert set(m) == {"t_decode_ms", "t_forward_ms"}
    assert "lumen_stage_seconds" in metrics.exposition().decode()
