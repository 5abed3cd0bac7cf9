"""CPU tests of the auxiliary utilities: JSONL metrics sink, timers, scaling efficiency
 and the roctx tracing ranges."""
import json

import pytest

from pytorch_distributed_training_tutorials_amd.utils import metrics, tracing


def test_jsonl_sink_rank0_only(tmp_path):
    p = tmp_path / "sub" / "m.jsonl"
    metrics.JsonlSink(str(p), rank=1).write(step=1)  # non-zero rank: disabled
    assert not p.exists()
    s = metrics.JsonlSink(str(p), rank=0)
    s.write(step=1, samples_per_s=10.0)
    s.write(step=2, samples_per_s=20.0, rank=7)  # explicit fields win over the defaults
    recs = [json.loads(l) for l in p.read_text().splitlines()]
    assert [r["step"] for r in recs] == [1, 2]
    assert recs[0]["rank"] == 0 and recs[1]["rank"] == 7 and "ts" in recs[0]


def test_jsonl_sink_all_ranks_and_disabled(tmp_path):
    p = tmp_path / "m.jsonl"
    metrics.JsonlSink(str(p), rank=3, all_ranks=True).write(x=1)
    assert json.loads(p.read_text())["rank"] == 3
    metrics.JsonlSink(None).write(x=2)  # no path: a no-op


def test_timer_calls_sync_on_both_edges():
    calls = []
    with metrics.Timer(sync=lambda: calls.append(1)) as t:
        pass
    assert len(calls) == 2 and t.elapsed >= 0.0


def test_scaling_efficiency():
    e = metrics.scaling_efficiency({1: 100.0, 2: 180.0, 8: 400.0})
    assert e == pytest.approx({1: 1.0, 2: 0.9, 8: 0.5})
    assert metrics.scaling_efficiency({2: 5.0}) == {}


def test_trace_is_a_noop_when_disabled(monkeypatch):
    tracing.enable(False)
    with tracing.trace("fwd"):
        pass
    tracing.mark("x")
    assert not tracing.enabled()


def test_trace_ranges_when_enabled():
    tracing.enable(True)
    try:
        if not tracing.enabled():
            pytest.skip("no libroctx64 in this environment")
        with tracing.trace("fwd"):  # push/pop through the real library
            tracing.mark("inside")
    finally:
        tracing.enable(False)
