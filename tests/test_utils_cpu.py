"""dtg.utils on the CPU: StepTimer (wall-clock fallback), MetricsLogger (JSONL), trace ranges (no-op
without a GPU, and a no-op when DTG_TRACE is off)."""
import json
import time

import dtg  # noqa: F401
from dtg.utils import MetricsLogger, StepTimer, trace_range, traced
from dtg.utils import trace as tr


def test_step_timer_cpu():
    t = StepTimer(batch_size=64, device="cpu")
    for _ in range(3):
        t.start()
        time.sleep(0.01)
        t.stop()
    ts = t.times_ms()
    assert len(ts) == 3 and all(v >= 9.0 for v in ts)
    s = t.summary()
    assert s["steps"] == 3 and abs(s["examples_per_sec"] - 64e3 / s["ms_median"]) < 1e-6


def test_metrics_logger_jsonl(tmp_path):
    path = tmp_path / "m" / "metrics.jsonl"
    log = MetricsLogger(str(path), rank=1, model="resnet50")
    log.log(step=1, loss=2.5)
    log.log(step=2, loss=2.0, images_per_sec=13950.0)
    recs = MetricsLogger.read(str(path))
    assert [r["step"] for r in recs] == [1, 2]
    assert recs[1]["rank"] == 1 and recs[1]["model"] == "resnet50" and recs[1]["images_per_sec"] == 13950.0
    assert json.loads(path.read_text().splitlines()[0])["loss"] == 2.5


def test_trace_ranges_are_noops_off_gpu():
    tr.set_trace(True)
    try:
        with trace_range("dtg.test"):
            x = 1

        @traced("dtg.fn")
        def f(a):
            return a + 1
        assert f(x) == 2
    finally:
        tr.set_trace(False)
    assert not tr.trace_enabled()
