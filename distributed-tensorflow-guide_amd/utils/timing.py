"""Per-step GPU timing without synchronising the training loop (SURVEY §5.1 "HIP-event step timers").

    timer = StepTimer(batch_size=512)
    for _ in range(steps):
        timer.start()
        step()
        timer.stop()
    print(timer.summary())        # ms/step (median / mean / min), examples/sec

``start``/``stop`` record HIP events on the current stream; their elapsed times are only read when
``summary()`` / ``times_ms()`` is called (one synchronisation at the end), so the host keeps
queueing work ahead of the GPU.  On CPU (or when no GPU is present) wall-clock time is used.
"""
import statistics
import time


class StepTimer:
    def __init__(self, batch_size=None, device=None):
        self.batch_size = batch_size
        self._pending = []      # (start, end) event pairs not yet read
        self._ms = []           # resolved step times
        self._cur = None
        self._cuda = False
        try:
            import torch
            self._cuda = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
            self._torch = torch
        except Exception:
            self._torch = None

    def start(self):
        if self._cuda:
            ev = self._torch.cuda.Event(enable_timing=True)
            ev.record()
            self._cur = ev
        else:
            self._cur = time.perf_counter()

    def stop(self):
        if self._cur is None:
            raise RuntimeError("StepTimer.stop() without start()")
        if self._cuda:
            ev = self._torch.cuda.Event(enable_timing=True)
            ev.record()
            self._pending.append((self._cur, ev))
        else:
            self._ms.append((time.perf_counter() - self._cur) * 1e3)
        self._cur = None

    def times_ms(self):
        """All step times so far (synchronises on the last recorded event once)."""
        if self._pending:
            self._pending[-1][1].synchronize()
            self._ms.extend(a.elapsed_time(b) for a, b in self._pending)
            self._pending = []
        return list(self._ms)

    def summary(self):
        ts = self.times_ms()
        if not ts:
            return {"steps": 0}
        out = {"steps": len(ts), "ms_median": statistics.median(ts), "ms_mean": statistics.fmean(ts),
               "ms_min": min(ts)}
        if self.batch_size:
            out["examples_per_sec"] = self.batch_size * 1e3 / out["ms_median"]
        return out
