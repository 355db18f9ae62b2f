"""Session-run hooks (README.md:73-92 glossary).

Same names and life-cycle as tf.train: ``begin`` -> ``after_create_session`` -> per run
``before_run``/``after_run`` -> ``end``.  ``before_run`` may request extra fetches through
``SessionRunArgs``; ``after_run`` receives their values.
"""
import collections
import json
import math
import os
import time

import numpy as np


class SessionRunArgs(collections.namedtuple("SessionRunArgs", ["fetches", "feed_dict", "options"])):
    def __new__(cls, fetches, feed_dict=None, options=None):
        return super().__new__(cls, fetches, feed_dict, options)


class SessionRunValues(collections.namedtuple("SessionRunValues", ["results", "options", "run_metadata"])):
    pass


class SessionRunContext:
    def __init__(self, original_args, session):
        self.original_args = original_args
        self.session = session
        self._stop = False

    def request_stop(self):
        self._stop = True

    @property
    def stop_requested(self):
        return self._stop


class SessionRunHook:
    def begin(self):
        pass

    def after_create_session(self, session, coord):
        pass

    def before_run(self, run_context):
        return None

    def after_run(self, run_context, run_values):
        pass

    def end(self, session):
        pass


def _gs_var():
    from .optimizer import get_global_step
    return get_global_step()


class StopAtStepHook(SessionRunHook):
    """Stop once global_step >= last_step (or after num_steps more steps).  ``last_step`` is
    absolute, so a resumed run that already reached it stops immediately."""

    def __init__(self, num_steps=None, last_step=None):
        if (num_steps is None) == (last_step is None):
            raise ValueError("exactly one of num_steps and last_step must be given")
        self._num_steps, self._last_step = num_steps, last_step

    def begin(self):
        self._gs = _gs_var()
        if self._gs is None:
            raise RuntimeError("Global step should be created to use StopAtStepHook.")

    def after_create_session(self, session, coord):
        if self._last_step is None:
            self._last_step = int(session._read(self._gs)) + self._num_steps

    def before_run(self, run_context):
        return SessionRunArgs(self._gs)

    def after_run(self, run_context, run_values):
        gs = int(run_values.results)
        if gs >= self._last_step:
            run_context.request_stop()

    def should_stop_for(self, gs):
        return self._last_step is not None and gs >= self._last_step


class NanLossDuringTrainingError(RuntimeError):
    pass


class NanTensorHook(SessionRunHook):
    def __init__(self, loss_tensor, fail_on_nan_loss=True):
        self._loss, self._fail = loss_tensor, fail_on_nan_loss

    def before_run(self, run_context):
        return SessionRunArgs(self._loss)

    def after_run(self, run_context, run_values):
        if np.isnan(np.asarray(run_values.results, dtype=np.float64)).any():
            if self._fail:
                raise NanLossDuringTrainingError("NaN loss during training.")
            run_context.request_stop()


class LoggingTensorHook(SessionRunHook):
    def __init__(self, tensors, every_n_iter=None, every_n_secs=None, at_end=False, formatter=None):
        if isinstance(tensors, (list, tuple)):
            tensors = {t.name if hasattr(t, "name") else str(t): t for t in tensors}
        self._tensors = dict(tensors)
        self._n, self._secs, self._at_end, self._fmt = every_n_iter, every_n_secs, at_end, formatter
        self._iter, self._last_t, self._last_vals = 0, 0.0, None

    def _due(self):
        if self._n is not None:
            return self._iter % self._n == 0
        if self._secs is not None:
            return time.time() - self._last_t >= self._secs
        return False

    def before_run(self, run_context):
        return SessionRunArgs(self._tensors) if self._due() else None

    def after_run(self, run_context, run_values):
        if run_values.results is not None:
            self._last_vals = run_values.results
            self._last_t = time.time()
            msg = self._fmt(run_values.results) if self._fmt else ", ".join(
                "%s = %s" % (k, v) for k, v in sorted(run_values.results.items()))
            print(msg, flush=True)
        self._iter += 1

    def end(self, session):
        if self._at_end and self._tensors:
            vals = session._run_raw(self._tensors)
            print(", ".join("%s = %s" % (k, v) for k, v in sorted(vals.items())), flush=True)


class StepCounterHook(SessionRunHook):
    """global_step/sec (and examples/sec when ``batch_size`` is given) to a JSONL metrics file, the TF event
    file of ``output_dir`` and, with ``log``, stdout.

    For eager GPU steps the host runs ahead of the device, so with ``sync_device`` (default: when CUDA is
    initialised) the hook synchronises the device at each report -- only then, every ``every_n_steps`` steps --
    and the rate is the device's.  ``aggregate=True`` (all-reduce data parallelism: every rank runs the hook at
    the same global steps) sums the per-worker examples/sec over the process group at each report, so each
    record carries ``examples/sec`` (this worker) and ``examples/sec/node`` (the whole job); that is a
    collective, so it needs step-based reporting (``every_n_secs`` is refused with it)."""

    def __init__(self, every_n_steps=100, every_n_secs=None, output_dir=None, summary_writer=None, batch_size=None,
                 metrics_path=None, aggregate=False, sync_device=None, log=False, process_group=None):
        if aggregate and every_n_secs is not None:
            raise ValueError("StepCounterHook(aggregate=True) reports at fixed steps: use every_n_steps")
        self._n, self._secs = every_n_steps, every_n_secs
        self._dir, self._writer, self._bs = output_dir, summary_writer, batch_size
        self._metrics = metrics_path
        self._aggregate, self._sync, self._log, self._pg = aggregate, sync_device, log, process_group
        self._last_step, self._last_t = None, None
        self.history = []

    def begin(self):
        self._gs = _gs_var()
        if self._writer is None and self._dir:
            from .summary import FileWriter
            self._writer = FileWriter.for_dir(self._dir)

    def before_run(self, run_context):
        return SessionRunArgs(self._gs) if self._gs is not None else None

    def _device_sync(self):
        sync = self._sync
        try:
            import torch
            if sync is None:
                sync = torch.cuda.is_available() and torch.cuda.is_initialized()
            if sync:
                torch.cuda.synchronize()
        except Exception:  # noqa: BLE001 - a CPU-only build
            pass

    def _node_total(self, eps):
        try:
            import torch
            import torch.distributed as dist
        except Exception:  # noqa: BLE001
            return eps, 1
        if not (dist.is_available() and dist.is_initialized()):
            return eps, 1
        w = dist.get_world_size(self._pg)
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(self._pg) == "nccl" \
            else torch.device("cpu")
        t = torch.tensor([float(eps)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, group=self._pg)
        return float(t.item()), w

    def after_run(self, run_context, run_values):
        if run_values.results is None:
            return
        step = int(run_values.results)
        if self._last_step is None:
            self._device_sync()
            self._last_step, self._last_t = step, time.time()
            return
        due = (self._secs is not None and time.time() - self._last_t >= self._secs) or \
              (self._secs is None and step - self._last_step >= (self._n or 1))
        if not due:
            return
        self._device_sync()
        now = time.time()
        dt = max(now - self._last_t, 1e-9)
        sps = (step - self._last_step) / dt
        rec = {"step": step, "global_step/sec": sps, "time": now}
        if self._bs:
            rec["examples/sec"] = sps * self._bs
            if self._aggregate:
                rec["examples/sec/node"], rec["workers"] = self._node_total(rec["examples/sec"])
        self.history.append(rec)
        if self._writer is not None:
            self._writer.add_scalar("global_step/sec", sps, step)
            if self._bs:
                self._writer.add_scalar("examples/sec", sps * self._bs, step)
                if "examples/sec/node" in rec:
                    self._writer.add_scalar("examples/sec/node", rec["examples/sec/node"], step)
        if self._metrics:
            with open(self._metrics, "a") as f:
                f.write(json.dumps(rec) + "\n")
        if self._log:
            msg = "global_step/sec: %.4g" % sps
            if self._bs:
                msg += ", examples/sec: %.6g" % rec["examples/sec"]
                if "examples/sec/node" in rec:
                    msg += " (node %.6g over %d workers)" % (rec["examples/sec/node"], rec["workers"])
            print(msg, flush=True)
        self._last_step, self._last_t = step, now


class CheckpointSaverHook(SessionRunHook):
    """Chief-only: saves every ``save_secs`` or ``save_steps`` and at the end."""

    def __init__(self, checkpoint_dir, save_secs=None, save_steps=None, saver=None, checkpoint_basename="model.ckpt",
                 scaffold=None, listeners=None):
        if (save_secs is None) == (save_steps is None):
            raise ValueError("exactly one of save_secs and save_steps")
        self._dir, self._secs, self._steps = checkpoint_dir, save_secs, save_steps
        self._saver, self._base, self._scaffold = saver, checkpoint_basename, scaffold
        self._listeners = listeners or []
        self._last_t, self._last_step = None, None
        self.saves = 0

    def begin(self):
        from .saver import Saver
        os.makedirs(self._dir, exist_ok=True)
        if self._saver is None:
            self._saver = (self._scaffold.saver if self._scaffold is not None and self._scaffold.saver else None) or Saver()
        self._gs = _gs_var()

    def after_create_session(self, session, coord):
        from .. import graph as G
        # TF's CheckpointSaverHook writes the graph next to the checkpoints (graph.pbtxt)
        G.write_graph(G.get_default_graph(), self._dir, "graph.pbtxt")
        self._last_t = time.time()
        step = int(session._read(self._gs)) if self._gs is not None else 0
        self._save(session, step)  # TF saves the initial state too
        self._last_step = step

    def before_run(self, run_context):
        return SessionRunArgs(self._gs) if self._gs is not None else None

    def after_run(self, run_context, run_values):
        step = int(run_values.results) if run_values.results is not None else 0
        now = time.time()
        if (self._secs is not None and now - self._last_t >= self._secs) or \
           (self._steps is not None and step - self._last_step >= self._steps):
            self._save(run_context.session, step)
            self._last_t, self._last_step = now, step

    def end(self, session):
        step = int(session._read(self._gs)) if self._gs is not None else 0
        if step != self._last_step:
            self._save(session, step)

    def _save(self, session, step):
        for l in self._listeners:
            getattr(l, "before_save", lambda *a: None)(session, step)
        self._saver.save(session, os.path.join(self._dir, self._base), global_step=step)
        self.saves += 1
        for l in self._listeners:
            getattr(l, "after_save", lambda *a: None)(session, step)


class SummarySaverHook(SessionRunHook):
    """Writes scalar fetches as TF event summaries every N steps / secs."""

    def __init__(self, save_steps=None, save_secs=None, output_dir=None, summary_writer=None, scaffold=None,
                 summary_op=None):
        self._steps, self._secs = save_steps, save_secs
        self._dir, self._writer, self._op = output_dir, summary_writer, summary_op
        self._last = None
        self._i = 0

    def begin(self):
        if self._writer is None and self._dir:
            from .summary import FileWriter
            self._writer = FileWriter.for_dir(self._dir)
        self._gs = _gs_var()

    def before_run(self, run_context):
        want = {}
        if self._gs is not None:
            want["gs"] = self._gs
        if self._op is not None and (self._steps is None or self._i % self._steps == 0):
            want["summ"] = self._op
        return SessionRunArgs(want)

    def after_run(self, run_context, run_values):
        self._i += 1
        r = run_values.results or {}
        if "summ" in r and self._writer is not None:
            vals = r["summ"]
            if isinstance(vals, dict):
                for k, v in vals.items():
                    self._writer.add_scalar(k, float(np.asarray(v).mean()), int(r.get("gs", self._i)))

    def end(self, session):
        if self._writer is not None:
            self._writer.flush()


class GlobalStepWaiterHook(SessionRunHook):
    """Delays a worker's first step until global_step >= wait_until_step."""

    def __init__(self, wait_until_step):
        self._wait = wait_until_step

    def begin(self):
        self._gs = _gs_var()

    def before_run(self, run_context):
        if self._wait <= 0 or self._gs is None:
            return None
        while int(run_context.session._read(self._gs)) < self._wait:
            time.sleep(0.05)
        self._wait = 0
        return None


class FinalOpsHook(SessionRunHook):
    def __init__(self, final_ops, final_ops_feed_dict=None):
        self._ops, self._feed = final_ops, final_ops_feed_dict
        self.final_ops_values = None

    def end(self, session):
        self.final_ops_values = session._run_raw(self._ops, self._feed)


class FeedFnHook(SessionRunHook):
    def __init__(self, feed_fn):
        self._fn = feed_fn

    def before_run(self, run_context):
        return SessionRunArgs(fetches=None, feed_dict=self._fn())


class ProfilerHook(SessionRunHook):
    """roctx ranges around each run (visible in rocprofv3 --marker-trace) -- SURVEY §5.1."""

    def __init__(self, name="dtg.run"):
        self._name = name
        try:
            import torch
            self._rng = torch.cuda.nvtx if torch.cuda.is_available() else None
        except Exception:
            self._rng = None

    def before_run(self, run_context):
        if self._rng is not None:
            self._rng.range_push(self._name)
        return None

    def after_run(self, run_context, run_values):
        if self._rng is not None:
            self._rng.range_pop()


def secs_to_str(s):
    return "%dh%02dm%02ds" % (s // 3600, (s % 3600) // 60, math.floor(s % 60))
