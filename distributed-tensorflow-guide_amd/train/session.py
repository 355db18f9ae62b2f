"""Session life-cycle: Scaffold, SessionManager, MonitoredTrainingSession, Supervisor, Coordinator
(SURVEY §1 L5, §3.2-3.5, §2.8).

Bootstrap semantics:
  chief      restore the latest checkpoint of checkpoint_dir/logdir if one exists, else run
             Scaffold.init_op (creates/initialises the global variables on the PS); then
             local_init_op.
  non-chief  poll ``ready_for_local_init_op`` / ``ready_op`` (uninitialised global variables on the
             PS) with backoff until the chief has initialised them -- a real rendezvous instead of
             the reference's sleeps (DOWNPOUR/DOWNPOUR.py:131, SSGD-diff-LR/ssgd.py:95); then
             local_init_op.
  close      hooks.end; workers report done to every PS task so ``Server.join()`` returns
             (the reference's PS never exits, README.md:55-59).
"""
import atexit
import os
import threading
import time

import numpy as np

from .. import fault
from .. import graph as G
from ..graph import RunContext, to_numpy
from ..variables import (client_for, close_connections, global_variables_initializer, local_variables_initializer,
                         report_uninitialized_variables, _this_server)
from .hooks import (CheckpointSaverHook, SessionRunArgs, SessionRunContext, SessionRunValues, StepCounterHook,
                    StopAtStepHook, SummarySaverHook)
from .saver import Saver, latest_checkpoint


class Coordinator:
    def __init__(self, clean_stop_exception_types=None):
        self._stop = threading.Event()
        self._exc = None

    def request_stop(self, ex=None):
        if ex is not None and self._exc is None:
            self._exc = ex
        self._stop.set()

    def should_stop(self):
        return self._stop.is_set()

    def wait_for_stop(self, timeout=None):
        return self._stop.wait(timeout)

    def clear_stop(self):
        self._stop.clear()

    def join(self, threads=None, stop_grace_period_secs=120, ignore_live_threads=False):
        for t in threads or []:
            t.join(stop_grace_period_secs)
        if self._exc is not None:
            raise self._exc

    def raise_requested_exception(self):
        if self._exc is not None:
            raise self._exc

    class _StopOnException:
        def __init__(self, coord):
            self.c = coord

        def __enter__(self):
            return self

        def __exit__(self, et, ev, tb):
            if ev is not None:
                self.c.request_stop(ev)
            return True

    def stop_on_exception(self):
        return Coordinator._StopOnException(self)


class Scaffold:
    def __init__(self, init_op=None, init_feed_dict=None, init_fn=None, ready_op=None, ready_for_local_init_op=None,
                 local_init_op=None, summary_op=None, saver=None, copy_from_scaffold=None):
        self.init_op = init_op
        self.init_feed_dict = init_feed_dict
        self.init_fn = init_fn
        self.ready_op = ready_op
        self.ready_for_local_init_op = ready_for_local_init_op
        self.local_init_op = local_init_op
        self.summary_op = summary_op
        self.saver = saver
        self._finalized = False

    def finalize(self):
        if self._finalized:
            return self
        if self.init_op is None:
            self.init_op = global_variables_initializer()
        if self.ready_op is None:
            self.ready_op = report_uninitialized_variables()
        if self.ready_for_local_init_op is None:
            self.ready_for_local_init_op = report_uninitialized_variables(
                G.get_collection(G.GraphKeys.GLOBAL_VARIABLES))
        if self.local_init_op is None:
            self.local_init_op = local_variables_initializer()
        if self.saver is None:
            self.saver = Saver()
        self._finalized = True
        return self


def _as_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple)) else [x]


class SessionManager:
    def __init__(self, local_init_op=None, ready_op=None, ready_for_local_init_op=None, recovery_wait_secs=0.05):
        self._local_init_op = local_init_op
        self._ready_op = ready_op
        self._ready_for_local = ready_for_local_init_op
        self._wait = recovery_wait_secs

    def _run(self, sess, fetch, feed=None):
        return RunContext(sess, feed).eval(fetch)

    def prepare_session(self, sess, init_op=None, saver=None, checkpoint_dir=None, init_fn=None, init_feed_dict=None):
        ckpt = latest_checkpoint(checkpoint_dir) if checkpoint_dir else None
        if ckpt and saver is not None:
            saver.restore(sess, ckpt)
            sess.restored_from = ckpt
        else:
            for op in _as_list(init_op):
                self._run(sess, op, init_feed_dict)
            if init_fn is not None:
                init_fn(sess)
        for op in _as_list(self._local_init_op):
            self._run(sess, op)
        return sess

    def wait_for_session(self, sess, max_wait_secs=7200):
        t0 = time.time()
        wait = self._wait
        gate = self._ready_for_local if self._ready_for_local is not None else self._ready_op
        while True:
            not_ready = self._run(sess, gate) if gate is not None else np.array([])
            if len(not_ready) == 0:
                break
            if time.time() - t0 > max_wait_secs:
                raise TimeoutError("chief did not initialise %s within %ss" % (list(not_ready), max_wait_secs))
            time.sleep(wait)
            wait = min(wait * 1.5, 1.0)
        for op in _as_list(self._local_init_op):
            self._run(sess, op)
        return sess


class _Session:
    """The object ``sess.run`` is called on.  Owns hooks and the stop flag."""

    def __init__(self, target="", is_chief=True, hooks=None, config=None, coord=None):
        self.target = target
        self.is_chief = is_chief
        self.hooks = list(hooks or [])
        self.config = config
        self.coord = coord or Coordinator()
        self._should_stop = False
        self._closed = False
        self.restored_from = None
        self.graph = G.get_default_graph()
        if config is not None and getattr(config, "log_device_placement", False):
            from ..placement import DeviceSpec  # noqa: F401
            for v in G.get_collection("_all_variables"):
                print("%s: (%s): %s" % (v.op.name, "VariableV2", v.device.to_string() or "/job:localhost"))

    # -- running ----------------------------------------------------------------------------------
    def _read(self, var):
        return to_numpy(var.read_value())

    def _run_raw(self, fetches, feed_dict=None):
        return to_numpy(RunContext(self, feed_dict).eval(fetches))

    def run(self, fetches, feed_dict=None, options=None, run_metadata=None):
        # TF raises "Run called even after should_stop requested." here, which makes the reference's
        # bootstrap runs crash when a finished job is resumed from its checkpoint (the first run's
        # StopAtStepHook already requests the stop).  dtg keeps running the fetches; the training
        # loop's should_stop() check then ends the job cleanly.
        self._runs = getattr(self, "_runs", 0) + 1
        if fault.config().get("kill_worker_at_run"):
            srv = _this_server()
            if srv is not None and srv.job_name == "worker":
                fault.maybe_kill_worker(srv.task_index, self._runs)
        rc = SessionRunContext(SessionRunArgs(fetches, feed_dict), self)
        hargs = [h.before_run(rc) for h in self.hooks]
        feed = dict(feed_dict or {})
        for a in hargs:
            if a is not None and a.feed_dict:
                feed.update(a.feed_dict)
        ctx = RunContext(self, feed)
        results = ctx.eval(fetches)
        hvals = [ctx.eval(a.fetches) if (a is not None and a.fetches is not None) else None for a in hargs]
        for h, v in zip(self.hooks, hvals):
            h.after_run(rc, SessionRunValues(to_numpy(v), options, run_metadata))
        if rc.stop_requested:
            self._should_stop = True
            self.coord.request_stop()
        return to_numpy(results)

    def should_stop(self):
        return self._should_stop or self.coord.should_stop()

    def request_stop(self):
        self._should_stop = True
        self.coord.request_stop()

    def _stop_requested_externally(self):
        """Used by blocking ops (sync-token wait): has the job reached a stop condition?"""
        if self.should_stop():
            return True
        from .optimizer import get_global_step
        gs = get_global_step()
        if gs is None:
            return False
        step = int(self._read(gs))
        return any(isinstance(h, StopAtStepHook) and h.should_stop_for(step) for h in self.hooks)

    def list_devices(self):
        s = _this_server()
        devs = []
        if s is None:
            devs.append("/job:localhost/replica:0/task:0/device:CPU:0")
        else:
            for job in s.cluster.jobs:
                for t in range(s.cluster.num_tasks(job)):
                    devs.append("/job:%s/replica:0/task:%d/device:CPU:0" % (job, t))
        try:
            import torch
            for i in range(torch.cuda.device_count() if torch.cuda.is_available() else 0):
                devs.append("/job:%s/replica:0/task:%d/device:GPU:%d" % (
                    s.job_name if s else "localhost", s.task_index if s else 0, i))
        except Exception:
            pass
        return devs

    # -- shutdown -----------------------------------------------------------------------------
    def _report_done(self):
        s = _this_server()
        if s is None or s.job_name == "ps":
            return
        for t in range(s.cluster.num_tasks("ps")):
            try:
                client_for("ps", t, timeout=2.0).worker_done(s.task_index)
            except Exception:
                pass

    def close(self):
        if self._closed:
            return
        self._closed = True
        for h in self.hooks:
            h.end(self)
        self._report_done()

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        self.close()
        return False


class _MonitoredSession(_Session):
    """A session that survives the loss of a PS task (TF's _RecoverableSession semantics): when a run
    fails because a PS connection dropped, it reconnects (waiting, with backoff, for the PS to come
    back), recreates the session -- the chief restores the latest checkpoint into the restarted PS,
    a non-chief waits until the chief has re-initialised it -- and re-runs the same fetches.
    SURVEY.md §5.3; exercised by tests/test_fault_cpu.py with DTG_FAULT=kill_ps_at_step:N."""

    max_recoveries = 10
    _recreate = None

    def run(self, fetches, feed_dict=None, options=None, run_metadata=None):
        attempts = 0
        while True:
            try:
                return _Session.run(self, fetches, feed_dict, options, run_metadata)
            except Exception as e:  # noqa: BLE001 - classified below
                if self._recreate is None or not fault.is_ps_failure(e) or attempts >= self.max_recoveries:
                    raise
                attempts += 1
                print("[dtg] PS failure during run (%s): recovering session (attempt %d)" % (e, attempts),
                      flush=True)
                self._recreate()


def _ps_backed():
    """Does any global variable live on a parameter server?  Without one (all-reduce data parallelism, eager
    models) a non-chief has nothing to wait for: it initialises its own variables, and the sync hook gives it
    the chief's state (train/eager.py broadcast_training_state)."""
    return any(getattr(v, "remote", False) for v in G.get_collection(G.GraphKeys.GLOBAL_VARIABLES))


def _make_recreate(sess, sm, scaffold, checkpoint_dir, is_chief, hooks, timeout):
    def recreate():
        close_connections()
        s = _this_server()
        if s is not None and "ps" in s.cluster.jobs:
            for t in range(s.cluster.num_tasks("ps")):
                client_for("ps", t, timeout=timeout).ping()  # blocks (with backoff) until the PS is back
        if is_chief:
            sm.prepare_session(sess, scaffold.init_op, scaffold.saver, checkpoint_dir, scaffold.init_fn,
                               scaffold.init_feed_dict)
        elif not _ps_backed():
            sm.prepare_session(sess, scaffold.init_op, None, None, scaffold.init_fn, scaffold.init_feed_dict)
        else:
            sm.wait_for_session(sess, timeout)
        print("[dtg] session recovered%s" % (" from " + sess.restored_from if sess.restored_from else ""),
              flush=True)
        for h in hooks:
            h.after_create_session(sess, sess.coord)
    return recreate


def MonitoredTrainingSession(master="", is_chief=True, checkpoint_dir=None, scaffold=None, hooks=None,
                             chief_only_hooks=None, save_checkpoint_secs=600, save_summaries_steps=100,
                             save_summaries_secs=None, config=None, stop_grace_period_secs=120,
                             log_step_count_steps=100, max_wait_secs=7200, save_checkpoint_steps=None,
                             summary_dir=None):
    """tf.train.MonitoredTrainingSession (DOWNPOUR/DOWNPOUR.py:121-127, Synchronous-SGD/ssgd.py:65-69)."""
    scaffold = (scaffold or Scaffold()).finalize()
    all_hooks = list(hooks or [])
    if is_chief:
        all_hooks += list(chief_only_hooks or [])
        out = summary_dir or checkpoint_dir
        if out:
            if log_step_count_steps and log_step_count_steps > 0:
                all_hooks.append(StepCounterHook(every_n_steps=log_step_count_steps, output_dir=out))
            if save_summaries_steps or save_summaries_secs:
                all_hooks.append(SummarySaverHook(save_steps=save_summaries_steps, save_secs=save_summaries_secs,
                                                  output_dir=out, scaffold=scaffold))
        if checkpoint_dir and (save_checkpoint_secs or save_checkpoint_steps):
            all_hooks.append(CheckpointSaverHook(checkpoint_dir, save_secs=save_checkpoint_secs if not
                                                 save_checkpoint_steps else None, save_steps=save_checkpoint_steps,
                                                 scaffold=scaffold))
    for h in all_hooks:
        h.begin()
    sess = _MonitoredSession(master, is_chief, all_hooks, config)
    sm = SessionManager(local_init_op=scaffold.local_init_op, ready_op=scaffold.ready_op,
                        ready_for_local_init_op=scaffold.ready_for_local_init_op)
    if is_chief:
        sm.prepare_session(sess, scaffold.init_op, scaffold.saver, checkpoint_dir, scaffold.init_fn,
                           scaffold.init_feed_dict)
    elif not _ps_backed():
        sm.prepare_session(sess, scaffold.init_op, None, None, scaffold.init_fn, scaffold.init_feed_dict)
    else:
        sm.wait_for_session(sess, max_wait_secs)
    for h in all_hooks:
        h.after_create_session(sess, sess.coord)
    sess._recreate = _make_recreate(sess, sm, scaffold, checkpoint_dir, is_chief, all_hooks,
                                    float(os.environ.get("DTG_RECOVERY_SECS", "120")))
    atexit.register(sess.close)
    return sess


class Supervisor:
    """tf.train.Supervisor (Hogwild/Hogwild.py:47-50, Distributed-Setup/dist_setup_sup.py:43-44)."""

    def __init__(self, graph=None, ready_op=0, is_chief=True, init_op=0, init_feed_dict=None, local_init_op=0,
                 logdir=None, summary_op=0, saver=0, global_step=0, save_summaries_secs=120, save_model_secs=600,
                 recovery_wait_secs=0.05, stop_grace_secs=120, checkpoint_basename="model.ckpt",
                 session_manager=None, summary_writer=0, init_fn=None):
        from .optimizer import get_global_step
        self.is_chief = is_chief
        self.logdir = logdir
        self.init_op = global_variables_initializer() if init_op == 0 else init_op
        self.local_init_op = local_variables_initializer() if local_init_op == 0 else local_init_op
        self.ready_op = report_uninitialized_variables() if ready_op == 0 else ready_op
        self.saver = Saver() if saver == 0 else saver
        self.global_step = get_global_step() if global_step == 0 else global_step
        self.save_model_secs = save_model_secs
        self.checkpoint_basename = checkpoint_basename
        self.init_fn = init_fn
        self.init_feed_dict = init_feed_dict
        self.coord = Coordinator()
        self._sess = None
        self._saver_thread = None
        self._stop_ev = threading.Event()
        self._sm = session_manager or SessionManager(local_init_op=self.local_init_op, ready_op=self.ready_op,
                                                     recovery_wait_secs=recovery_wait_secs)

    @property
    def save_path(self):
        return os.path.join(self.logdir, self.checkpoint_basename) if self.logdir else None

    def prepare_or_wait_for_session(self, master="", config=None, wait_for_checkpoint=False, max_wait_secs=7200,
                                    start_standard_services=True):
        sess = _Session(master, self.is_chief, [], config, self.coord)
        if self.is_chief:
            if self.logdir:
                os.makedirs(self.logdir, exist_ok=True)
                from .. import graph as G
                G.write_graph(G.get_default_graph(), self.logdir, "graph.pbtxt")  # Supervisor._write_graph
            self._sm.prepare_session(sess, self.init_op, self.saver, self.logdir, self.init_fn, self.init_feed_dict)
            if start_standard_services and self.logdir and self.save_model_secs and self.save_model_secs > 0:
                self._saver_thread = threading.Thread(target=self._save_loop, daemon=True, name="sv_saver")
                self._saver_thread.start()
        else:
            self._sm.wait_for_session(sess, max_wait_secs)
        self._sess = sess
        atexit.register(self.stop)
        return sess

    def _save(self):
        if self.saver is None or not self.logdir:
            return
        gs = None
        if self.global_step is not None:
            gs = int(to_numpy(self.global_step.read_value()))
        self.saver.save(self._sess, self.save_path, global_step=gs)

    def _save_loop(self):
        while not self._stop_ev.wait(self.save_model_secs):
            try:
                self._save()
            except Exception as e:  # pragma: no cover - best effort background service
                print("supervisor checkpoint failed:", e)

    def should_stop(self):
        return self.coord.should_stop()

    def request_stop(self, ex=None):
        self.coord.request_stop(ex)

    def stop(self, threads=None, close_summary_writer=True, ignore_live_threads=False):
        if self._stop_ev.is_set():
            return
        self._stop_ev.set()
        self.coord.request_stop()
        if self._saver_thread is not None:
            self._saver_thread.join(5)
        if self.is_chief and self._sess is not None and self.logdir:
            try:
                self._save()
            except Exception:
                pass
        if self._sess is not None:
            self._sess.close()

    def managed_session(self, master="", config=None, start_standard_services=True):
        sv = self

        class _Ctx:
            def __enter__(self_inner):
                return sv.prepare_or_wait_for_session(master, config, start_standard_services=start_standard_services)

            def __exit__(self_inner, et, ev, tb):
                sv.stop()
                return False
        return _Ctx()


class Session(_Session):
    """tf.Session(target): a plain session (Servers.ipynb:180)."""

    def __init__(self, target="", graph=None, config=None):
        super().__init__(target, True, [], config)


class ChiefSessionCreator:
    def __init__(self, scaffold=None, master="", config=None, checkpoint_dir=None):
        self.scaffold, self.master, self.config, self.checkpoint_dir = scaffold, master, config, checkpoint_dir

    def create_session(self):
        return MonitoredTrainingSession(self.master, True, self.checkpoint_dir, self.scaffold, config=self.config,
                                        save_checkpoint_secs=None)


class WorkerSessionCreator:
    def __init__(self, scaffold=None, master="", config=None):
        self.scaffold, self.master, self.config = scaffold, master, config

    def create_session(self):
        return MonitoredTrainingSession(self.master, False, None, self.scaffold, config=self.config,
                                        save_checkpoint_secs=None)


def MonitoredSession(session_creator=None, hooks=None):
    s = (session_creator or ChiefSessionCreator()).create_session()
    for h in hooks or []:
        h.begin()
        h.after_create_session(s, s.coord)
        s.hooks.append(h)
    return s
