"""Test-only fault injection and the failure classification used by recovery.

``DTG_FAULT`` holds comma-separated directives:

* ``kill_ps_at_step:N``  -- a PS task whose ``global_step`` variable reaches N dies abruptly
  (``os._exit(23)``, no clean shutdown: connections drop mid-request), once per process;
* ``kill_rank_at_step:R@N`` -- rank R of a sync-DP job dies abruptly (``os._exit(23)``) when it is about to
  run training step N (examples/ResNet50/resnet50_train.py; the survivors' watchdog or collective reports it);
* ``kill_worker_at_run:T@N`` -- worker task T of a PS job dies abruptly at its N-th session run
  (train/session.py; its PS connection drops mid-job: backup workers / timeouts must cope);
* ``drop_grad:P``        -- a worker silently drops each gradient push with probability P (a lost
  update; the async algorithms must tolerate it, sync ones need backup workers);
* ``seed:S``             -- seed of the drop decisions (default 0).

The reference has no fault handling at all (PS processes never exit, README.md:55-59); TF's
MonitoredSession recreates the session after AbortedError/UnavailableError and restores the last
checkpoint, which is what dtg's MonitoredTrainingSession does on a PS failure (train/session.py).
"""
import os
import random

KILL_EXIT_CODE = 23


def _parse():
    out = {}
    for item in os.environ.get("DTG_FAULT", "").split(","):
        item = item.strip()
        if not item:
            continue
        k, _, v = item.partition(":")
        out[k] = v
    return out


def config():
    return _parse()


def kill_ps_step():
    v = _parse().get("kill_ps_at_step")
    return int(v) if v else None


def maybe_kill_rank(rank, step):
    """``kill_rank_at_step:R@N``: die like a crashed process if this is rank R about to run step N."""
    v = _parse().get("kill_rank_at_step")
    if not v:
        return
    r, _, n = v.partition("@")
    if int(r) == int(rank) and int(n) == int(step):
        import sys
        print("dtg.fault: killing rank %d at step %d" % (rank, step), file=sys.stderr, flush=True)
        os._exit(KILL_EXIT_CODE)


def maybe_kill_worker(task, run):
    """``kill_worker_at_run:T@N``: die like a crashed process if this is worker task T at its N-th run."""
    v = _parse().get("kill_worker_at_run")
    if not v:
        return
    t, _, n = v.partition("@")
    if int(t) == int(task) and int(n) == int(run):
        import sys
        print("dtg.fault: killing worker %d at run %d" % (task, run), file=sys.stderr, flush=True)
        os._exit(KILL_EXIT_CODE)


_rng = None


def should_drop_grad():
    global _rng
    p = _parse().get("drop_grad")
    if not p:
        return False
    if _rng is None:
        _rng = random.Random(int(_parse().get("seed", "0") or 0))
    return _rng.random() < float(p)


class UnavailableError(RuntimeError):
    """A parameter-server task is unreachable (crashed, restarting, network gone)."""


def is_ps_failure(exc):
    """Did this exception come from losing a PS connection (vs. a program error)?"""
    if isinstance(exc, UnavailableError):
        return True
    msg = str(exc)
    return isinstance(exc, RuntimeError) and (msg.startswith("ps client:") or "connection lost" in msg
                                               or "send failed" in msg)
