"""Test-only fault injection and the failure classification used by recovery.

``DTG_FAULT`` holds comma-separated directives:

* ``kill_ps_at_step:N``  -- a PS task whose ``global_step`` variable reaches N dies abruptly
  (``os._exit(23)``, no clean shutdown: connections drop mid-request), once per process;
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
