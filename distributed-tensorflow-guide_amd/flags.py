"""Command-line flags shared by every example (SURVEY §2.2 "Role flags", §5.6).

Same two flags as the reference with the same defaults, parsed with ``parse_known_args`` so
unknown flags are ignored (e.g. Hogwild/Hogwild.py:59-76).  dtg adds optional extensions:
``--cluster`` (JSON, or ``$DTG_CLUSTER``) to override the hard-coded ClusterSpec,
``--observe_sleep`` to keep or drop the reference's "so we can observe training" sleeps
(default: keep, for demo parity; the tests pass 0), and ``--logdir``.
"""
import argparse
import json
import os


def parser(description=None):
    p = argparse.ArgumentParser(description=description)
    p.add_argument("--job_name", type=str, default="", help="One of 'ps', 'worker'")
    p.add_argument("--task_index", type=int, default=0, help="Index of task within the job")
    p.add_argument("--cluster", type=str, default=os.environ.get("DTG_CLUSTER", ""),
                   help="JSON cluster spec overriding the script's default (dtg extension)")
    p.add_argument("--observe_sleep", type=float, default=float(os.environ.get("DTG_OBSERVE_SLEEP", "1")),
                   help="scale for the reference's observation sleeps (0 = no sleeping)")
    p.add_argument("--logdir", type=str, default=None, help="checkpoint/log directory override")
    p.add_argument("--init_tokens", type=int, default=-1,
                   help="SyncReplicas initial tokens: -1 = TF default (replicas_to_aggregate, lets workers run "
                        "one step ahead); 0 = strict lock-step (every step aggregates fresh gradients)")
    return p


def parse(argv=None, description=None, extra=None):
    p = parser(description)
    if extra:
        extra(p)
    flags, _unparsed = p.parse_known_args(argv)
    return flags


def cluster_from(flags, default):
    from .cluster import ClusterSpec
    return ClusterSpec(json.loads(flags.cluster)) if getattr(flags, "cluster", "") else ClusterSpec(default)


def sleep(flags, secs):
    """The reference's throttling sleeps, scaled by --observe_sleep."""
    import time
    s = secs * float(getattr(flags, "observe_sleep", 1.0))
    if s > 0:
        time.sleep(s)
