"""Launch an example as a localhost cluster of processes (the reference's own multi-node method:
one process per task), on free ports, and collect every task's output."""
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def run_cluster(script, n_ps=1, n_workers=2, args=(), timeout=120, cwd=None, env=None):
    ports = free_ports(n_ps + n_workers)
    spec = {"ps": ["127.0.0.1:%d" % p for p in ports[:n_ps]],
            "worker": ["127.0.0.1:%d" % p for p in ports[n_ps:]]}
    path = os.path.join(ROOT, "examples", script)
    base = [sys.executable, path, "--cluster", json.dumps(spec), "--observe_sleep", "0"] + list(args)
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("OMP_NUM_THREADS", "1")
    procs = []
    for t in range(n_ps):
        procs.append(("ps", t, subprocess.Popen(base + ["--job_name", "ps", "--task_index", str(t)], cwd=cwd, env=e,
                                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    for t in range(n_workers):
        procs.append(("worker", t, subprocess.Popen(base + ["--job_name", "worker", "--task_index", str(t)], cwd=cwd,
                                                    env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    out = {}
    deadline = time.time() + timeout
    try:
        for job, t, p in procs:
            left = max(1.0, deadline - time.time())
            o, _ = p.communicate(timeout=left)
            out[(job, t)] = (p.returncode, o)
    finally:
        for job, t, p in procs:
            if p.poll() is None:
                p.kill()
                p.communicate()
    return out


_NUM = r"[-+]?\d*\.\d+(?:[eE][-+]?\d+)?|[-+]?\d+"


def last_vector(text, marker):
    """First number of the last printed array on a line containing ``marker``."""
    lines = [l for l in text.splitlines() if marker in l]
    assert lines, "no line with %r in:\n%s" % (marker, text[-2000:])
    m = re.search(r"\[\s*(%s)" % _NUM, lines[-1])
    return float(m.group(1))


def last_int_after(text, marker):
    lines = [l for l in text.splitlines() if marker in l]
    m = re.search(re.escape(marker) + r"\s*\[?\s*(\d+)", lines[-1])
    return int(m.group(1))
