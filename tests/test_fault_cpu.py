"""Fault injection: the PS dies mid-run (DTG_FAULT=kill_ps_at_step:N), the
harness restarts it, and the worker's MonitoredTrainingSession reconnects, restores the latest
checkpoint into the new PS and finishes the job."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JOB = os.path.join(ROOT, "tests", "jobs", "fault_job.py")


def _free_port():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    return free_ports(2)


def _spawn(role, cluster, logdir, env_extra=None):
    env = dict(os.environ)
    env.pop("DTG_FAULT", None)
    env.update(env_extra or {})
    env["DTG_RECOVERY_SECS"] = "60"
    return subprocess.Popen([sys.executable, JOB, "--job_name", role, "--task_index", "0", "--cluster",
                             json.dumps(cluster), "--logdir", logdir], stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT, text=True, env=env)


def test_ps_crash_restart_recovers_from_checkpoint(tmp_path):
    p_ps, p_w = _free_port()
    cluster = {"ps": ["127.0.0.1:%d" % p_ps], "worker": ["127.0.0.1:%d" % p_w]}
    logdir = str(tmp_path / "logdir")
    ps = _spawn("ps", cluster, logdir, {"DTG_FAULT": "kill_ps_at_step:17"})
    worker = _spawn("worker", cluster, logdir)
    procs = [ps, worker]
    try:
        ps_out, _ = ps.communicate(timeout=120)
        assert ps.returncode == 23, ps_out  # fault.KILL_EXIT_CODE
        assert "killing ps task 0" in ps_out
        time.sleep(0.5)  # the worker notices the lost connection and starts retrying
        ps2 = _spawn("ps", cluster, logdir)
        procs.append(ps2)
        w_out, _ = worker.communicate(timeout=180)
        assert worker.returncode == 0, w_out
        ps2.communicate(timeout=60)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    res = json.loads([l for l in w_out.splitlines() if l.startswith("RESULT ")][-1][len("RESULT "):])
    assert "recovering session" in w_out and "session recovered from" in w_out, w_out
    assert res["final_step"] >= 60
    # the restored checkpoint is one the first PS incarnation wrote before it died
    killed_at = int(ps_out.split("at global_step")[1].split()[0])
    restored = int(res["restored_from"].rsplit("-", 1)[1])
    assert restored % 5 == 0 and 5 <= restored <= killed_at, (restored, killed_at)


def test_dropped_gradient_pushes_are_lost_updates(tmp_path):
    """DTG_FAULT=drop_grad:0.5 on the worker: about half the pushes (and the global-step increments
    they carry) never reach the PS, yet async training still reaches last_step."""
    p_ps, p_w = _free_port()
    cluster = {"ps": ["127.0.0.1:%d" % p_ps], "worker": ["127.0.0.1:%d" % p_w]}
    ps = _spawn("ps", cluster, str(tmp_path / "l"))
    worker = subprocess.Popen([sys.executable, JOB, "--job_name", "worker", "--cluster", json.dumps(cluster),
                               "--logdir", str(tmp_path / "l"), "--last_step", "30", "--step_sleep", "0"],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                              env=dict(os.environ, DTG_FAULT="drop_grad:0.5,seed:3"))
    try:
        w_out, _ = worker.communicate(timeout=120)
        ps.communicate(timeout=60)
    finally:
        for p in (ps, worker):
            if p.poll() is None:
                p.kill()
    assert worker.returncode == 0, w_out
    res = json.loads([l for l in w_out.splitlines() if l.startswith("RESULT ")][-1][len("RESULT "):])
    assert res["final_step"] >= 30
    assert res["local_runs"] > 1.4 * res["final_step"], res


def test_ssgd_backup_workers_survive_a_dead_worker():
    """SURVEY §4.2 fault injection, sync mode: 3 workers aggregating 2 per step (one backup); worker 2 dies at
    its 3rd run.  The chief keeps aggregating the two live workers' gradients to the last step, and the PS
    counts the dead worker as finished (its watched connection dropped) so it exits too."""
    from _cluster import last_int_after, run_cluster
    # the guide's pacing at 1/10 (the chief 0.2 s per step): with none, the two live workers could finish all
    # 10 steps before worker 2 reached its 3rd run, and it then exited cleanly instead of dying
    out = run_cluster("Synchronous-SGD/ssgd.py", 1, 3, ["--init_tokens", "0", "--observe_sleep", "0.1"],
                      env={"DTG_FAULT": "kill_worker_at_run:2@3"}, timeout=120)
    assert out[("worker", 2)][0] == 23
    for t in (0, 1):
        rc, o = out[("worker", t)]
        assert rc == 0, o[-2000:]
    assert last_int_after(out[("worker", 0)][1], "step: ") >= 10
    assert out[("ps", 0)][0] == 0


def test_ssgd_without_backups_fails_cleanly_on_a_dead_worker():
    """Same loss without a backup (2 of 2): the survivor cannot complete a step; it fails with a clear
    SyncTimeoutError (TF: DeadlineExceededError) instead of waiting forever."""
    from _cluster import run_cluster
    out = run_cluster("Synchronous-SGD/ssgd.py", 1, 2, ["--init_tokens", "0"],
                      env={"DTG_FAULT": "kill_worker_at_run:1@3", "DTG_SYNC_TIMEOUT": "20"}, timeout=120)
    assert out[("worker", 1)][0] == 23
    rc, o = out[("worker", 0)]
    assert rc != 0 and "SyncTimeoutError" in o and "a worker may be lost" in o, o[-2000:]
