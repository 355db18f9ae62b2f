"""Integration tests: every reference example run as a localhost multi-process cluster on the CPU,
checked against the analytic oracles of SURVEY §4.3 (TF is not installed, so these closed-form
end states replace running the reference) or, where interleaving makes values timing-dependent,
against invariants (global_step reaches last_step, c moves monotonically toward 100, every task
exits -- including the parameter server, which the reference has to pkill)."""
import os

import pytest

from _cluster import last_int_after, last_vector, run_cluster


def _ok(out):
    for (job, t), (rc, o) in out.items():
        assert rc == 0, "%s:%d exited %s\n%s" % (job, t, rc, o[-3000:])


def test_downpour_one_worker_oracle(tmp_path):
    out = run_cluster("DOWNPOUR/DOWNPOUR.py", 1, 1, ["--logdir", str(tmp_path / "logdir")])
    _ok(out)
    w = out[("worker", 0)][1]
    assert abs(last_vector(w, "global step") - 0.00281919) < 1e-7
    assert last_int_after(w, "global step:") == 60
    assert last_int_after(w, "local step:") == 120  # T-1 = 2 local applies per global step
    assert "Session from worker 0 closed cleanly" in w
    # TF-layout checkpoint with the g/ mirror keys and the PS-side Adagrad slots
    import dtg
    ck = dtg.train.latest_checkpoint(str(tmp_path / "logdir"))
    assert ck.endswith("model.ckpt-60")
    keys = dtg.train.NewCheckpointReader(ck).get_variable_to_shape_map()
    assert {"global_step", "g/Variable", "g/Variable_1", "g/Variable/Adagrad", "g/Variable_1/Adagrad"} <= set(keys)
    assert "Variable" not in keys and "local_step" not in keys  # local variables are not saved
    # graph.pbtxt next to the checkpoints (TF's CheckpointSaverHook): the chief's GraphDef text proto
    gp = (tmp_path / "logdir" / "graph.pbtxt").read_text()
    assert 'name: "global_step"' in gp and 'op: "VariableV2"' in gp and gp.rstrip().endswith("}")
    assert 'name: "g/Variable"' in gp and 'device: "/job:ps/task:0' in gp


def test_downpour_resume_stops_immediately(tmp_path):
    logdir = str(tmp_path / "logdir")
    _ok(run_cluster("DOWNPOUR/DOWNPOUR.py", 1, 1, ["--logdir", logdir]))
    out = run_cluster("DOWNPOUR/DOWNPOUR.py", 1, 1, ["--logdir", logdir])
    _ok(out)
    w = out[("worker", 0)][1]
    # restored global_step = 60 >= last_step (absolute): the job stops before any training step
    assert "global step:" not in w
    assert "Session from worker 0 closed cleanly" in w
    import dtg
    r = dtg.train.NewCheckpointReader(dtg.train.latest_checkpoint(logdir))
    assert int(r.get_tensor("global_step")) == 60


def test_downpour_two_workers(tmp_path):
    out = run_cluster("DOWNPOUR/DOWNPOUR.py", 1, 2, ["--logdir", str(tmp_path / "l")])
    _ok(out)
    steps = [last_int_after(out[("worker", i)][1], "global step:") for i in range(2)]
    assert max(steps) >= 60
    c = last_vector(out[("worker", 0)][1], "global step")
    assert 0.0 < c < 100.0


def test_downpour_easy(tmp_path):
    out = run_cluster("DOWNPOUR-Easy/DOWNPOUR.py", 1, 2, ["--logdir", str(tmp_path / "l")])
    _ok(out)
    assert max(last_int_after(out[("worker", i)][1], "global step:") for i in range(2)) >= 60


def test_adag_one_worker_oracle(tmp_path):
    out = run_cluster("ADAG/ADAG.py", 1, 1, ["--logdir", str(tmp_path / "l"), "--debug_window", "0"])
    _ok(out)
    w = out[("worker", 0)][1]
    assert abs(last_vector(w, "global step") - 0.79672914) < 2e-6
    assert last_int_after(w, "global step:") == 40


def test_adag_two_workers_with_debug_prints(tmp_path):
    out = run_cluster("ADAG/ADAG.py", 1, 2, ["--logdir", str(tmp_path / "l")])
    _ok(out)


def test_ssgd_lockstep_oracle():
    out = run_cluster("Synchronous-SGD/ssgd.py", 1, 2, ["--init_tokens", "0"])
    _ok(out)
    for i in range(2):
        w = out[("worker", i)][1]
        assert abs(last_vector(w, "step:") - 0.1998201) < 2e-6
        assert last_int_after(w, "step: ") == 10


def test_ssgd_tf_token_semantics():
    """TF default tokens: workers may run one step ahead; accepted run-ahead gradients are computed
    one step stale, so c lands within a step of the lock-step oracle and global_step hits 10."""
    out = run_cluster("Synchronous-SGD/ssgd.py", 1, 2)
    _ok(out)
    w = out[("worker", 0)][1]
    assert abs(last_vector(w, "step:") - 0.1998201) < 2e-4
    assert last_int_after(w, "step: ") >= 10


def test_ssgd_backup_worker_drops_gradients():
    """3 workers, aggregate 2: the third gradient of each step is a backup (dropped as stale)."""
    out = run_cluster("Synchronous-SGD/ssgd.py", 1, 3, ["--init_tokens", "0"])
    _ok(out)
    assert last_int_after(out[("worker", 0)][1], "step: ") >= 10


def test_ssgd_different_lr_oracle():
    out = run_cluster("Synchronous-SGD-different-learning-rates/ssgd.py", 1, 2, ["--init_tokens", "0"])
    _ok(out)
    assert abs(last_vector(out[("worker", 0)][1], "step:") - 89.289395) < 1e-3


def test_sdag_equals_ssgd():
    out = run_cluster("SDAG/dist_cpu_sing_mach_sync.py", 1, 2, ["--init_tokens", "0"])
    _ok(out)
    lines = [l for l in out[("worker", 1)][1].splitlines() if l.startswith("[")]
    assert abs(float(lines[-1].strip("[").split()[0]) - 0.1998201) < 2e-6


def test_hogwild_two_workers(tmp_path):
    out = run_cluster("Hogwild/Hogwild.py", 1, 2, ["--steps", "300", "--logdir", str(tmp_path / "l")])
    _ok(out)
    import re
    # both elements of every printed c (the two start from different random values, so each is checked against its
    # own trajectory)
    vals = [[float(v) for v in re.findall(r"[-\d.e+]+", l)] for l in out[("worker", 0)][1].splitlines()
            if l.startswith("[")]
    assert len(vals) == 30 and all(len(v) == 2 for v in vals)
    gaps = [[100 - v for v in row] for row in vals]
    assert all(b[e] <= a[e] + 1e-3 for a, b in zip(gaps, gaps[1:]) for e in range(2))  # monotone toward 100
    import dtg
    ck = dtg.train.latest_checkpoint(str(tmp_path / "l"))
    # the reference minimises without a global step (Hogwild/Hogwild.py:44), so its Supervisor writes a plain
    # model.ckpt holding only the two variables
    assert os.path.basename(ck) == "model.ckpt", ck
    r = dtg.train.NewCheckpointReader(ck)
    assert set(r.get_variable_to_shape_map()) == {"Variable", "Variable_1"}
    # the chief's final save holds its own 300 applies and whatever of the other worker's had landed: c moved
    # from ~0 most of the way a 300-step run gets toward 100
    c = r.get_tensor("Variable") + r.get_tensor("Variable_1")
    assert all(100 - c[e] <= gaps[-1][e] + 1e-3 for e in range(2))


def test_distributed_setup_mts():
    _ok(run_cluster("Distributed-Setup/dist_setup.py", 1, 1, ["--steps", "50"]))


def test_distributed_setup_supervisor(tmp_path):
    out = run_cluster("Distributed-Setup/dist_setup_sup.py", 1, 1, ["--steps", "50", "--logdir", str(tmp_path / "l")])
    _ok(out)
    assert os.path.exists(tmp_path / "l" / "checkpoint")
    assert 'op: "VariableV2"' in (tmp_path / "l" / "graph.pbtxt").read_text()  # Supervisor writes the graph


def test_multi_gpu_example_runs_on_cpu(tmp_path):
    out = run_cluster("Multiple-GPUs-Single-Machine/dist_mult_gpu_sing_mach.py", 1, 2,
                      ["--steps", "40", "--logdir", str(tmp_path / "l")], env={"HIP_VISIBLE_DEVICES": "-1"})
    _ok(out)
    import dtg
    ck = dtg.train.latest_checkpoint(str(tmp_path / "l"))  # no global step in the reference either
    assert os.path.basename(ck) == "model.ckpt", ck
    assert set(dtg.train.NewCheckpointReader(ck).get_variable_to_shape_map()) == {"Variable", "Variable_1"}


def test_non_distributed_gap_factor():
    import subprocess
    import sys
    from _cluster import ROOT
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "Non-Distributed_Setup.py"), "--observe_sleep",
                        "0"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    import re
    vals = [float(re.search(r"\[\s*([-\d.e+]+)", l).group(1)) for l in p.stdout.splitlines() if l.startswith("[")]
    assert len(vals) == 100
    ratio = (100 - vals[-1]) / (100 - vals[0])
    assert abs(ratio - 0.9998 ** 990) < 1e-4  # gap shrinks by (1 - 2 lr) per step; it does not converge


def _aeasgd_oracle(steps_global, tau, alpha, lr, momentum=0.0):
    """One worker, sequential: local (momentum-)SGD on c = a + b -> 100, elastic coupling every tau."""
    import numpy as np
    a = np.zeros(2, np.float64)
    b = np.zeros(2, np.float64)
    ca, cb = a.copy(), b.copy()
    ma, mb = np.zeros(2), np.zeros(2)
    gs = 0
    while gs < steps_global:
        for _ in range(tau):
            g = (a + b - 100.0)  # d/da mean((a+b-100)^2) over 2 elements = 2(c-100)/2
            if momentum > 0:
                ma = momentum * ma + g
                mb = momentum * mb + g
                a, b = a - lr * ma, b - lr * mb
            else:
                a, b = a - lr * g, b - lr * g
        da, db = alpha * (a - ca), alpha * (b - cb)
        a, b = a - da, b - db
        ca, cb = ca + da, cb + db
        gs += 1
    return a + b, ca + cb


def test_aeasgd_single_worker_matches_oracle():
    from _cluster import run_cluster
    out = run_cluster("AEASGD/AEASGD.py", n_ps=1, n_workers=1,
                      args=["--tau", "3", "--alpha", "0.5", "--lr", "0.1", "--last_step", "8"])
    rc, o = out[("worker", 0)]
    assert rc == 0, o
    c_local, c_center = _aeasgd_oracle(8, 3, 0.5, 0.1)
    center_line = [l for l in o.splitlines() if l.startswith("center")][-1]
    vals = [float(x) for x in center_line.split("[")[1].split("]")[0].split()]
    assert abs(vals[0] - c_center[0]) < 1e-3 * max(1.0, abs(c_center[0])), (vals, c_center)


def test_aemasgd_two_workers_converge():
    from _cluster import run_cluster
    out = run_cluster("AEASGD/AEASGD.py", n_ps=1, n_workers=2,
                      args=["--tau", "2", "--alpha", "0.3", "--lr", "0.05", "--momentum", "0.5", "--last_step", "30"])
    for t in range(2):
        rc, o = out[("worker", t)]
        assert rc == 0, o
    center_line = [l for l in out[("worker", 0)][1].splitlines() if l.startswith("center")][-1]
    vals = [float(x) for x in center_line.split("[")[1].split("]")[0].split()]
    assert all(abs(v - 100.0) < 5.0 for v in vals), vals


def test_notebook_shared_ps_protocol():
    """Basics-Tutorial/Multiple-Workers through its run.sh: both workers move the ONE shared `g/a` on the PS,
    +0.1 per global update whichever worker applies it (Local-then-Global-Variables-Worker1.ipynb:224, :286,
    :313 and -Worker2.ipynb:217, :286: -1.17584 -> -1.07584 -> -0.97584); every task exits 0."""
    import json
    import re
    import subprocess
    from _cluster import ROOT, free_ports
    ports = free_ports(3)
    spec = {"ps": ["127.0.0.1:%d" % ports[0]], "worker": ["127.0.0.1:%d" % p for p in ports[1:]]}
    sh = os.path.join(ROOT, "examples", "Basics-Tutorial", "Multiple-Workers", "run.sh")
    p = subprocess.run(["bash", sh, "--cluster", json.dumps(spec)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert p.returncode == 0, p.stdout + p.stderr

    def val(label):
        got = [float(re.search(r"\[\s*([-\d.e+]+)", l).group(1)) for l in p.stdout.splitlines() if l.startswith(label)]
        assert got, (label, p.stdout)
        return got
    x0 = val("a_global init:")[0]
    assert -2.0 < x0 < 2.0  # Glorot-random start, like the notebook's -1.26032 / -1.17584
    assert val("local a:") == [pytest.approx(0.1)]  # the local step leaves the global copy alone
    assert val("a_global after worker 1 update:")[0] == pytest.approx(x0 + 0.1, abs=1e-6)
    assert val("a_global seen by worker 2:")[0] == pytest.approx(x0 + 0.1, abs=1e-6)
    after2 = val("a_global after worker 2 update:")
    assert len(after2) == 2 and all(v == pytest.approx(x0 + 0.2, abs=1e-6) for v in after2)


@pytest.mark.gpu
def test_multi_gpu_example_workers_on_gpu(tmp_path):
    """The Multiple-GPUs-Single-Machine example with its workers' compute on the GPU (both on cuda:0 of a
    one-GPU box; one GPU per worker through HIP_VISIBLE_DEVICES on a node, dist_mult_gpu_sing_mach.sh;
    reference dist_mult_gpu_sing_mach.py:31-39): ConfigProto.hip_device / placement resolve to cuda."""
    out = run_cluster("Multiple-GPUs-Single-Machine/dist_mult_gpu_sing_mach.py", 1, 2,
                      ["--steps", "30", "--logdir", str(tmp_path / "l")], timeout=240)
    _ok(out)
    for t in range(2):
        w = out[("worker", t)][1]
        assert "worker %d computes on cuda:0" % t in w, w[-2000:]
