"""SyncReplicasOptimizer's all-reduce mode and session-driven eager training (train/eager.py), on 2 gloo ranks:

* the eager train op under MonitoredTrainingSession (sync hook, StopAtStepHook) is bit-identical to the plain
  DataParallel loop (``dp.step(opt)``) -- parameters and momentum slots;
* checkpoints written by CheckpointSaverHook are keyed by the model's parameter names (+ slots, global_step),
  and a job stopped at step 3 and resumed to step 6 ends bit-identical to an uninterrupted 6-step job, with the
  global step continuing from the checkpoint and the non-chief rank taking the chief's restored state;
* StepCounterHook(aggregate=True) reports per-worker and whole-job examples/sec;
* graph variables not on a PS (the reference's ssgd.py shape without a PS) are averaged over ranks;
* backup workers (R < M) and a replica count that is not the world size are refused in all-reduce mode.

Reference: /root/reference/Synchronous-SGD/ssgd.py:51-69, /root/reference/DOWNPOUR/DOWNPOUR.py:116-127.
"""
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mlp():
    from dtg.models.layers import Linear

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = Linear(16, 32, act="relu")
            self.b = Linear(32, 32, act="relu")
            self.c = Linear(32, 4)

        def forward(self, x):
            return self.c(self.b(self.a(x)))
    return M()


def _init(rank, world, port):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DTG_WATCHDOG="0")
    import dtg  # noqa: F401
    from dtg.parallel import comm
    comm.init("gloo")


def _batch(step, rank):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(8, 16, generator=g), torch.randint(0, 4, (8,), generator=g)


def _spawn(fn, *args, world=2):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    res = dict(q.get(timeout=5) for _ in range(world))
    for p in procs:
        if p.is_alive():
            p.kill()
    return res


# ---- 1. eager train op == DataParallel loop ----------------------------------------------------------------
def _rank_equiv(rank, world, port, q):
    try:
        _init(rank, world, port)
        import dtg
        from dtg import ops
        from dtg.optim import FusedSGD
        from dtg.parallel import DataParallel, FlatParams, comm
        torch.manual_seed(0)
        ma = _mlp()
        torch.manual_seed(0)
        mb = _mlp()
        fa = FlatParams(ma, compute_dtype=torch.float32)
        fb = FlatParams(mb, compute_dtype=torch.float32)
        # A: the TF-shaped path
        x_ph, y_ph = dtg.placeholder(), dtg.placeholder()
        gs = dtg.train.get_or_create_global_step()
        sro = dtg.train.SyncReplicasOptimizer(FusedSGD(fa, lr=0.1, momentum=0.9, weight_decay=1e-4),
                                              replicas_to_aggregate=world, total_num_replicas=world, bucket_mb=0.001)
        train_op = sro.minimize(lambda x, y: ops.softmax_cross_entropy(ma(x), y), global_step=gs, inputs=(x_ph, y_ph))
        assert sro.mode == "allreduce" and len(sro.dp.buckets) > 2
        hooks = [sro.make_session_run_hook(rank == 0), dtg.train.StopAtStepHook(last_step=4)]
        losses = []
        with dtg.train.MonitoredTrainingSession(is_chief=rank == 0, hooks=hooks) as sess:
            while not sess.should_stop():
                step = int(sess.run(gs))
                x, y = _batch(step, rank)
                _, loss, g = sess.run([train_op, train_op.loss, gs], feed_dict={x_ph: x, y_ph: y})
                losses.append(float(loss))
        assert int(g) == 4 and len(losses) == 4
        # B: the plain loop
        dp = DataParallel(fb, bucket_mb=0.001)
        dp.broadcast_parameters(0)
        ob = FusedSGD(fb, lr=0.1, momentum=0.9, weight_decay=1e-4)
        for step in range(4):
            x, y = _batch(step, rank)
            ops.softmax_cross_entropy(mb(x), y).backward()
            dp.step(ob)
        for ga, gb in zip(fa, fb):
            assert torch.equal(ga.master, gb.master), ga.name
            assert torch.equal(ga.state["momentum"], gb.state["momentum"]), ga.name
        assert sro._flat_opt.step_count == ob.step_count == 4
        comm.shutdown()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


def test_sync_replicas_allreduce_equals_dataparallel():
    assert _spawn(_rank_equiv) == {0: "ok", 1: "ok"}


# ---- 2. checkpoint keys + resume equivalence ------------------------------------------------------------
def _rank_job(rank, world, port, q, ckpt_dir, last_step, out, metrics):
    try:
        _init(rank, world, port)
        import dtg
        from dtg import ops
        from dtg.optim import FusedSGD
        from dtg.parallel import FlatParams, comm
        torch.manual_seed(rank + 7)  # ranks start DIFFERENT: the sync hook must hand them the chief's state
        m = _mlp()
        flat = FlatParams(m, compute_dtype=torch.float32)
        x_ph, y_ph = dtg.placeholder(), dtg.placeholder()
        gs = dtg.train.get_or_create_global_step()
        sro = dtg.train.SyncReplicasOptimizer(dtg.train.MomentumOptimizer(0.05, 0.9), world, world)
        train_op = sro.minimize(lambda x, y: ops.softmax_cross_entropy(m(x), y), global_step=gs,
                                inputs=(x_ph, y_ph), var_list=flat)
        counter = dtg.train.StepCounterHook(every_n_steps=1, batch_size=8, aggregate=True,
                                            metrics_path=metrics if rank == 0 else None)
        hooks = [sro.make_session_run_hook(rank == 0), dtg.train.StopAtStepHook(last_step=last_step), counter]
        first = None
        with dtg.train.MonitoredTrainingSession(is_chief=rank == 0, checkpoint_dir=ckpt_dir, hooks=hooks,
                                                save_checkpoint_secs=None, save_checkpoint_steps=1,
                                                log_step_count_steps=None, save_summaries_steps=None) as sess:
            while not sess.should_stop():
                step = int(sess.run(gs))
                first = step if first is None else first
                x, y = _batch(step, rank)
                sess.run(train_op, feed_dict={x_ph: x, y_ph: y})
        from dtg.train.eager import broadcast_training_state  # noqa: F401 - import check
        for g in flat:  # replicas identical
            t = g.master.clone()
            ts = [torch.empty_like(t) for _ in range(world)]
            torch.distributed.all_gather(ts, t)
            assert all(torch.equal(ts[0], v) for v in ts), g.name
        if rank == 0:
            torch.save({"masters": [g.master.clone() for g in flat],
                        "mom": [g.state["momentum"].clone() for g in flat],
                        "first": first, "gs": int(gs.read_value().item()),
                        "names": [n for n, _ in m.named_parameters()],
                        "history": counter.history}, out)
        comm.shutdown()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_checkpoint_keys_and_resume_equivalence(tmp_path):
    import dtg
    ck, ck_full = str(tmp_path / "ck"), str(tmp_path / "ck_full")
    a, b, full = (str(tmp_path / n) for n in ("a.pt", "b.pt", "full.pt"))
    metrics = str(tmp_path / "metrics.jsonl")
    assert _spawn(_rank_job, ck, 3, a, metrics) == {0: "ok", 1: "ok"}
    ra = torch.load(a, weights_only=True)
    assert ra["first"] == 0 and ra["gs"] == 3
    prefix = dtg.train.latest_checkpoint(ck)
    assert prefix.endswith("model.ckpt-3"), prefix
    keys = set(dtg.train.NewCheckpointReader(prefix).get_variable_to_shape_map())
    names = set(ra["names"])
    assert names <= keys
    assert {n + "/momentum" for n in names} <= keys
    assert {"global_step", "optimizer/step"} <= keys
    assert keys - names - {n + "/momentum" for n in names} <= {"global_step", "optimizer/step", "dtg/slot_layout"}
    # resume to 6
    assert _spawn(_rank_job, ck, 6, b, metrics) == {0: "ok", 1: "ok"}
    rb = torch.load(b, weights_only=True)
    assert rb["first"] == 3 and rb["gs"] == 6
    # uninterrupted 6 steps
    assert _spawn(_rank_job, ck_full, 6, full, str(tmp_path / "m2.jsonl")) == {0: "ok", 1: "ok"}
    rf = torch.load(full, weights_only=True)
    for x, y in zip(rb["masters"] + rb["mom"], rf["masters"] + rf["mom"]):
        assert torch.equal(x, y)
    # the aggregated throughput records
    h = rf["history"]
    assert h and all(r["workers"] == 2 and r["examples/sec/node"] >= r["examples/sec"] > 0 for r in h)
    with open(metrics) as f:
        assert sum(1 for _ in f) >= 2


# ---- 3. graph variables without a PS ----------------------------------------------------------------------
def _rank_graph(rank, world, port, q):
    try:
        _init(rank, world, port)
        import numpy as np
        import dtg
        from dtg.parallel import comm
        a = dtg.Variable(dtg.constant(0., shape=[2]))
        b = dtg.Variable(dtg.constant(0., shape=[2]))
        c = a + b
        gs = dtg.Variable(0, dtype=dtg.int64, trainable=False, name="global_step")
        target = dtg.constant(100. * (rank + 1), shape=[2])
        loss = dtg.reduce_mean(dtg.square(c - target))
        opt = dtg.train.SyncReplicasOptimizer(dtg.train.GradientDescentOptimizer(0.01), world, world)
        train_op = opt.minimize(loss, global_step=gs)
        assert opt.mode == "allreduce"
        with dtg.train.MonitoredTrainingSession(is_chief=rank == 0, hooks=[opt.make_session_run_hook(rank == 0),
                                                dtg.train.StopAtStepHook(last_step=5)]) as sess:
            while not sess.should_stop():
                _, cv, g = sess.run([train_op, c, gs])
        # oracle: mean gradient over the two targets (100, 200): d/da mean((a+b-t)^2) = (a+b-t) per element
        av = np.zeros(2)
        for _ in range(5):
            grad = np.mean([(2 * av - t) for t in (100., 200.)], axis=0)
            av = av - 0.01 * grad
        assert int(g) == 5
        assert np.allclose(a.numpy(), av, rtol=1e-5), (a.numpy(), av)
        comm.shutdown()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_graph_variables_allreduce_mode():
    assert _spawn(_rank_graph) == {0: "ok", 1: "ok"}


# ---- 4. refused combinations (one process, no process group) ----------------------------------------------
def test_allreduce_mode_refuses_backups_and_wrong_replica_count():
    import dtg
    from dtg.optim import FusedSGD
    from dtg.parallel import FlatParams
    dtg.reset_default_graph()
    torch.manual_seed(0)
    m = _mlp()
    flat = FlatParams(m, compute_dtype=torch.float32)
    gs = dtg.train.get_or_create_global_step()
    with pytest.raises(ValueError, match="backup workers"):
        dtg.train.SyncReplicasOptimizer(FusedSGD(flat, lr=0.1), 1, 2).minimize(lambda: m(torch.zeros(1, 16)).sum(),
                                                                                global_step=gs)
    with pytest.raises(ValueError, match="process group has 1"):
        dtg.train.SyncReplicasOptimizer(FusedSGD(flat, lr=0.1), 2, 2).minimize(lambda: m(torch.zeros(1, 16)).sum(),
                                                                                global_step=gs)
    with pytest.raises(TypeError):
        dtg.train.SyncReplicasOptimizer(dtg.train.GradientDescentOptimizer(0.1), 1, 1).minimize(
            lambda: m(torch.zeros(1, 16)).sum(), global_step=gs)


def test_single_replica_session_checkpoint_roundtrip(tmp_path):
    """One process, FusedAdagrad through opt.minimize (no data parallelism): Saver keys, restore on a fresh
    graph, global step and the Adagrad accumulator carried over."""
    import dtg
    from dtg import ops
    from dtg.optim import FusedAdagrad
    from dtg.parallel import FlatParams

    def job(last):
        dtg.reset_default_graph()
        torch.manual_seed(0)
        m = _mlp()
        flat = FlatParams(m, compute_dtype=torch.float32)
        opt = FusedAdagrad(flat, lr=0.05)
        x_ph, y_ph = dtg.placeholder(), dtg.placeholder()
        gs = dtg.train.get_or_create_global_step()
        op = opt.minimize(lambda x, y: ops.softmax_cross_entropy(m(x), y), global_step=gs, inputs=(x_ph, y_ph))
        with dtg.train.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), hooks=[dtg.train.StopAtStepHook(
                last_step=last)], save_checkpoint_secs=None, save_checkpoint_steps=2, log_step_count_steps=None,
                save_summaries_steps=None) as sess:
            while not sess.should_stop():
                s = int(sess.run(gs))
                x, y = _batch(s, 0)
                sess.run(op, feed_dict={x_ph: x, y_ph: y})
        return flat, opt, int(gs.read_value().item())

    _, _, g1 = job(2)
    flat, opt, g2 = job(4)
    assert (g1, g2) == (2, 4) and opt.step_count == 4
    dtg.reset_default_graph()
    torch.manual_seed(0)
    m = _mlp()
    ref = FlatParams(m, compute_dtype=torch.float32)
    ro = FusedAdagrad(ref, lr=0.05)
    for s in range(4):
        x, y = _batch(s, 0)
        ops.softmax_cross_entropy(m(x), y).backward()
        ro.step()
    for a, b in zip(flat, ref):
        assert torch.equal(a.master, b.master) and torch.equal(a.state["acc"], b.state["acc"])


def _clean_env():
    e = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DTG_FAULT"):
        e.pop(k, None)
    return e


def test_bert_train_example_two_ranks_resume(tmp_path):
    """examples/BERT/bert_train.py (tiny config) on 2 gloo ranks: stops at 4, resumes to 6 from the chief's
    checkpoint; the checkpoint holds the AdamW slots under the parameter names."""
    import subprocess
    import dtg
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    ck = str(tmp_path / "ck")
    script = os.path.join(ROOT, "examples", "BERT", "bert_train.py")

    def launch(last):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
               "127.0.0.1", "--master-port", str(free_ports(1)[0]), script, "--tiny", "--batch", "4", "--steps",
               str(last), "--save_every", "2", "--log_every", "2", "--warmup", "2", "--ckpt_dir", ck]
        return subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_clean_env())

    r1 = launch(4)
    assert r1.returncode == 0, r1.stdout + r1.stderr[-3000:]
    assert "done at global step 4" in r1.stdout and "over 2 workers" in r1.stdout, r1.stdout
    r2 = launch(6)
    assert r2.returncode == 0, r2.stdout + r2.stderr[-3000:]
    assert "resumed from" in r2.stdout and "(global step 4)" in r2.stdout and "done at global step 6" in r2.stdout
    rd = dtg.train.NewCheckpointReader(dtg.train.latest_checkpoint(ck))
    keys = set(rd.get_variable_to_shape_map())
    assert int(rd.get_tensor("global_step")) == 6 and int(rd.get_tensor("optimizer/step")) == 6
    assert {"emb.word", "emb.word/m", "emb.word/v", "layers.0.w_qkv/m"} <= keys, sorted(keys)[:20]


def test_mnist_mirrored_example_resume(tmp_path):
    import subprocess
    script = os.path.join(ROOT, "examples", "MNIST", "mnist_mirrored.py")
    ck = str(tmp_path / "ck")
    r1 = subprocess.run([sys.executable, script, "--steps", "60", "--batch", "32", "--ckpt_dir", ck],
                        capture_output=True, text=True, timeout=300, env=_clean_env())
    assert r1.returncode == 0, r1.stderr[-3000:]
    assert "global step 60" in r1.stdout and "images/sec (node)" in r1.stdout
    r2 = subprocess.run([sys.executable, script, "--steps", "80", "--batch", "32", "--ckpt_dir", ck],
                        capture_output=True, text=True, timeout=300, env=_clean_env())
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert "resumed from" in r2.stdout and "global step 80" in r2.stdout, r2.stdout
