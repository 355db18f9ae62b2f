"""Semantics of the deferred dataflow graph, variables and sessions (single process, no PS)."""
import numpy as np
import pytest
import torch

import dtg


@pytest.fixture(autouse=True)
def fresh_graph():
    dtg.reset_default_graph()
    yield
    dtg.reset_default_graph()


def test_each_fetch_evaluated_once_per_run():
    calls = []
    a = dtg.Variable(torch.zeros(2))
    t = dtg.Tensor(lambda c, x: calls.append(1) or x + 1, [a], "count")
    u = t * 2
    s = dtg.train.Session()
    s.run(a.initializer)
    r = s.run([t, u, t])
    assert len(calls) == 1 and np.allclose(r[1], 2)


def test_control_dependencies_and_unused_ops_not_run():
    a = dtg.Variable(torch.zeros(()), collections=[dtg.GraphKeys.LOCAL_VARIABLES])
    inc1 = dtg.assign_add(a, 1.0)
    with dtg.control_dependencies([inc1]):
        read = dtg.identity(a)
    dtg.assign_add(a, 100.0)  # nothing depends on it: never executed
    s = dtg.train.Session()
    s.run(dtg.local_variables_initializer())
    assert float(s.run(read)) == 1.0
    assert float(s.run(read)) == 2.0  # runs again in the next run


def test_window_unroll_executes_t_minus_1_local_applies():
    """DOWNPOUR/ADAG unrolled window: the last local apply has no consumer."""
    a = dtg.Variable(dtg.constant(0., shape=[2]), collections=[dtg.GraphKeys.LOCAL_VARIABLES])
    step = dtg.Variable(0, dtype=dtg.int32, trainable=False, collections=["local_non_trainable"])
    loss = dtg.reduce_mean(dtg.square(a - 100.))
    opt = dtg.train.GradientDescentOptimizer(1e-3)
    grad_list, app = [], None
    for t in range(3):
        with dtg.control_dependencies([app] if t else []):
            gv = opt.compute_gradients(loss, var_list=[a])
        grad_list.append([g for g, _ in gv])
        app = opt.apply_gradients(gv, global_step=step)
    total = dtg.reduce_sum(grad_list, axis=0)
    s = dtg.train.Session()
    s.run(dtg.variables_initializer([a, step]))
    s.run(total)
    assert int(s.run(step)) == 2


def test_gradients_match_autograd():
    w = dtg.Variable(torch.tensor([1.0, -2.0, 3.0]))
    x = dtg.constant([0.5, 0.25, 2.0])
    loss = dtg.reduce_sum(dtg.square(w * x))
    (g, v), = dtg.train.GradientDescentOptimizer(0.1).compute_gradients(loss)
    s = dtg.train.Session()
    s.run(w.initializer)
    np.testing.assert_allclose(s.run(g), 2 * np.array([1.0, -2.0, 3.0]) * np.array([0.5, 0.25, 2.0]) ** 2)


@pytest.mark.parametrize("opt_cls,kw", [(dtg.train.GradientDescentOptimizer, {}),
                                        (dtg.train.AdagradOptimizer, {}),
                                        (dtg.train.MomentumOptimizer, {"momentum": 0.9}),
                                        (dtg.train.AdamOptimizer, {})])
def test_local_optimizers_decrease_loss(opt_cls, kw):
    w = dtg.Variable(torch.tensor([5.0, -3.0]))
    loss = dtg.reduce_sum(dtg.square(w))
    train = opt_cls(0.1, **kw).minimize(loss)
    s = dtg.train.Session()
    s.run(w.initializer)
    l0 = float(s.run(loss))
    for _ in range(20):
        s.run(train)
    assert float(s.run(loss)) < l0


def test_non_distributed_sgd_gap_factor():
    a = dtg.Variable(torch.tensor([1.0, 2.0]))
    b = dtg.Variable(torch.tensor([3.0, -1.0]))
    c = a + b
    loss = dtg.reduce_mean(dtg.square(c - 100.))
    gs = dtg.train.get_or_create_global_step()
    opt = dtg.train.GradientDescentOptimizer(1e-4).minimize(loss, global_step=gs)
    sess = dtg.train.MonitoredTrainingSession(hooks=[dtg.train.StopAtStepHook(last_step=1000)])
    c0 = sess.run(c)
    while not sess.should_stop():
        sess.run(opt)
    c1 = sess.run(c)
    np.testing.assert_allclose((100 - c1) / (100 - c0), 0.9998 ** 1000, rtol=1e-4)
    assert int(sess.run(gs)) == 1000
    sess.close()


def test_mts_checkpoint_and_restore(tmp_path):
    w = dtg.Variable(torch.tensor([1.0, 2.0]), name="w")
    gs = dtg.train.get_or_create_global_step()
    train = dtg.train.GradientDescentOptimizer(0.5).minimize(dtg.reduce_sum(dtg.square(w)), global_step=gs)
    d = str(tmp_path / "ckpt")
    sess = dtg.train.MonitoredTrainingSession(checkpoint_dir=d, save_checkpoint_steps=2,
                                              hooks=[dtg.train.StopAtStepHook(last_step=5)])
    while not sess.should_stop():
        sess.run(train)
    sess.close()
    saved = dtg.train.NewCheckpointReader(dtg.train.latest_checkpoint(d))
    assert int(saved.get_tensor("global_step")) == 5
    w5 = saved.get_tensor("w")
    # restore into a fresh graph
    dtg.reset_default_graph()
    w2 = dtg.Variable(torch.tensor([9.0, 9.0]), name="w")
    dtg.train.get_or_create_global_step()
    s2 = dtg.train.MonitoredTrainingSession(checkpoint_dir=d, save_checkpoint_secs=None)
    np.testing.assert_allclose(s2.run(w2), w5)
    assert s2.restored_from is not None
    s2.close()


def test_hooks_surface():
    w = dtg.Variable(torch.tensor([1.0]))
    gs = dtg.train.get_or_create_global_step()
    loss = dtg.reduce_sum(dtg.square(w))
    train = dtg.train.GradientDescentOptimizer(0.1).minimize(loss, global_step=gs)
    final = dtg.train.FinalOpsHook(loss)
    counter = dtg.train.StepCounterHook(every_n_steps=1, batch_size=32)
    sess = dtg.train.MonitoredTrainingSession(hooks=[dtg.train.StopAtStepHook(num_steps=4), final, counter,
                                                     dtg.train.NanTensorHook(loss),
                                                     dtg.train.LoggingTensorHook({"loss": loss}, every_n_iter=2)])
    while not sess.should_stop():
        sess.run(train)
    sess.close()
    assert final.final_ops_values is not None and counter.history and "examples/sec" in counter.history[-1]


def test_graph_def_text_proto(tmp_path):
    import dtg
    from dtg import graph as G
    G.reset_default_graph()
    with dtg.device("/job:ps/task:0"):
        a = dtg.Variable([1.0, 2.0], name="a")
    with dtg.device("/job:worker/task:0"):
        b = dtg.constant(3.0)
        with dtg.control_dependencies([a.initializer]):
            c = a * b
    gd = G.get_default_graph().as_graph_def()
    txt = str(gd)
    assert 'name: "a"\n  op: "VariableV2"' in txt and "dim { size: 2 }" in txt and 'device: "/job:ps/task:0"' in txt
    assert 'name: "mul"\n  op: "Mul"\n  input: "a"\n  input: "Const"\n  input: "^a/Assign"' in txt
    path = dtg.train.write_graph(gd, str(tmp_path), "graph.pbtxt")
    assert open(path).read() == txt and txt.endswith("versions {\n  producer: 24\n}\n")
    assert [n.name for n in G.get_default_graph().get_operations()][:2] == ["a:0", "Const:0"]
    G.reset_default_graph()
