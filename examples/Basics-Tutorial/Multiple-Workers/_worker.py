"""Shared body of the two Multiple-Workers scripts: two workers update ONE variable on the PS.

Worker 1 (task 0) initialises its local `a` and the global `g/a`, takes a local step, then a global
step (+0.1); worker 2 (task 1) initialises only its local variable, sees worker 1's value, applies
its own global step (+0.1); worker 1 then re-reads +0.2 in total.  Reference notebooks:
Basics-Tutorial/Multiple-Workers/Local-then-Global-Variables-Worker1.ipynb:205-322 and -Worker2.ipynb:205-286
(the recorded sequence -1.17584 -> -1.07584 -> -0.97584).  PS barriers order the two scripts the
way the notebook author ordered the cells by hand.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir, os.pardir))

import dtg  # noqa: E402


def run(task_index, argv=None):
    flags = dtg.flags.parse(argv)
    cluster = dtg.flags.cluster_from(flags, {'ps': ['localhost:2222'], 'worker': ['localhost:2223', 'localhost:2224']})
    server = dtg.train.Server(cluster, job_name='worker', task_index=task_index)
    with dtg.device('/job:worker/task:%d' % task_index):
        a = dtg.Variable(dtg.constant(0., shape=[1]), name='a', collections=[dtg.GraphKeys.LOCAL_VARIABLES])
        loss = dtg.abs(a - 100.)
        opt = dtg.train.GradientDescentOptimizer(.1)
        grads = opt.compute_gradients(loss, var_list=[a])
        local_update = opt.apply_gradients(grads)
    with dtg.device('/job:ps/task:0'):
        a_global = dtg.get_variable('g/a', shape=[1], dtype=dtg.float32)
        global_update = opt.apply_gradients([(g, a_global) for g, _ in grads])
    sess = dtg.train.Session(server.target)
    if task_index == 0:
        sess.run([dtg.variables_initializer([a]), dtg.variables_initializer([a_global])])
        print('a_global init:', sess.run(a_global))
        sess.run(local_update)
        print('local a:', sess.run(a))
        sess.run(global_update)
        print('a_global after worker 1 update:', sess.run(a_global))
        dtg.train.barrier('w1_updated')          # worker 2 may go
        dtg.train.barrier('w2_updated')          # wait for worker 2's update
        print('a_global after worker 2 update:', sess.run(a_global))
    else:
        dtg.train.barrier('w1_updated')
        sess.run(dtg.variables_initializer([a]))  # local only: the global one is shared
        print('a_global seen by worker 2:', sess.run(a_global))
        sess.run(global_update)
        print('a_global after worker 2 update:', sess.run(a_global))
        dtg.train.barrier('w2_updated')
    sess.close()
