"""AEASGD / AEAMSGD (asynchronous elastic-averaging SGD, Zhang, Choromanska & LeCun 2015) on dtg --
listed as TODO in the reference (README.md:40-42, paper link README.md:99), built here on the same
toy problem and script conventions as its DOWNPOUR/ADAG examples.

Each worker keeps a local replica (a, b) trained by local SGD (``--momentum > 0``: AEAMSGD); every
``--tau`` local steps it couples to the center variable (g/a, g/b) on the PS:
    d = alpha * (local - center);  local -= d;  center += d        (one exchange = one global step)
The center update is an unlocked assign_add on the PS, so concurrent workers race like Hogwild.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))

import dtg  # noqa: E402

FLAGS = None
CLUSTER = {'ps': ['localhost:2222'], 'worker': ['localhost:2223', 'localhost:2224']}


def main():
    cluster = dtg.flags.cluster_from(FLAGS, CLUSTER)
    if FLAGS.job_name == 'ps':
        dtg.train.Server(cluster, job_name='ps', task_index=FLAGS.task_index).join()
        return
    is_chief = FLAGS.task_index == 0
    server = dtg.train.Server(cluster, job_name='worker', task_index=FLAGS.task_index)

    with dtg.device('/job:worker/replica:0/task:%d' % FLAGS.task_index):
        a = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32, collections=[dtg.GraphKeys.LOCAL_VARIABLES])
        b = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32, collections=[dtg.GraphKeys.LOCAL_VARIABLES])
        c = a + b
        target = dtg.constant(100., shape=[2], dtype=dtg.float32)
        loss = dtg.reduce_mean(dtg.square(c - target))
        if FLAGS.momentum > 0:
            local_opt = dtg.train.MomentumOptimizer(FLAGS.lr, FLAGS.momentum)
        else:
            local_opt = dtg.train.GradientDescentOptimizer(FLAGS.lr)
        local_train = local_opt.minimize(loss, var_list=[a, b])

    with dtg.device('/job:ps/task:0'):
        global_step = dtg.Variable(0, dtype=dtg.int32, trainable=False, name='global_step')
        center = {v: dtg.get_variable('g/' + v.op.name, shape=v.shape, dtype=v.dtype,
                                      collections=[dtg.GraphKeys.GLOBAL_VARIABLES]) for v in (a, b)}
    # elastic exchange: the differences are evaluated once per run (read local and center first)
    diffs = {v: FLAGS.alpha * (v - g) for v, g in center.items()}
    with dtg.control_dependencies(list(diffs.values())):
        exchange = dtg.group(*([dtg.assign(v, v - d) for v, d in diffs.items()] +
                               [dtg.assign_add(center[v], d) for v, d in diffs.items()] +
                               [dtg.assign_add(global_step, 1)]))
    assign_center = dtg.group(*[dtg.assign(g, v) for v, g in center.items()])
    grab_center = dtg.group(*[dtg.assign(v, g) for v, g in center.items()])
    init_local = dtg.variables_initializer(dtg.local_variables())
    init = dtg.global_variables_initializer()

    hooks = [dtg.train.StopAtStepHook(last_step=FLAGS.last_step)]
    scaffold = dtg.train.Scaffold(init_op=init, local_init_op=init_local)
    sess = dtg.train.MonitoredTrainingSession(master=server.target, is_chief=is_chief, scaffold=scaffold,
                                              hooks=hooks, checkpoint_dir=FLAGS.logdir or None)
    if is_chief:
        sess.run(assign_center)
    dtg.train.barrier('aeasgd/bootstrap')
    sess.run(grab_center)
    print('Starting training on worker %d' % FLAGS.task_index)
    step = 0
    while not sess.should_stop():
        sess.run(local_train)
        step += 1
        if step % FLAGS.tau == 0:
            _, r, gs = sess.run([exchange, c, global_step])
            print(r, "global step: " + str(gs), "worker: " + str(FLAGS.task_index), "local step: " + str(step))
        dtg.flags.sleep(FLAGS, .1)
    print('center', sess.run([center[a] + center[b]])[0], 'worker', FLAGS.task_index)
    print('Done', FLAGS.task_index)
    sess.close()


def _extra(p):
    p.add_argument('--tau', type=int, default=3, help='local steps between elastic exchanges')
    p.add_argument('--alpha', type=float, default=0.5, help='elastic coupling (moving rate)')
    p.add_argument('--lr', type=float, default=0.1)
    p.add_argument('--momentum', type=float, default=0.0, help='> 0: AEAMSGD (momentum local optimizer)')
    p.add_argument('--last_step', type=int, default=10, help='number of elastic exchanges (global steps)')


if __name__ == '__main__':
    FLAGS = dtg.flags.parse(extra=_extra)
    main()
