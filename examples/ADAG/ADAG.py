"""ADAG (asynchronous distributed adaptive gradients) on dtg.

Like DOWNPOUR but with local SGD inside the T = 3 window, the window gradients AVERAGED (not
summed) and a global SGD step on the PS.  Reference: ADAG/ADAG.py:15-135 (lr 1e-4 local and
global, last_step 40, debug print of the window gradients when gs % 7 == 1 -- which re-runs the
window, exactly as the reference's extra sess.run does).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))

import dtg  # noqa: E402

FLAGS = None
CLUSTER = {'ps': ['localhost:2222'], 'worker': ['localhost:2223', 'localhost:2224']}


def main():
    config = dtg.ConfigProto(log_device_placement=False)
    cluster = dtg.flags.cluster_from(FLAGS, CLUSTER)
    n_pss = cluster.num_tasks('ps')
    if FLAGS.job_name == 'ps':
        dtg.train.Server(cluster, job_name='ps', task_index=FLAGS.task_index, config=config).join()
        return

    is_chief = FLAGS.task_index == 0
    server = dtg.train.Server(cluster, job_name='worker', task_index=FLAGS.task_index, config=config)

    with dtg.device('/job:worker/replica:0/task:%d' % FLAGS.task_index):
        a = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32,
                         collections=[dtg.GraphKeys.LOCAL_VARIABLES])
        b = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32,
                         collections=[dtg.GraphKeys.LOCAL_VARIABLES])
        c = a + b
        local_step = dtg.Variable(0, dtype=dtg.int32, trainable=False, name='local_step',
                                  collections=['local_non_trainable'])

    with dtg.device(dtg.train.replica_device_setter(
            ps_tasks=n_pss, worker_device='/job:%s/task:%d' % (FLAGS.job_name, FLAGS.task_index))):
        global_step = dtg.Variable(0, dtype=dtg.int32, trainable=False, name='global_step')
        target = dtg.constant(100., shape=[2], dtype=dtg.float32)
        loss = dtg.reduce_mean(dtg.square(c - target))
        lr = .0001
        local_opt = dtg.train.GradientDescentOptimizer(lr)
        global_opt = dtg.train.GradientDescentOptimizer(lr)
        local_to_global, global_to_local = create_global_variables()

        window = 3
        grad_list = []
        local_apply = None
        for t in range(window):
            with dtg.control_dependencies([local_apply] if t else []):
                grads, varss = zip(*local_opt.compute_gradients(loss, var_list=dtg.local_variables()))
            grad_list.append(grads)
            local_apply = local_opt.apply_gradients(zip(grads, varss), global_step=local_step)
        mean = dtg.reduce_mean(grad_list, axis=0)
        grads = tuple(mean[i] for i in range(len(varss)))
        opt = global_opt.apply_gradients(zip(grads, [local_to_global[v] for v in varss]), global_step=global_step)
        with dtg.control_dependencies([opt]):
            assign_locals = pull(global_to_local)
        init_local = dtg.variables_initializer(dtg.local_variables() + dtg.get_collection('local_non_trainable'))
        init = dtg.global_variables_initializer()
        grab_global_init = pull(global_to_local)
        assign_global = push(local_to_global)

    hooks = [dtg.train.StopAtStepHook(last_step=40)]
    scaffold = dtg.train.Scaffold(init_op=init, local_init_op=init_local)
    sess = dtg.train.MonitoredTrainingSession(master=server.target, is_chief=is_chief, config=config,
                                              scaffold=scaffold, hooks=hooks, save_checkpoint_secs=1,
                                              checkpoint_dir=FLAGS.logdir or 'logdir')
    if is_chief:
        sess.run(assign_global)
    dtg.train.barrier('adag/bootstrap')

    print('Starting training on worker %d' % FLAGS.task_index)
    sess.run(grab_global_init)
    while not sess.should_stop():
        _, _, r, gs, ls = sess.run([opt, assign_locals, c, global_step, local_step])
        print(r, "global step: " + str(gs), "worker: " + str(FLAGS.task_index), "local step: " + str(ls))
        if gs % 7 == 1 and getattr(FLAGS, 'debug_window', 1):
            for j in grad_list:
                print(sess.run(j), FLAGS.task_index)
        dtg.flags.sleep(FLAGS, 1)
    print('Done', FLAGS.task_index)
    dtg.flags.sleep(FLAGS, 10)
    sess.close()
    print('Session from worker %d closed cleanly' % FLAGS.task_index)


def pull(global_to_local):
    return dtg.group(*[dtg.assign(local, glob) for glob, local in global_to_local.items()])


def push(local_to_global):
    return dtg.group(*[dtg.assign(glob, local) for local, glob in local_to_global.items()])


def create_global_variables():
    local_to_global, global_to_local = {}, {}
    with dtg.device('/job:ps/task:0'):
        for v in dtg.local_variables():
            g = dtg.get_variable('g/' + v.op.name, shape=v.shape, dtype=v.dtype, trainable=True,
                                 collections=[dtg.GraphKeys.GLOBAL_VARIABLES, dtg.GraphKeys.TRAINABLE_VARIABLES])
            local_to_global[v], global_to_local[g] = g, v
    return local_to_global, global_to_local


def _extra(p):
    p.add_argument('--debug_window', type=int, default=1, help='print the window gradients when gs % 7 == 1')


if __name__ == '__main__':
    FLAGS = dtg.flags.parse(extra=_extra)
    print(FLAGS.task_index)
    main()
