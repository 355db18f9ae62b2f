"""DOWNPOUR-Easy on dtg: DOWNPOUR with plain SGD as the local (worker) optimizer.

Each worker keeps local copies of the parameters, takes T = 3 gradient evaluations with local
SGD steps in between (no local optimizer slots, so none of DOWNPOUR's slot bookkeeping), pushes the
SUM of the window's gradients to the PS (global Adagrad step + global_step) and pulls the globals.

Reference: DOWNPOUR-Easy/DOWNPOUR.py:17-139.  The local learning rate is lr * task_index as in the
reference (DOWNPOUR-Easy/DOWNPOUR.py:53), so the chief never updates locally;
the global optimizer is still Adagrad.  Same cluster, lr 1e-4, T = 3, last_step 60, 1 s
checkpoints, prints).  As in the reference's unrolled window, only T-1 local applies execute per
global step: local_step advances by 2 per global step.
Bootstrap: the chief's initial-value push is followed by a PS barrier instead of a 10 s sleep.
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
        server = dtg.train.Server(cluster, job_name='ps', task_index=FLAGS.task_index, config=config)
        server.join()
        return

    is_chief = FLAGS.task_index == 0
    server = dtg.train.Server(cluster, job_name='worker', task_index=FLAGS.task_index, config=config)

    # worker-resident copies of the parameters and the local optimizer
    with dtg.device('/job:worker/replica:0/task:%d' % FLAGS.task_index):
        a = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32,
                         collections=[dtg.GraphKeys.LOCAL_VARIABLES])
        b = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32,
                         collections=[dtg.GraphKeys.LOCAL_VARIABLES])
        c = a + b
        local_step = dtg.Variable(0, dtype=dtg.int32, trainable=False, name='local_step',
                                  collections=['local_non_trainable'])
        lr = .0001
        local_opt = dtg.train.GradientDescentOptimizer(lr * FLAGS.task_index)
        target = dtg.constant(100., shape=[2], dtype=dtg.float32)
        loss = dtg.reduce_mean(dtg.square(c - target))

        window = 3
        grad_list = []
        local_apply = None
        for t in range(window):
            with dtg.control_dependencies([local_apply] if t else []):
                grads, varss = zip(*local_opt.compute_gradients(loss, var_list=dtg.local_variables()))
            grad_list.append(grads)
            local_apply = local_opt.apply_gradients(zip(grads, varss), global_step=local_step)
        window_sum = dtg.reduce_sum(grad_list, axis=0)
        grads = tuple(window_sum[i] for i in range(len(varss)))

    with dtg.device(dtg.train.replica_device_setter(
            ps_tasks=n_pss, worker_device='/job:%s/task:%d' % (FLAGS.job_name, FLAGS.task_index))):
        global_step = dtg.Variable(0, dtype=dtg.int32, trainable=False, name='global_step')
        global_opt = dtg.train.AdagradOptimizer(lr)
        local_to_global, global_to_local = create_global_variables()
        opt = global_opt.apply_gradients(zip(grads, [local_to_global[v] for v in varss]), global_step=global_step)
        with dtg.control_dependencies([opt]):
            assign_locals = pull(global_to_local)
        grab_global_init = pull(global_to_local)
        assign_global = push(local_to_global)
        init = dtg.global_variables_initializer()
        init_local = dtg.variables_initializer(dtg.local_variables() + dtg.get_collection('local_non_trainable'))

    hooks = [dtg.train.StopAtStepHook(last_step=60)]
    scaffold = dtg.train.Scaffold(init_op=init, local_init_op=[init_local])
    logdir = FLAGS.logdir or 'logdir'
    sess = dtg.train.MonitoredTrainingSession(master=server.target, is_chief=is_chief, config=config,
                                              scaffold=scaffold, hooks=hooks, save_checkpoint_secs=1,
                                              checkpoint_dir=logdir)
    if is_chief:
        sess.run(assign_global)  # the chief's initial values become the global ones
    dtg.train.barrier('downpour_easy/bootstrap')

    print('Starting training on worker %d' % FLAGS.task_index)
    sess.run(grab_global_init)
    while not sess.should_stop():
        _, _, r, gs, ls = sess.run([opt, assign_locals, c, global_step, local_step])
        print(r, "global step: " + str(gs), "worker: " + str(FLAGS.task_index), "local step: " + str(ls))
        dtg.flags.sleep(FLAGS, 1)  # so we can observe training
    print('Done', FLAGS.task_index)
    dtg.flags.sleep(FLAGS, 10)
    sess.close()
    print('Session from worker %d closed cleanly' % FLAGS.task_index)


def pull(global_to_local):
    """Op: copy every global (PS) value into its worker-local variable."""
    return dtg.group(*[dtg.assign(local, glob) for glob, local in global_to_local.items()])


def push(local_to_global):
    """Op: copy every worker-local value into its global (PS) variable."""
    return dtg.group(*[dtg.assign(glob, local) for local, glob in local_to_global.items()])


def create_global_variables():
    """A ``g/<name>`` PS mirror of each local variable (names appear as checkpoint keys)."""
    local_to_global, global_to_local = {}, {}
    with dtg.device('/job:ps/task:0'):
        for v in dtg.local_variables():
            g = dtg.get_variable('g/' + v.op.name, shape=v.shape, dtype=v.dtype, trainable=True,
                                 collections=[dtg.GraphKeys.GLOBAL_VARIABLES, dtg.GraphKeys.TRAINABLE_VARIABLES])
            local_to_global[v] = g
            global_to_local[g] = v
    return local_to_global, global_to_local


if __name__ == '__main__':
    FLAGS = dtg.flags.parse()
    print(FLAGS.task_index)
    main()
