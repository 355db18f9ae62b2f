"""SDAG (synchronous distributed adaptive gradients, WIP in the reference) on dtg.

A "window" of T = 5 gradient evaluations is averaged and applied synchronously through
SyncReplicasOptimizer.  As in the reference there is no local update between the window's
evaluations, so the T gradients are identical and the run equals plain SSGD.
Reference: SDAG/dist_cpu_sing_mach_sync.py:16-117 (lr 1e-4, R = 2 of 2, last_step 10, hand-wired
Scaffold, chief runs init_tokens_op explicitly, prints ``r, gs, i``; the chief prints twice).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))

import dtg  # noqa: E402

FLAGS = None
REPLICAS_TO_AGGREGATE = 2
CLUSTER = {'ps': ['localhost:2222'], 'worker': ['localhost:2223', 'localhost:2224']}


def main():
    config = dtg.ConfigProto(log_device_placement=False)
    cluster = dtg.flags.cluster_from(FLAGS, CLUSTER)
    if FLAGS.job_name == 'ps':
        dtg.train.Server(cluster, job_name='ps', task_index=FLAGS.task_index, config=config).join()
        return
    is_chief = FLAGS.task_index == 0
    server = dtg.train.Server(cluster, job_name='worker', task_index=FLAGS.task_index, config=config)
    n_workers = cluster.num_tasks('worker')
    replicas = min(REPLICAS_TO_AGGREGATE, n_workers)

    with dtg.device(dtg.train.replica_device_setter(ps_tasks=cluster.num_tasks('ps'),
                                                    worker_device='/job:worker/task:%d/cpu:0' % FLAGS.task_index)):
        a = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32)
        b = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32)
        c = a + b
        global_step = dtg.Variable(0, dtype=dtg.int32, trainable=False, name='global_step')
        target = dtg.constant(100., shape=[2], dtype=dtg.float32)
        loss = dtg.reduce_mean(dtg.square(c - target))

        base = dtg.train.GradientDescentOptimizer(.0001)
        sync_opt = dtg.train.SyncReplicasOptimizer(base, replicas_to_aggregate=replicas,
                                                   total_num_replicas=n_workers)
        window = 5
        grad_list = []
        for _ in range(window):
            grads, varss = zip(*sync_opt.compute_gradients(loss))
            grad_list.append(grads)
        mean = dtg.reduce_mean(grad_list, axis=0)
        opt = sync_opt.apply_gradients(zip([mean[i] for i in range(len(varss))], varss), global_step=global_step)

    sync_hook = sync_opt.make_session_run_hook(is_chief, num_tokens=FLAGS.init_tokens)
    init_tokens_op = sync_opt.get_init_tokens_op()
    local_init = sync_opt.chief_init_op if is_chief else sync_opt.local_step_init_op
    scaffold = dtg.train.Scaffold(init_op=dtg.global_variables_initializer(), local_init_op=local_init,
                                  ready_for_local_init_op=sync_opt.ready_for_local_init_op)
    sess = dtg.train.MonitoredTrainingSession(master=server.target, is_chief=is_chief, config=config,
                                              scaffold=scaffold,
                                              hooks=[sync_hook, dtg.train.StopAtStepHook(last_step=10)],
                                              stop_grace_period_secs=10)
    if is_chief and FLAGS.init_tokens != 0:
        sess.run(init_tokens_op)
    dtg.train.barrier('sdag/bootstrap')

    print('Starting training on worker %d' % FLAGS.task_index)
    while not sess.should_stop():
        _, r, gs = sess.run([opt, c, global_step])
        print(r, gs, FLAGS.task_index)
        if is_chief:
            print(r, gs, FLAGS.task_index)
            dtg.flags.sleep(FLAGS, 1)  # the chief paces an extra second (SDAG/dist_cpu_sing_mach_sync.py:111)
        dtg.flags.sleep(FLAGS, 1)
    print('Done', FLAGS.task_index)
    dtg.flags.sleep(FLAGS, 10)
    sess.close()
    print('Session from worker %d closed cleanly' % FLAGS.task_index)


if __name__ == '__main__':
    FLAGS = dtg.flags.parse()
    print(FLAGS.task_index)
    main()
