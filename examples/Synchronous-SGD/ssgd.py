"""Synchronous SGD through SyncReplicasOptimizer (PS-accumulator mode) on dtg.

Variables live on the PS (replica_device_setter); each step the chief aggregates
REPLICAS_TO_AGGREGATE gradients (their mean) in the PS's conditional accumulators, applies them and
hands out sync tokens.  With more workers than replicas to aggregate, the surplus gradients are
backups and get dropped.  Reference: Synchronous-SGD/ssgd.py:15-81 (lr 1e-4, R = 2 of 2,
StopAtStepHook(10), prints ``r, 'step: ', gs, 'worker: ', i``).
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

    worker_device = '/job:%s/task:%d/cpu:0' % (FLAGS.job_name, FLAGS.task_index)
    with dtg.device(dtg.train.replica_device_setter(ps_tasks=1, worker_device=worker_device)):
        a = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32)
        b = dtg.Variable(dtg.constant(0., shape=[2]), dtype=dtg.float32)
        c = a + b
        global_step = dtg.Variable(0, dtype=dtg.int32, trainable=False, name='global_step')
        target = dtg.constant(100., shape=[2], dtype=dtg.float32)
        loss = dtg.reduce_mean(dtg.square(c - target))

        base = dtg.train.GradientDescentOptimizer(.0001)
        sync_opt = dtg.train.SyncReplicasOptimizer(base, replicas_to_aggregate=replicas,
                                                   total_num_replicas=n_workers)
        opt = sync_opt.minimize(loss, global_step=global_step)  # the PS averages the replicas

    hooks = [sync_opt.make_session_run_hook(is_chief, num_tokens=FLAGS.init_tokens),
             dtg.train.StopAtStepHook(last_step=10)]
    sess = dtg.train.MonitoredTrainingSession(master=server.target, is_chief=is_chief, config=config, hooks=hooks,
                                              stop_grace_period_secs=10)

    print('Starting training on worker %d' % FLAGS.task_index)
    while not sess.should_stop():
        _, r, gs = sess.run([opt, c, global_step])
        print(r, 'step: ', gs, 'worker: ', FLAGS.task_index)
        if is_chief:
            dtg.flags.sleep(FLAGS, 1)
        dtg.flags.sleep(FLAGS, 1)
    print('Done', FLAGS.task_index)
    dtg.flags.sleep(FLAGS, 10)
    sess.close()
    print('Session from worker %d closed cleanly' % FLAGS.task_index)


if __name__ == '__main__':
    FLAGS = dtg.flags.parse()
    print(FLAGS.task_index)
    main()
