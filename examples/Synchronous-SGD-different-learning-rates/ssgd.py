"""Synchronous SGD with a different learning rate per worker, on dtg.

The sync optimizer runs with base_lr = 1.0 and each worker pre-scales its gradients by
(lr_i / base_lr) * replicas, so the PS's mean over the replicas becomes the weighted SUM
sum_i lr_i * g_i.  Worker 0 uses lr 0.1, the others 1e-4.  The Scaffold is wired
by hand (chief_init_op / local_step_init_op / ready_for_local_init_op) and the chief also runs the
init-tokens op explicitly -- as the reference does, giving the workers one extra step of run-ahead
(SURVEY App. B #8).  Reference: Synchronous-SGD-different-learning-rates/ssgd.py:14-107.
The chief's 40 s warm-up sleep is replaced by a PS barrier.
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

        base_lr = 1.0
        base = dtg.train.GradientDescentOptimizer(base_lr)
        sync_opt = dtg.train.SyncReplicasOptimizer(base, replicas_to_aggregate=replicas,
                                                   total_num_replicas=n_workers)
        my_lr = .1 if FLAGS.task_index == 0 else .0001
        scale = (my_lr / base_lr) * replicas  # undo the PS mean: sum_i lr_i * g_i
        grads_and_vars = sync_opt.compute_gradients(loss)
        scaled = [(g * scale, v) for g, v in grads_and_vars]
        opt = sync_opt.apply_gradients(scaled, global_step=global_step)

    sync_hook = sync_opt.make_session_run_hook(is_chief, num_tokens=FLAGS.init_tokens)
    init_tokens_op = sync_opt.get_init_tokens_op()
    local_init = sync_opt.chief_init_op if is_chief else sync_opt.local_step_init_op
    scaffold = dtg.train.Scaffold(init_op=dtg.global_variables_initializer(), local_init_op=local_init,
                                  ready_for_local_init_op=sync_opt.ready_for_local_init_op)
    hooks = [sync_hook, dtg.train.StopAtStepHook(last_step=10)]
    sess = dtg.train.MonitoredTrainingSession(master=server.target, is_chief=is_chief, config=config,
                                              scaffold=scaffold, hooks=hooks, stop_grace_period_secs=10)
    if is_chief and FLAGS.extra_init_tokens and FLAGS.init_tokens != 0:
        sess.run(init_tokens_op)  # the reference's explicit (second) token initialisation
    dtg.train.barrier('ssgd_lr/bootstrap')

    print('Starting training on worker %d' % FLAGS.task_index)
    while not sess.should_stop():
        _, r, gs = sess.run([opt, c, global_step])
        print(r, 'step: ', gs, 'worker: ', FLAGS.task_index)
        if is_chief:
            dtg.flags.sleep(FLAGS, 1)  # the chief paces an extra second (ssgd.py:101 of the reference)
        dtg.flags.sleep(FLAGS, 1)
    print('Done', FLAGS.task_index)
    dtg.flags.sleep(FLAGS, 10)
    sess.close()
    print('Session from worker %d closed cleanly' % FLAGS.task_index)


def _extra(p):
    p.add_argument('--extra_init_tokens', type=int, default=1,
                   help='reproduce the reference chief running init_tokens_op a second time')


if __name__ == '__main__':
    FLAGS = dtg.flags.parse(extra=_extra)
    print(FLAGS.task_index)
    main()
