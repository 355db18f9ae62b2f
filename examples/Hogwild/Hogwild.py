"""Hogwild! on dtg: lock-free asynchronous SGD from 2 workers on parameters held by 1 PS.

Each worker's apply runs on the PS without locking (use_locking=False): the PS service updates
elements with relaxed atomic loads/stores, so concurrent workers can overwrite each other's
updates -- the algorithm's intended race, free of undefined behaviour.
Reference: Hogwild/Hogwild.py:18-57 (lr 1e-4, 1000 steps/worker, Supervisor with 30 s
checkpoints, print c every 10 steps, 0.1 s sleep).  The reference's bare /cpu:0 placement is
ambiguous; dtg puts the shared parameters on the PS, which is the intent.
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

    with dtg.device(dtg.train.replica_device_setter(ps_tasks=cluster.num_tasks('ps'),
                                                    worker_device='/job:worker/task:%d/cpu:0' % FLAGS.task_index)):
        a = dtg.Variable(dtg.truncated_normal(shape=[2]), dtype=dtg.float32)
        b = dtg.Variable(dtg.truncated_normal(shape=[2]), dtype=dtg.float32)
        c = a + b
        target = dtg.constant(100., shape=[2], dtype=dtg.float32)
        loss = dtg.reduce_mean(dtg.square(c - target))
        # no global step, as in the reference (minimize(loss) only): the Supervisor's checkpoints are plain
        # `model.ckpt` files holding just Variable and Variable_1
        opt = dtg.train.GradientDescentOptimizer(.0001).minimize(loss)

    logdir = FLAGS.logdir or os.path.join(os.getcwd(), 'logdir')
    sv = dtg.train.Supervisor(logdir=logdir, is_chief=is_chief, save_model_secs=30)
    sess = sv.prepare_or_wait_for_session(server.target)
    for i in range(FLAGS.steps):
        if sv.should_stop():
            break
        sess.run(opt)
        if i % 10 == 0:
            print(sess.run(c))
        dtg.flags.sleep(FLAGS, .1)
    sv.stop()


def _extra(p):
    p.add_argument('--steps', type=int, default=1000)


if __name__ == '__main__':
    FLAGS = dtg.flags.parse(extra=_extra)
    main()
