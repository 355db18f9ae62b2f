"""Distributed "hello world" on dtg: 1 PS + 1 worker, MonitoredTrainingSession, no checkpoints.

Reference: Distributed-Setup/dist_setup.py:17-57.  The reference leaves placement to TF's placer
(bare /cpu:0); dtg places the variables on the PS with replica_device_setter,
which is the intent (the PS holds the shared parameters).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))

import dtg  # noqa: E402

FLAGS = None
CLUSTER = {'ps': ['localhost:2222'], 'worker': ['localhost:2223']}


def main():
    cluster = dtg.flags.cluster_from(FLAGS, CLUSTER)
    if FLAGS.job_name == 'ps':
        server = dtg.train.Server(cluster, job_name='ps', task_index=FLAGS.task_index)
        server.join()
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
        opt = dtg.train.GradientDescentOptimizer(.0001).minimize(loss)

    sess = dtg.train.MonitoredTrainingSession(master=server.target, is_chief=is_chief)
    for i in range(FLAGS.steps):
        if sess.should_stop():
            break
        sess.run(opt)
        if i % 10 == 0:
            r = sess.run(c)
            print(r)
        dtg.flags.sleep(FLAGS, .1)
    sess.close()


def _extra(p):
    p.add_argument('--steps', type=int, default=1000)


if __name__ == '__main__':
    FLAGS = dtg.flags.parse(extra=_extra)
    main()
