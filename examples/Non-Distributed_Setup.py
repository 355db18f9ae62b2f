"""Single-process baseline on dtg: the toy problem c = a + b -> 100 with SGD (lr 1e-4).

Reference: Non-Distributed_Setup.py:10-30 (truncated-normal init, 1000 iterations, prints c
every 10 steps, 0.1 s sleep per step).  No cluster: variables are local, the Supervisor has no
logdir.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dtg  # noqa: E402

FLAGS = None


def main():
    with dtg.device('/cpu:0'):
        a = dtg.Variable(dtg.truncated_normal(shape=[2]), dtype=dtg.float32)
        b = dtg.Variable(dtg.truncated_normal(shape=[2]), dtype=dtg.float32)
        c = a + b
        target = dtg.constant(100., shape=[2], dtype=dtg.float32)
        loss = dtg.reduce_mean(dtg.square(c - target))
        opt = dtg.train.GradientDescentOptimizer(.0001).minimize(loss)

    sv = dtg.train.Supervisor()
    sess = sv.prepare_or_wait_for_session()
    for i in range(FLAGS.steps):
        if sv.should_stop():
            break
        sess.run(opt)
        if i % 10 == 0:
            print(sess.run(c))
        dtg.flags.sleep(FLAGS, .1)
    return sess.run(c)


def _extra(p):
    p.add_argument('--steps', type=int, default=1000)


if __name__ == '__main__':
    FLAGS = dtg.flags.parse(extra=_extra)
    main()
