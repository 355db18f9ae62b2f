"""Asynchronous data parallelism with one GPU per worker process, PS on the CPU.

The launcher gives each worker its own GPU through HIP_VISIBLE_DEVICES (the PS gets none); inside
the worker the compute runs on /gpu:0 of what it can see (its own MI355X), gradients go to the PS
which applies them (Hogwild-style).  Reference: Multiple-GPUs-Single-Machine/
dist_mult_gpu_sing_mach.py:14-57 -- which does not parse (mixed tabs/spaces, ``config`` used
before assignment); this is its intent.  Falls back to the CPU when no GPU is
visible, so the example also runs in CPU-only CI.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))

import dtg  # noqa: E402

FLAGS = None
CLUSTER = {'ps': ['localhost:2222'], 'worker': ['localhost:2223', 'localhost:2224']}


def main():
    config = dtg.ConfigProto(log_device_placement=False, allow_soft_placement=True,
                             gpu_options=dtg.GPUOptions(allow_growth=True, allocator_type="BFC",
                                                        visible_device_list="0"))
    cluster = dtg.flags.cluster_from(FLAGS, CLUSTER)
    if FLAGS.job_name == 'ps':
        dtg.train.Server(cluster, job_name='ps', task_index=FLAGS.task_index, config=config).join()
        return
    is_chief = FLAGS.task_index == 0
    server = dtg.train.Server(cluster, job_name='worker', task_index=FLAGS.task_index, config=config)

    with dtg.device(dtg.train.replica_device_setter(ps_tasks=cluster.num_tasks('ps'),
                                                    worker_device='/job:worker/task:%d/gpu:0' % FLAGS.task_index)):
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
    sess = sv.prepare_or_wait_for_session(server.target, config=config)
    print('worker %d computes on %s' % (FLAGS.task_index, config.hip_device()))
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
