"""Local-then-global variables with one worker and one PS.

A worker-local variable `a` (LOCAL_VARIABLES, on /job:worker/task:0) and its global mirror `g/a`
on /job:ps/task:0 (Glorot-random until assigned).  Loss |a - 100| with GD(0.1): a local update
changes only `a` (0 -> 0.1); applying the same local gradients to the global variable moves `g/a`
by exactly +0.1.  Reference notebook: Basics-Tutorial/Local-then-Global-Variables.ipynb:104-181.
Run with Parameter-Server.py in another shell (or via ../Multiple-Workers/run.sh).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))

import dtg  # noqa: E402

FLAGS = dtg.flags.parse()
cluster = dtg.flags.cluster_from(FLAGS, {'worker': ['localhost:2223'], 'ps': ['localhost:2222']})
server = dtg.train.Server(cluster, job_name='worker', task_index=FLAGS.task_index)

with dtg.device('/job:worker/task:%d' % FLAGS.task_index):
    a = dtg.Variable(dtg.constant(0., shape=[1]), name='a', collections=[dtg.GraphKeys.LOCAL_VARIABLES])
    loss = dtg.abs(a - 100.)
    opt = dtg.train.GradientDescentOptimizer(.1)
    grads = opt.compute_gradients(loss, var_list=[a])
    local_update = opt.apply_gradients(grads)
with dtg.device('/job:ps/task:0'):
    a_global = dtg.get_variable('g/a', shape=[1], dtype=dtg.float32)
    global_update = opt.apply_gradients([(g, a_global) for g, _ in grads])

print('global_update placed on', global_update.device.to_string() or a_global.op.device)
print('a_global placed on', a_global.op.device)
sess = dtg.train.Session(server.target)
sess.run([dtg.variables_initializer([a]), dtg.variables_initializer([a_global])])
print('a_global (random init):', sess.run(a_global))
sess.run(local_update)
print('after local update:  a =', sess.run(a), ' a_global =', sess.run(a_global))
before = sess.run(a_global)
sess.run(global_update)
after = sess.run(a_global)
print('after global update: a_global =', after, ' delta =', after - before)
sess.close()
