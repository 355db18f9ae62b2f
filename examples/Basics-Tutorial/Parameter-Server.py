"""A parameter-server task: serves variables until every worker reports done.
Reference notebook: Basics-Tutorial/Parameter-Server.ipynb:29-31 (there join() blocks forever)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))

import dtg  # noqa: E402

FLAGS = dtg.flags.parse()
cluster = dtg.flags.cluster_from(FLAGS, {'worker': ['localhost:2223'], 'ps': ['localhost:2222']})
server = dtg.train.Server(cluster, job_name='ps', task_index=FLAGS.task_index)
print('parameter server listening on', server.target)
server.join()
