"""The PS task of the two-worker tutorial; exits once both workers close their sessions."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir, os.pardir))

import dtg  # noqa: E402

flags = dtg.flags.parse()
cluster = dtg.flags.cluster_from(flags, {'ps': ['localhost:2222'], 'worker': ['localhost:2223', 'localhost:2224']})
dtg.train.Server(cluster, job_name='ps', task_index=0).join()
