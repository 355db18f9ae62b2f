"""Servers: a cluster with one task, its target and server_def, a session on it, and a local server.
Reference notebook: Basics-Tutorial/Servers.ipynb (cells at :68-89, :153, :180, :198, :246)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), os.pardir, os.pardir))

import dtg  # noqa: E402

FLAGS = dtg.flags.parse()
cluster = dtg.flags.cluster_from(FLAGS, {'worker': ['localhost:2222']})
server = dtg.train.Server(cluster, job_name='worker', task_index=0)
print(server.target)            # dtg://localhost:2222  (the reference: grpc://localhost:2222)
print(server.server_def)
sess = dtg.train.Session(target=server.target)
print(sess.list_devices())
local = dtg.train.Server.create_local_server()
print(local.target)
local.stop()
server.stop()
