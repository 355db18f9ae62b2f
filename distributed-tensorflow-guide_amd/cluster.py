"""ClusterSpec / Server: the task-addressing layer of the reference.

``Server(cluster, job_name, task_index)`` starts dtg's native C++ service (csrc/ps/server.cc) on
the task's ``host:port``: it is the variable store + apply engine for variables placed on that
task (TF's gRPC master/worker services).  ``server.join()`` blocks until every
worker has reported done (or a shutdown request) -- unlike the reference's PS, which never exits
and has to be ``pkill``-ed (README.md:55-59).

Reference call sites: Hogwild/Hogwild.py:20-33, DOWNPOUR/DOWNPOUR.py:24-41,
Basics-Tutorial/Servers.ipynb:68-89 (target), :153-162 (server_def), :198 (create_local_server).
"""
import json
import os


class ClusterSpec:
    """Dict-compatible job -> [host:port, ...] map (tf.train.ClusterSpec)."""

    def __init__(self, cluster):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.as_dict()
        if isinstance(cluster, str):
            cluster = json.loads(cluster)
        self._spec = {}
        for job, tasks in cluster.items():
            if isinstance(tasks, dict):
                n = max(tasks) + 1 if tasks else 0
                lst = [None] * n
                for k, v in tasks.items():
                    lst[int(k)] = v
                tasks = lst
            self._spec[job] = list(tasks)

    @property
    def jobs(self):
        return list(self._spec)

    def as_dict(self):
        return {j: list(t) for j, t in self._spec.items()}

    def num_tasks(self, job):
        return len(self._spec.get(job, []))

    def job_tasks(self, job):
        return list(self._spec[job])

    def task_indices(self, job):
        return list(range(self.num_tasks(job)))

    def task_address(self, job, index):
        return self._spec[job][index]

    def __getitem__(self, job):
        return self._spec[job]

    def __contains__(self, job):
        return job in self._spec

    def __eq__(self, other):
        return isinstance(other, ClusterSpec) and self.as_dict() == other.as_dict()

    def __repr__(self):
        return "ClusterSpec(%r)" % (self._spec,)

    @staticmethod
    def from_env(default=None, env="DTG_CLUSTER"):
        """Cluster from ``$DTG_CLUSTER`` (JSON) if set, else ``default`` (the script's literal)."""
        v = os.environ.get(env)
        return ClusterSpec(json.loads(v)) if v else ClusterSpec(default)


def split_address(addr):
    host, port = addr.rsplit(":", 1)
    return host, int(port)


class Server:
    """An in-process task server.  Starts the native PS service on this task's address."""

    def __init__(self, server_or_cluster_def, job_name=None, task_index=0, protocol="dtg", config=None,
                 start=True, num_workers=None):
        self.cluster = ClusterSpec(server_or_cluster_def)
        if job_name is None:
            job_name = self.cluster.jobs[0]
        self.job_name = job_name
        self.task_index = int(task_index)
        self.protocol = protocol
        self.config = config
        self.address = self.cluster.task_address(job_name, self.task_index)
        host, port = split_address(self.address)
        from . import _runtime
        nw = self.cluster.num_tasks("worker") if num_workers is None else num_workers
        # only parameter servers wait for worker completion in join(); workers' services exit with them
        self._svc = _runtime.PSServer(host if host != "localhost" else "127.0.0.1", port,
                                      nw if job_name == "ps" else 0)
        self._started = False
        if start:
            self.start()
        from . import graph
        graph._register_server(self)

    def start(self):
        if not self._started:
            self._svc.start()
            self._started = True
            if self.address.endswith(":0"):  # ephemeral port: publish the real one
                host = self.address.rsplit(":", 1)[0]
                self.address = "%s:%d" % (host, self._svc.port)
                self.cluster._spec[self.job_name][self.task_index] = self.address

    @property
    def target(self):
        return "dtg://" + self.address

    @property
    def server_def(self):
        return {"cluster": {"job": [{"name": j, "tasks": dict(enumerate(t))} for j, t in self.cluster.as_dict().items()]},
                "job_name": self.job_name, "task_index": self.task_index, "protocol": self.protocol}

    @property
    def service(self):
        return self._svc

    def join(self, timeout=None):
        """Block until all workers reported done (PS) or shutdown was requested.

        With ``DTG_FAULT=kill_ps_at_step:N`` (tests only, dtg/fault.py) a PS dies abruptly once its
        ``global_step`` reaches N."""
        from . import fault
        kill_at = fault.kill_ps_step() if self.job_name == "ps" else None
        if kill_at is not None:
            import os
            import time
            t_end = None if timeout is None else time.time() + float(timeout)
            while t_end is None or time.time() < t_end:
                if self._svc.join(0.05):
                    self._svc.stop()
                    return True
                try:
                    gs = int(self._svc.read_var("global_step").reshape(-1)[0])
                except Exception:  # not created yet
                    gs = -1
                if gs >= kill_at:
                    print("[dtg.fault] killing ps task %d at global_step %d" % (self.task_index, gs), flush=True)
                    os._exit(fault.KILL_EXIT_CODE)
            return False
        done = self._svc.join(-1.0 if timeout is None else float(timeout))
        if done:
            self._svc.stop()
        return done

    def stop(self):
        self._svc.stop()

    @staticmethod
    def create_local_server(config=None, start=True):
        """Single-task in-process server on an ephemeral localhost port (Servers.ipynb:198)."""
        return Server(ClusterSpec({"localhost": ["127.0.0.1:0"]}), "localhost", 0, config=config, start=start)

    def __repr__(self):
        return "Server(%s, job=%s, task=%d)" % (self.target, self.job_name, self.task_index)
