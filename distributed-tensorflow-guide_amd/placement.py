"""Device strings, ``device()`` stacking and ``replica_device_setter``.

Device strings follow the reference: ``/job:<ps|worker>/replica:0/task:<i>/<cpu|gpu>:<k>``
(DOWNPOUR/DOWNPOUR.py:45, Synchronous-SGD/ssgd.py:38, Servers.ipynb:246).  A variable whose
resolved device names a task other than this process's own task is *remote*: it lives in that
task's native PS service.  ``replica_device_setter`` round-robins variables over the PS tasks and
puts everything else on the worker device (TF's placer semantics, DOWNPOUR/DOWNPOUR.py:86-87).
"""
import re

import torch

_RE = re.compile(r"/?(job|replica|task|device|cpu|gpu|CPU|GPU)[:]([^/]+)")


class DeviceSpec:
    __slots__ = ("job", "replica", "task", "device_type", "device_index")

    def __init__(self, job=None, replica=None, task=None, device_type=None, device_index=None):
        self.job, self.replica, self.task = job, replica, task
        self.device_type, self.device_index = device_type, device_index

    @staticmethod
    def from_string(s):
        d = DeviceSpec()
        if not s:
            return d
        for k, v in _RE.findall(s):
            kl = k.lower()
            if kl == "job":
                d.job = v
            elif kl == "replica":
                d.replica = int(v)
            elif kl == "task":
                d.task = int(v)
            elif kl == "device":
                typ, _, idx = v.partition(":")
                d.device_type = typ.lower()
                d.device_index = int(idx) if idx and idx != "*" else 0
            else:  # cpu:0 / gpu:1
                d.device_type = kl
                d.device_index = int(v) if v != "*" else 0
        return d

    def merged_over(self, base):
        """self's set fields override base's."""
        out = DeviceSpec(base.job, base.replica, base.task, base.device_type, base.device_index)
        for f in self.__slots__:
            v = getattr(self, f)
            if v is not None:
                setattr(out, f, v)
        return out

    def to_string(self):
        parts = []
        if self.job is not None:
            parts.append(f"/job:{self.job}")
        if self.replica is not None:
            parts.append(f"/replica:{self.replica}")
        if self.task is not None:
            parts.append(f"/task:{self.task}")
        if self.device_type is not None:
            parts.append(f"/device:{self.device_type.upper()}:{self.device_index or 0}")
        return "".join(parts)

    def __repr__(self):
        return self.to_string() or "''"

    def __eq__(self, o):
        return isinstance(o, DeviceSpec) and all(getattr(self, f) == getattr(o, f) for f in self.__slots__)

    __hash__ = object.__hash__


class _ReplicaDeviceChooser:
    def __init__(self, ps_tasks, ps_device, worker_device, merge_devices, ps_strategy):
        self.ps_tasks = ps_tasks
        self.ps_device = ps_device
        self.worker_device = worker_device
        self.merge_devices = merge_devices
        self.ps_strategy = ps_strategy or _RoundRobin(ps_tasks)

    def __call__(self, node):
        if getattr(node, "_is_variable", False) and self.ps_tasks > 0:
            spec = DeviceSpec.from_string(self.ps_device)
            if spec.task is None:
                spec.task = self.ps_strategy(node)
            return spec.to_string()
        return self.worker_device or ""


class _RoundRobin:
    def __init__(self, n):
        self.n = max(1, n)
        self.next = 0

    def __call__(self, node):
        t = self.next
        self.next = (self.next + 1) % self.n
        return t


def replica_device_setter(ps_tasks=0, ps_device="/job:ps", worker_device="/job:worker", merge_devices=True,
                          cluster=None, ps_ops=None, ps_strategy=None):
    """Variables -> PS tasks (round robin), everything else -> ``worker_device``."""
    if cluster is not None and ps_tasks == 0:
        from .cluster import ClusterSpec
        ps_tasks = ClusterSpec(cluster).num_tasks("ps")
    return _ReplicaDeviceChooser(ps_tasks, ps_device, worker_device, merge_devices, ps_strategy)


def resolve_device(stack, node=None):
    spec = DeviceSpec()
    for entry in stack:
        if entry is None:
            spec = DeviceSpec()
            continue
        s = entry(node) if callable(entry) else entry
        spec = DeviceSpec.from_string(s).merged_over(spec)
    return spec


def torch_device(spec, default="cpu"):
    """Compute device for a (local) DeviceSpec: /gpu:k -> cuda:k if available."""
    if spec is not None and spec.device_type == "gpu" and torch.cuda.is_available():
        n = torch.cuda.device_count()
        return torch.device("cuda", (spec.device_index or 0) % max(1, n))
    return torch.device(default)


def place_tasks_on_gpus(cluster, job, task, visible=None):
    """SURVEY §5.6 device mapping: ps task k -> GPU k; worker i -> GPU n_ps + i (unless the
    process already sees a single GPU through HIP_VISIBLE_DEVICES, as the reference's .sh does)."""
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if n == 0:
        return torch.device("cpu")
    if n == 1:
        return torch.device("cuda", 0)
    n_ps = cluster.num_tasks("ps")
    idx = task if job == "ps" else n_ps + task
    return torch.device("cuda", idx % n)
