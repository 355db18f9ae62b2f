"""Variables: local (worker-resident torch tensors) or remote (owned by a PS task's native
service), with TF-1.x collections, naming and initialisers (SURVEY §2.2 "Local vars + global
mirrors", §2.5 N3/N8/N12, §2.8).

Placement comes from the device stack at creation: a variable placed on a task other than this
process's task (``/job:ps/task:0`` via ``device`` or ``replica_device_setter``) is *remote*;
reading it is a READ on that task's service, assigning is an ASSIGN, applying gradients is an
APPLY executed on the PS (colocated with the variable, as TF does).
"""
import threading

import numpy as np
import torch

from . import graph as G
from .graph import GraphKeys, Node, Op, Tensor
from .placement import DeviceSpec, torch_device

# ------------------------------------------------------------------------------------------------
# connections to task services
# ------------------------------------------------------------------------------------------------
_conns = {}
_conn_lock = threading.Lock()


def _this_server():
    srv = G.get_default_graph().servers
    return srv[-1] if srv else None


def task_address(job, task):
    s = _this_server()
    if s is None:
        raise RuntimeError("no dtg.Server in this process: create one from a ClusterSpec before using "
                           "variables placed on /job:%s/task:%d" % (job, task))
    return s.cluster.task_address(job, task)


def client_for(job, task, timeout=120.0):
    addr = task_address(job, task)
    with _conn_lock:
        c = _conns.get(addr)
        if c is None:
            from . import _runtime
            host, port = addr.rsplit(":", 1)
            c = _runtime.PSClient("127.0.0.1" if host == "localhost" else host, int(port), timeout)
            s = _this_server()
            if s is not None and s.job_name == "worker" and job == "ps":
                # if this worker process dies, the PS counts it as finished instead of joining forever
                c.watch("__worker__", s.task_index)
            _conns[addr] = c
        return c


def new_client(job, task, timeout=120.0):
    """A private connection (not shared through client_for): for a thread that makes long blocking calls
    (the SyncReplicas chief's accumulator waits), so it never holds the shared connection's lock against
    the training thread."""
    from . import _runtime
    host, port = task_address(job, task).rsplit(":", 1)
    return _runtime.PSClient("127.0.0.1" if host == "localhost" else host, int(port), timeout)


def close_connections():
    with _conn_lock:
        for c in _conns.values():
            try:
                c.unwatch()
            except Exception:
                pass
            try:
                c.close()
            except Exception:
                pass
        _conns.clear()


def _is_remote(spec: DeviceSpec):
    if spec.job is None:
        return False
    s = _this_server()
    if s is None:
        return spec.job == "ps"
    task = spec.task if spec.task is not None else 0
    return not (spec.job == s.job_name and task == s.task_index)


_NP = {torch.float32: np.float32, torch.float64: np.float64, torch.int32: np.int32, torch.int64: np.int64}


def _as_np(t):
    t = t.detach()
    if t.dtype == torch.bfloat16:
        t = t.float()
    return np.array(t.cpu().numpy(), order="C", copy=True)  # keeps 0-d shapes (ascontiguousarray does not)


# ------------------------------------------------------------------------------------------------
class _OpRef:
    def __init__(self, v):
        self._v = v

    @property
    def name(self):
        return self._v._name

    @property
    def device(self):
        return self._v.device.to_string()


class Variable(Tensor):
    _is_variable = True
    _no_cache = True

    def __init__(self, initial_value=None, trainable=True, collections=None, name=None, dtype=None, shape=None,
                 validate_shape=True):
        super().__init__(lambda c: None, [], name or "Variable", "Variable")
        self._init = initial_value
        self.dtype = dtype
        self.trainable = trainable
        self.remote = _is_remote(self.device)
        self.ps_task = (self.device.job, self.device.task or 0) if self.remote else None
        self._local = None
        self._initialized = False
        self._lock = threading.Lock()
        init_val = self._initial_tensor(peek=True)
        self.shape = tuple(init_val.shape) if init_val is not None else tuple(shape or ())
        if self.dtype is None:
            self.dtype = init_val.dtype if init_val is not None else torch.float32
        if collections is None:
            collections = [GraphKeys.GLOBAL_VARIABLES]
        if trainable and GraphKeys.TRAINABLE_VARIABLES not in collections:
            collections = list(collections) + [GraphKeys.TRAINABLE_VARIABLES]
        self.collections = list(collections)
        g = G.get_default_graph()
        for c in self.collections:
            g.add_to_collection(c, self)
        g.add_to_collection("_all_variables", self)

    # -- names -------------------------------------------------------------------------------
    @property
    def name(self):
        return self._name + ":0"

    @property
    def op(self):
        return _OpRef(self)

    def get_shape(self):
        return self.shape

    # -- initial value ---------------------------------------------------------------------------
    def _initial_tensor(self, peek=False):
        v = self._init
        if isinstance(v, Node):
            if peek and (v.inputs or v.control_inputs or isinstance(v, Variable)):
                return None
            v = G.RunContext().eval(v)
        if callable(v) and not isinstance(v, torch.Tensor):
            v = v()
        if v is None:
            return None
        t = torch.as_tensor(v if not isinstance(v, np.ndarray) else v.copy())
        if self.dtype is not None and t.dtype != self.dtype:
            t = t.to(self.dtype)
        return t.clone()

    @property
    def compute_device(self):
        return torch_device(self.device)

    # -- storage ----------------------------------------------------------------------------------
    def _client(self):
        return client_for(*self.ps_task)

    def read_value(self):
        """Current value as a torch tensor on the compute device (a PS READ when remote)."""
        if self.remote:
            arr = self._client().read([self._name])[0]
            return torch.from_numpy(arr).to(self.compute_device)
        if self._local is None:
            raise RuntimeError(f"Attempting to use uninitialized value {self._name}")
        return self._local

    def _eval(self, ctx):
        if self in ctx.var_override:
            return ctx.var_override[self]
        return self.read_value()

    def initialize(self):
        t = self._initial_tensor()
        self.load(t, create=True)

    def load(self, value, create=False):
        t = torch.as_tensor(value).to(self.dtype)
        if self.remote:
            if create:
                self._client().create(self._name, _as_np(t), True)
            else:
                self._client().assign([(self._name, _as_np(t))])
        else:
            with self._lock:
                if self._local is None or self._local.shape != t.shape:
                    self._local = t.to(self.compute_device).clone()
                else:
                    self._local.copy_(t.to(self._local.device))
        self._initialized = True

    def is_initialized(self):
        if self.remote:
            return bool(self._client().is_init([self._name])[0])
        return self._local is not None

    @property
    def initializer(self):
        return Op(lambda c: self.initialize(), [], self._name + "/Assign")

    def assign(self, value, name=None):
        return assign(self, value, name)

    def assign_add(self, delta, name=None):
        return assign_add(self, delta, name)

    def value(self):
        return self

    def numpy(self):
        return G.to_numpy(self.read_value())


class _RefVariable(Variable):
    pass


# ------------------------------------------------------------------------------------------------
def assign(ref, value, name=None):
    value = G.convert_to_tensor(value)

    def run(ctx, v):
        t = v.detach() if isinstance(v, torch.Tensor) else torch.as_tensor(v)
        ref.load(t)
        return t

    return Op(run, [value], name or (ref._name + "/Assign"))


def assign_add(ref, delta, name=None):
    delta = G.convert_to_tensor(delta)

    def run(ctx, d):
        d = torch.as_tensor(d).to(ref.dtype)
        if ref.remote:
            out = ref._client().assign_add(ref._name, _as_np(d))
            return torch.from_numpy(out)
        with ref._lock:
            ref._local.add_(d.to(ref._local.device))
            return ref._local.clone()

    return Op(run, [delta], name or (ref._name + "/AssignAdd"))


def global_variables():
    return G.get_collection(GraphKeys.GLOBAL_VARIABLES)


def local_variables():
    return G.get_collection(GraphKeys.LOCAL_VARIABLES)


def trainable_variables():
    return G.get_collection(GraphKeys.TRAINABLE_VARIABLES)


def all_variables():
    return G.get_collection("_all_variables")


def variables_initializer(var_list, name="init"):
    vl = list(var_list)
    return Op(lambda c: [v.initialize() for v in vl] and None, [], name)


def global_variables_initializer():
    return variables_initializer(global_variables(), "init")


def local_variables_initializer():
    return variables_initializer(local_variables(), "init_1")


def report_uninitialized_variables(var_list=None, name="report_uninitialized_variables"):
    def run(ctx):
        vl = global_variables() if var_list is None else list(var_list)
        return np.array([v._name for v in vl if not v.is_initialized()], dtype=object)

    return Tensor(run, [], name)


def is_variable_initialized(v):
    return Tensor(lambda c: v.is_initialized(), [], v._name + "/IsVariableInitialized")


def glorot_uniform_initializer(seed=None):
    def init(shape, dtype=torch.float32):
        shape = tuple(shape)
        if len(shape) == 0:
            fan_in = fan_out = 1
        elif len(shape) == 1:
            fan_in = fan_out = shape[0]
        else:
            rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
            fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
        lim = float(np.sqrt(6.0 / (fan_in + fan_out)))
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        return (torch.rand(shape, generator=g, dtype=torch.float64) * 2 * lim - lim).to(dtype)
    return init


def truncated_normal(shape, mean=0.0, stddev=1.0, dtype=torch.float32, seed=None):
    """TF TruncatedNormal: resample values beyond 2 stddev (Non-Distributed_Setup.py:13)."""
    g = torch.Generator().manual_seed(seed) if seed is not None else None
    shape = (shape,) if isinstance(shape, int) else tuple(shape)
    t = torch.empty(shape, dtype=torch.float64)
    torch.nn.init.trunc_normal_(t, 0.0, 1.0, -2.0, 2.0, generator=g)
    return (t * stddev + mean).to(dtype)


def zeros_initializer():
    return lambda shape, dtype=torch.float32: torch.zeros(tuple(shape), dtype=dtype)


def constant_initializer(value=0.0):
    return lambda shape, dtype=torch.float32: torch.full(tuple(shape), value, dtype=dtype)


def get_variable(name, shape=None, dtype=torch.float32, initializer=None, trainable=True, collections=None):
    """TF get_variable: exact name (no uniquifying), default Glorot-uniform initializer
    (Local-then-Global-Variables.ipynb:117-123 -> random -1.26 at :222)."""
    g = G.get_default_graph()
    for v in G.get_collection("_all_variables"):
        if v._name == name:
            return v
    init = initializer or (glorot_uniform_initializer() if dtype.is_floating_point else zeros_initializer())
    shp = tuple(shape) if shape is not None else ()
    v = Variable(lambda: init(shp, dtype), trainable=trainable, collections=collections, name=name, dtype=dtype,
                 shape=shp)
    # get_variable names are exact: undo the uniquifier's suffix if one was applied
    v._name = name
    return v
