"""A minimal deferred dataflow graph with TF-1.x run semantics, executed eagerly by PyTorch.

The reference's scripts build a TF graph once and then call ``sess.run(fetches)`` repeatedly
(e.g. DOWNPOUR/DOWNPOUR.py:43-137).  To keep that programming model -- and its exact semantics --
dtg provides symbolic :class:`Tensor` / :class:`Op` nodes:

* every fetch is evaluated at most once per ``run`` (a per-run memo cache), so ``c``, the
  gradients and the apply of one step all see the same variable snapshot;
* ``control_dependencies`` adds ordering edges: a node first evaluates its control inputs;
* ``compute_gradients`` is a node whose evaluation runs the loss forward on leaf copies of the
  variables and differentiates with torch.autograd;
* variables placed on a parameter-server task are read through the native PS service once per run
  (``Variable``, variables.py), and applies run on the PS (colocated with the variable, as in TF).

Side-effecting nodes that nothing depends on are simply never executed, which reproduces
reference behaviours such as the T-1 local applies of the DOWNPOUR/ADAG windows
without special-casing them.
"""
import contextlib
import itertools
import threading
from collections import defaultdict

import numpy as np
import torch


class GraphKeys:
    GLOBAL_VARIABLES = "variables"
    LOCAL_VARIABLES = "local_variables"
    TRAINABLE_VARIABLES = "trainable_variables"
    MODEL_VARIABLES = "model_variables"
    GLOBAL_STEP = "global_step"
    SUMMARIES = "summaries"
    UPDATE_OPS = "update_ops"
    INIT_OP = "init_op"
    LOCAL_INIT_OP = "local_init_op"
    READY_OP = "ready_op"
    SAVERS = "savers"
    QUEUE_RUNNERS = "queue_runners"


# ------------------------------------------------------------------------------------------------
# default graph: names, collections, device / control-dependency stacks
# ------------------------------------------------------------------------------------------------
class Graph:
    def __init__(self):
        self._names = defaultdict(int)
        self._collections = defaultdict(list)
        self._device_stack = []
        self._control_stack = []
        self._name_stack = []
        self._lock = threading.RLock()
        self.servers = []
        self._nodes = []  # every node in creation order (as_graph_def / write_graph)

    def unique_name(self, base, mark_used=True):
        scope = "/".join(self._name_stack)
        full = f"{scope}/{base}" if scope else base
        with self._lock:
            n = self._names[full]
            if mark_used:
                self._names[full] += 1
        return full if n == 0 else f"{full}_{n}"

    def add_to_collection(self, key, value):
        self._collections[key].append(value)

    def get_collection(self, key):
        return list(self._collections.get(key, []))

    def get_collection_ref(self, key):
        return self._collections[key]

    def clear_collection(self, key):
        self._collections[key] = []

    @contextlib.contextmanager
    def device(self, spec):
        self._device_stack.append(spec)
        try:
            yield
        finally:
            self._device_stack.pop()

    @contextlib.contextmanager
    def control_dependencies(self, deps):
        if deps is None:  # tf semantics: clear
            saved, self._control_stack = self._control_stack, []
            try:
                yield
            finally:
                self._control_stack = saved
            return
        self._control_stack.append([d for d in deps if d is not None])
        try:
            yield
        finally:
            self._control_stack.pop()

    @contextlib.contextmanager
    def name_scope(self, name):
        self._name_stack.append(name)
        try:
            yield name
        finally:
            self._name_stack.pop()

    def current_control_inputs(self):
        return list(itertools.chain.from_iterable(self._control_stack))

    def current_device(self, node=None):
        from .placement import resolve_device
        return resolve_device(self._device_stack, node)

    def get_operations(self):
        return list(self._nodes)

    def as_graph_def(self, add_shapes=False):
        """The graph as a TF ``GraphDef`` (text-proto serialisable, ``str(graph_def)``)."""
        return GraphDef(self._nodes, add_shapes)


_default = Graph()


def get_default_graph():
    return _default


def reset_default_graph():
    global _default
    _default = Graph()
    return _default


def _register_server(server):
    _default.servers.append(server)


def add_to_collection(key, value):
    _default.add_to_collection(key, value)


def get_collection(key):
    return _default.get_collection(key)


def get_collection_ref(key):
    return _default.get_collection_ref(key)


def control_dependencies(deps):
    return _default.control_dependencies(deps)


def name_scope(name):
    return _default.name_scope(name)


def device(spec):
    """``with dtg.device('/job:ps/task:0')`` or ``with dtg.device(replica_device_setter(...))``."""
    return _default.device(spec)


# ------------------------------------------------------------------------------------------------
# run context
# ------------------------------------------------------------------------------------------------
class RunContext:
    """Per-``run`` evaluation state: memo cache + the session that owns the connections."""

    def __init__(self, session=None, feed_dict=None):
        self.session = session
        self.cache = {}
        self.feed = dict(feed_dict or {})
        self.var_override = {}  # Variable -> leaf tensor while differentiating

    def eval(self, x):
        if isinstance(x, Node):
            if x in self.feed:
                return _to_torch(self.feed[x])
            key = id(x)
            if key not in self.cache:
                for c in x.control_inputs:
                    self.eval(c)
                v = x._eval(self)
                if x._no_cache:  # variable reads happen each time they execute (after control deps)
                    return v
                self.cache[key] = v
            return self.cache[key]
        if isinstance(x, (list, tuple)):
            return type(x)(self.eval(v) for v in x)
        if isinstance(x, dict):
            return {k: self.eval(v) for k, v in x.items()}
        return x


_tls = threading.local()


def _to_torch(v):
    if isinstance(v, torch.Tensor):
        return v
    return torch.as_tensor(np.asarray(v))


def to_numpy(v):
    if isinstance(v, torch.Tensor):
        v = v.detach()
        if v.dtype == torch.bfloat16:
            v = v.float()
        a = v.cpu().numpy()
        return a
    if isinstance(v, (list, tuple)):
        return type(v)(to_numpy(x) for x in v)
    if isinstance(v, dict):
        return {k: to_numpy(x) for k, x in v.items()}
    return v


# ------------------------------------------------------------------------------------------------
# nodes
# ------------------------------------------------------------------------------------------------
class Node:
    _is_op = False
    _no_cache = False

    def __init__(self, fn, inputs=(), name=None, kind="Tensor"):
        g = get_default_graph()
        self._name = g.unique_name(name or kind)
        self._fn = fn
        self.inputs = list(inputs)
        self.control_inputs = g.current_control_inputs()
        self.device = g.current_device(self)
        self.op_type = _op_type(name or kind, kind)
        g._nodes.append(self)

    # TF-compat: t.name == 'add:0', t.op.name == 'add'
    @property
    def name(self):
        return self._name if self._is_op else self._name + ":0"

    @property
    def op(self):
        return _NodeOpRef(self)

    def _eval(self, ctx):
        return self._fn(ctx, *[ctx.eval(i) for i in self.inputs])

    def eval(self, session=None, feed_dict=None):
        ctx = RunContext(session, feed_dict)
        return to_numpy(ctx.eval(self))

    def __repr__(self):
        return f"<dtg.{type(self).__name__} '{self.name}' device={self.device}>"

    __hash__ = object.__hash__


# TF op type of a node, from the base name its constructor was given (graph.pbtxt)
_OP_TYPES = {"add": "Add", "sub": "Sub", "mul": "Mul", "truediv": "RealDiv", "pow": "Pow", "strided_slice": "StridedSlice",
             "group_deps": "NoOp", "init": "NoOp", "init_1": "NoOp", "Op": "NoOp", "Tensor": "Identity",
             "Variable": "VariableV2"}


def _op_type(base, kind):
    if kind == "Variable":
        return "VariableV2"
    b = base.rsplit("/", 1)[-1]
    if b in _OP_TYPES:
        return _OP_TYPES[b]
    return "".join(p[:1].upper() + p[1:] for p in b.split("_") if p) or "NoOp"


def _tf_dtype(dt):
    return {torch.float32: "DT_FLOAT", torch.float64: "DT_DOUBLE", torch.int32: "DT_INT32", torch.int64: "DT_INT64",
            torch.bfloat16: "DT_BFLOAT16", torch.float16: "DT_HALF", torch.bool: "DT_BOOL"}.get(dt, "DT_FLOAT")


def _q(s):
    return '"' + str(s).replace("\\", "\\\\").replace('"', '\\"') + '"'


class GraphDef:
    """``tf.GraphDef`` of a dtg graph: one ``node`` per graph node (name, TF op type, data inputs, ``^control``
    inputs, device; dtype/shape attrs on variables).  ``str()`` is the text proto TF writes as graph.pbtxt
    (DOWNPOUR/DOWNPOUR.py:121-127 gets one from MonitoredTrainingSession's checkpoint_dir)."""

    def __init__(self, nodes, add_shapes=False):
        self.node = list(nodes)
        self.add_shapes = add_shapes

    def _node_text(self, n):
        lines = ["node {", f"  name: {_q(n._name)}", f"  op: {_q(n.op_type)}"]
        for i in n.inputs:
            if isinstance(i, Node):
                lines.append(f"  input: {_q(i._name)}")
        for c in n.control_inputs:
            if isinstance(c, Node):
                lines.append(f"  input: {_q('^' + c._name)}")
        dev = n.device.to_string() if getattr(n, "device", None) is not None else ""
        if dev:
            lines.append(f"  device: {_q(dev)}")
        if getattr(n, "_is_variable", False):
            dims = " ".join(f"dim {{ size: {int(d)} }}" for d in n.shape)
            lines.append(f"  attr {{ key: \"dtype\" value {{ type: {_tf_dtype(n.dtype)} }} }}")
            lines.append(f"  attr {{ key: \"shape\" value {{ shape {{ {dims} }} }} }}")
        lines.append("}")
        return "\n".join(lines)

    def __str__(self):
        return "\n".join([self._node_text(n) for n in self.node] + ["versions {", "  producer: 24", "}"]) + "\n"

    def SerializeToString(self):  # noqa: N802 - tf name (text form; TF's binary proto is not reproduced)
        return str(self).encode()


def write_graph(graph_or_graph_def, logdir, name, as_text=True):
    """tf.train.write_graph: <logdir>/<name> as a GraphDef text proto."""
    import os
    gd = graph_or_graph_def.as_graph_def() if isinstance(graph_or_graph_def, Graph) else graph_or_graph_def
    os.makedirs(logdir, exist_ok=True)
    path = os.path.join(logdir, name)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(str(gd))
    os.replace(tmp, path)
    return path


class _NodeOpRef:
    def __init__(self, n):
        self._n = n

    @property
    def name(self):
        return self._n._name

    @property
    def device(self):
        return self._n.device.to_string()


class Tensor(Node):
    """A symbolic value.  Arithmetic builds new nodes; evaluation happens inside ``run``."""

    def __add__(self, o): return _binop(torch.add, self, o, "add")
    def __radd__(self, o): return _binop(torch.add, o, self, "add")
    def __sub__(self, o): return _binop(torch.sub, self, o, "sub")
    def __rsub__(self, o): return _binop(torch.sub, o, self, "sub")
    def __mul__(self, o): return _binop(torch.mul, self, o, "mul")
    def __rmul__(self, o): return _binop(torch.mul, o, self, "mul")
    def __truediv__(self, o): return _binop(torch.div, self, o, "truediv")
    def __rtruediv__(self, o): return _binop(torch.div, o, self, "truediv")
    def __neg__(self): return Tensor(lambda c, a: -a, [self], "Neg")
    def __pow__(self, p): return _binop(torch.pow, self, p, "pow")
    def __getitem__(self, idx): return Tensor(lambda c, a: a[idx], [self], "strided_slice")


class Op(Node):
    """A side-effecting node (apply / assign / group); evaluates to None unless it returns a value."""
    _is_op = True

    def __init__(self, fn, inputs=(), name=None):
        super().__init__(fn, inputs, name, "Op")

    def __call__(self, session=None):  # handy for eager use
        return self.eval(session)


def _const_node(v):
    if isinstance(v, Node):
        return v
    t = _to_torch(v) if not isinstance(v, (int, float)) else v
    return Tensor(lambda c: t, [], "Const")


def _binop(f, a, b, name):
    return Tensor(lambda c, x, y: f(x, y), [_const_node(a), _const_node(b)], name)


def convert_to_tensor(v):
    return _const_node(v)


def constant(value, shape=None, dtype=torch.float32, name="Const"):
    t = torch.as_tensor(value, dtype=dtype)
    if shape is not None:
        t = t.expand(*([shape] if isinstance(shape, int) else shape)).clone()
    return Tensor(lambda c: t, [], name)


def placeholder(dtype=None, shape=None, name="Placeholder"):
    """tf.placeholder: a value supplied through ``feed_dict`` at run time.  Fed torch tensors are used as they
    are (a GPU batch stays on the GPU), so an eager train step (dtg.train.eager) takes its batch this way."""
    def run(ctx):
        raise ValueError("You must feed a value for placeholder tensor '%s'" % t._name)
    t = Tensor(run, [], name)
    t.dtype, t.shape = dtype, shape
    return t


def no_op(name="NoOp"):
    return Op(lambda c: None, [], name)


def group(*ops, name="group_deps"):
    flat = []
    for o in ops:
        flat.extend(o if isinstance(o, (list, tuple)) else [o])
    return Op(lambda c, *a: None, flat, name)


def identity(x, name="Identity"):
    return Tensor(lambda c, a: a, [_const_node(x)], name)


# ---- math -------------------------------------------------------------------------------------
def _unary(f, name):
    def op(x, name_=None):
        return Tensor(lambda c, a: f(a), [_const_node(x)], name_ or name)
    return op


square = _unary(torch.square, "Square")
abs = _unary(torch.abs, "Abs")  # noqa: A001 - tf name
sqrt = _unary(torch.sqrt, "Sqrt")
exp = _unary(torch.exp, "Exp")
log = _unary(torch.log, "Log")
relu = _unary(torch.relu, "Relu")
tanh = _unary(torch.tanh, "Tanh")


def _reduce(f, name):
    def op(x, axis=None, keepdims=False, name_=None):
        def run(c, a):
            if isinstance(a, (list, tuple)):
                a = torch.stack([torch.stack(list(e)) if isinstance(e, (list, tuple)) else e for e in a])
            if axis is None:
                return f(a)
            return f(a, dim=axis, keepdim=keepdims)
        xs = x if isinstance(x, (list, tuple)) else [x]
        if isinstance(x, (list, tuple)):
            return _ListReduce(run, x, name_ or name)
        return Tensor(run, [_const_node(xs[0])], name_ or name)
    return op


class _ListReduce(Tensor):
    """reduce_* over a python list of per-window gradient tuples (DOWNPOUR/DOWNPOUR.py:77)."""

    def __init__(self, run, lst, name):
        self._run = run
        self._lst = lst
        super().__init__(lambda c: None, [], name)

    def _eval(self, ctx):
        vals = ctx.eval(self._lst)
        return self._run(ctx, vals)

    def __getitem__(self, i):
        return Tensor(lambda c, a: a[i], [self], "strided_slice")


reduce_mean = _reduce(torch.mean, "Mean")
reduce_sum = _reduce(torch.sum, "Sum")
reduce_max = _reduce(torch.amax, "Max")


def matmul(a, b, name="MatMul"):
    return Tensor(lambda c, x, y: x @ y, [_const_node(a), _const_node(b)], name)


def as_fetch(x):
    return x
