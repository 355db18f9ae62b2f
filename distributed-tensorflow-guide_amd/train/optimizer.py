"""Graph-mode optimizers (tf.train.*Optimizer equivalents).

``compute_gradients`` returns (gradient node, variable) pairs; ``apply_gradients`` returns an Op
that, when run, applies every gradient where its variable lives:
  * local variables are updated in-process (torch, on the worker's compute device), with
    optimizer slots (Adagrad accumulators, momenta) kept next to them;
  * remote variables are updated ON the parameter server by one batched APPLY request per PS
    task (the native apply loop of csrc/ps/server.cc), which also bumps ``global_step`` when it is
    colocated -- exactly TF's placement of ApplyGradientDescent/ApplyAdagrad with the variable
    (SURVEY §2.5 N4/N5).  ``use_locking=False`` (the TF default) gives Hogwild semantics.
"""
from collections import defaultdict

from .. import fault

import numpy as np
import torch

from .. import graph as G
from ..graph import Node, Op, Tensor
from ..variables import Variable, _as_np, trainable_variables


class _Gradients(Node):
    """Evaluates d(loss)/d(var) for a var list in one backward pass."""

    def __init__(self, loss, var_list):
        super().__init__(lambda c: None, [], "gradients")
        self.loss = loss
        self.var_list = list(var_list)

    def _eval(self, ctx):
        leaves = {}
        for v in self.var_list:
            val = v.read_value() if not isinstance(v, torch.Tensor) else v
            leaf = val.detach().clone()
            if not leaf.is_floating_point():
                leaf = leaf.float()
            leaves[v] = leaf.requires_grad_(True)
        sub = G.RunContext(ctx.session, ctx.feed)
        sub.var_override = leaves
        loss = sub.eval(self.loss)
        if not isinstance(loss, torch.Tensor):
            loss = torch.as_tensor(loss)
        grads = torch.autograd.grad(loss, [leaves[v] for v in self.var_list], allow_unused=True)
        return [g if g is not None else torch.zeros_like(leaves[v]) for g, v in zip(grads, self.var_list)]


class _GradSlice(Tensor):
    def __init__(self, grads, i):
        self._src = grads
        self._i = i
        super().__init__(lambda c, gs: gs[i], [grads], "gradients/grad")


class Optimizer:
    PS_KIND = 0  # _runtime.SGD

    def __init__(self, learning_rate, use_locking=False, name="Optimizer"):
        self._lr = learning_rate
        self._use_locking = use_locking
        self._name = name
        self._slots = defaultdict(dict)
        self._t = 0

    # -- graph construction ------------------------------------------------------------------
    def compute_gradients(self, loss, var_list=None, **kw):
        vl = list(var_list) if var_list is not None else trainable_variables()
        if not vl:
            raise ValueError("No variables to optimize.")
        node = _Gradients(loss, vl)
        return [(_GradSlice(node, i), v) for i, v in enumerate(vl)]

    def apply_gradients(self, grads_and_vars, global_step=None, name=None):
        gv = [(g, v) for g, v in grads_and_vars]
        return _ApplyOp(self, gv, global_step, name or self._name)

    def minimize(self, loss, global_step=None, var_list=None, name=None):
        return self.apply_gradients(self.compute_gradients(loss, var_list), global_step, name)

    def get_slot(self, var, name):
        return self._slots[name].get(var)

    def get_slot_names(self):
        return list(self._slots)

    def variables(self):
        return [s for d in self._slots.values() for s in d.values()]

    # -- execution -----------------------------------------------------------------------------
    def _lr_value(self, ctx):
        lr = self._lr
        if isinstance(lr, Node):
            lr = ctx.eval(lr)
        return float(lr)

    def _hyper(self, lr):
        return [lr, 0.0, 0.0, 0.0, float(self._t)]

    def _apply_local(self, var, g, lr):
        with var._lock:
            var._local.sub_(lr * g.to(var._local.device, var._local.dtype))


class GradientDescentOptimizer(Optimizer):
    """w -= lr * g  (ApplyGradientDescent)."""

    def __init__(self, learning_rate, use_locking=False, name="GradientDescent"):
        super().__init__(learning_rate, use_locking, name)


class AdagradOptimizer(Optimizer):
    """acc += g^2; w -= lr * g / sqrt(acc), accumulator initialised to 0.1 (TF default)."""
    PS_KIND = 1

    def __init__(self, learning_rate, initial_accumulator_value=0.1, use_locking=False, name="Adagrad"):
        super().__init__(learning_rate, use_locking, name)
        self._init_acc = initial_accumulator_value

    def _hyper(self, lr):
        return [lr, self._init_acc, 0.0, 0.0, 0.0]

    def _apply_local(self, var, g, lr):
        acc = self._slots["accumulator"].get(var)
        if acc is None:
            acc = torch.full_like(var._local, self._init_acc)
            self._slots["accumulator"][var] = acc
        g = g.to(var._local.device, var._local.dtype)
        with var._lock:
            acc.add_(g * g)
            var._local.sub_(lr * g / acc.sqrt())


class MomentumOptimizer(Optimizer):
    """accum = mu*accum + g; w -= lr*accum  (TF ApplyMomentum)."""
    PS_KIND = 2

    def __init__(self, learning_rate, momentum, use_locking=False, name="Momentum", use_nesterov=False):
        super().__init__(learning_rate, use_locking, name)
        self._mu = momentum
        self._nesterov = use_nesterov

    def _hyper(self, lr):
        return [lr, self._mu, 0.0, 0.0, 0.0]

    def _apply_local(self, var, g, lr):
        m = self._slots["momentum"].get(var)
        if m is None:
            m = torch.zeros_like(var._local)
            self._slots["momentum"][var] = m
        g = g.to(var._local.device, var._local.dtype)
        with var._lock:
            m.mul_(self._mu).add_(g)
            var._local.sub_(lr * (g + self._mu * m if self._nesterov else m))


class AdamOptimizer(Optimizer):
    PS_KIND = 3

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, use_locking=False, name="Adam"):
        super().__init__(learning_rate, use_locking, name)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon

    def _hyper(self, lr):
        return [lr, self._b1, self._b2, self._eps, float(self._t)]

    def _apply_local(self, var, g, lr):
        m = self._slots["m"].setdefault(var, torch.zeros_like(var._local))
        v = self._slots["v"].setdefault(var, torch.zeros_like(var._local))
        g = g.to(var._local.device, var._local.dtype)
        t = self._t
        lrt = lr * (1 - self._b2 ** t) ** 0.5 / (1 - self._b1 ** t)
        with var._lock:
            m.mul_(self._b1).add_(g, alpha=1 - self._b1)
            v.mul_(self._b2).addcmul_(g, g, value=1 - self._b2)
            var._local.sub_(lrt * m / (v.sqrt() + self._eps))


class _ApplyOp(Op):
    def __init__(self, opt, gv, global_step, name):
        self.opt = opt
        self.gv = gv
        self.global_step = global_step
        super().__init__(lambda c: None, [g for g, _ in gv], name)

    def _eval(self, ctx):
        opt = self.opt
        grads = [ctx.eval(g) for g, _ in self.gv]
        lr = opt._lr_value(ctx)
        opt._t += 1
        gs = self.global_step
        gs_done = False
        by_task = defaultdict(list)
        for g, (_, v) in zip(grads, self.gv):
            if g is None:
                continue
            if isinstance(v, Variable) and v.remote:
                by_task[v.ps_task].append((v, g))
            else:
                opt._apply_local(v, g, lr)
        from .. import _runtime  # noqa: F401
        for task, items in by_task.items():
            gs_name = ""
            if gs is not None and not gs_done and isinstance(gs, Variable) and gs.remote and gs.ps_task == task:
                gs_name = gs._name
                gs_done = True
            if fault.should_drop_grad():  # DTG_FAULT=drop_grad:P -- the whole push is lost in transit
                opt.dropped_pushes = getattr(opt, "dropped_pushes", 0) + 1
                continue
            client = items[0][0]._client()
            step, _ = client.apply(opt.PS_KIND, opt._hyper(lr), bool(opt._use_locking), gs_name,
                                   [(v._name, _as_np(g.float())) for v, g in items], False)
        if gs is not None and not gs_done:
            if gs.remote:
                gs._client().assign_add(gs._name, np.ones(gs.shape, dtype=_np_dtype(gs.dtype)))
            else:
                with gs._lock:
                    gs._local.add_(1)
        return None


def _np_dtype(dt):
    return {torch.int32: np.int32, torch.int64: np.int64, torch.float32: np.float32, torch.float64: np.float64}[dt]


# ---- global step ----------------------------------------------------------------------------------
def get_global_step(graph=None):
    coll = G.get_collection(G.GraphKeys.GLOBAL_STEP)
    if coll:
        return coll[0]
    for v in G.get_collection(G.GraphKeys.GLOBAL_VARIABLES):
        if v.op.name == "global_step":
            return v
    return None


def create_global_step(graph=None):
    from ..graph import GraphKeys
    v = Variable(torch.tensor(0, dtype=torch.int64), trainable=False, name="global_step",
                 collections=[GraphKeys.GLOBAL_VARIABLES, GraphKeys.GLOBAL_STEP])
    return v


def get_or_create_global_step(graph=None):
    return get_global_step() or create_global_step()
