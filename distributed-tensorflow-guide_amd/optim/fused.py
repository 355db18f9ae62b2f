"""Fused flat-buffer optimizers for the north-star models (one kernel launch per dtype group).

The per-step hyper-parameters (learning rate, step count) live in a device tensor so a whole
training step can be captured in a hipGraph and replayed with a new schedule value.
"""
import torch

from ..ops import optim_kernels as K
from ..utils.trace import trace_range


class _FlatOptimizer:
    def __init__(self, flat, lr, weight_decay=0.0, wd_groups=("compute",)):
        self.flat = flat
        groups = list(flat)
        dev = groups[0].master.device if groups else torch.device("cpu")
        self.hyper = torch.tensor([float(lr), 0.0], dtype=torch.float32, device=dev)
        self.lr = float(lr)
        self.weight_decay = weight_decay
        self.wd_groups = set(wd_groups)
        self.step_count = 0

    def new_slot(self, g, key):
        """Allocate (and initialise) group ``g``'s optimizer slot ``key`` -- also its alignment padding, which no
        checkpoint holds (a restore allocates the slots it loads through this)."""
        return g.state_buffer(key)

    def set_lr(self, lr):
        self.lr = float(lr)
        self.hyper[0].fill_(self.lr)

    def _wd(self, g):
        return self.weight_decay if g.name in self.wd_groups else 0.0

    def step(self, grad_scale=1.0, zero_grad=True, ranges=None):
        """One optimizer step over every flat group.  ``ranges`` (DataParallel.step): a list of
        (group, lo, hi, ready) covering the groups, applied in that order, each after ``ready()`` has made the
        current stream wait for that slice's gradient (its bucket's collective) -- so the apply of the buckets
        reduced early runs while the last bucket's collective is still on the wire."""
        from ..parallel import overlap
        overlap.join()  # side-stream weight gradients done before the apply reads them
        self.step_count += 1
        with trace_range("dtg.apply"):  # roctx range (DTG_TRACE=1)
            if self.hyper.is_cuda:
                K.hyper_tick(self.hyper)  # dtg kernel (no framework elementwise launch on the step)
            else:
                self.hyper[1].add_(1.0)
            if ranges is None:
                for g in self.flat:
                    self._apply(g, grad_scale, zero_grad)
            else:
                for g, lo, hi, ready in ranges:
                    ready()
                    self._apply(_Slice(g, lo, hi), grad_scale, zero_grad)

    def minimize(self, loss_fn, global_step=None, inputs=(), name=None):
        """A train op for dtg sessions (``sess.run(op, feed_dict)``): forward + backward of ``loss_fn(*inputs)``,
        this optimizer's fused apply, global_step += 1, on one replica (train/eager.py; for several ranks wrap it
        in ``dtg.train.SyncReplicasOptimizer``, the all-reduce mode)."""
        from ..train.eager import minimize
        return minimize(self, loss_fn, global_step, inputs, None, name)

    def state_dict(self):
        return {"step": self.step_count, "lr": self.lr,
                "state": {g.name: {k: v for k, v in g.state.items()} for g in self.flat}}

    def load_state_dict(self, sd):
        self.step_count = int(sd.get("step", 0))
        self.set_lr(sd.get("lr", self.lr))
        self.hyper[1].fill_(float(self.step_count))
        for g in self.flat:
            for k, v in sd.get("state", {}).get(g.name, {}).items():
                g.state_buffer(k).copy_(v)


class _Slice:
    """A contiguous element range [lo, hi) of a flat group, with the group's name / buffers sliced alike (the
    fused applies are elementwise, so applying a group slice by slice is bit-identical to applying it whole)."""

    def __init__(self, g, lo, hi):
        self._g, self.lo, self.hi = g, lo, hi
        self.name = g.name
        self.master = g.master[lo:hi]
        self.grad = g.grad[lo:hi]
        self.mirror = g.mirror[lo:hi] if g.mirror is not None else None
        self.state = g.state

    def state_buffer(self, key):
        return self._g.state_buffer(key)[self.lo:self.hi]


class FusedSGD(_FlatOptimizer):
    """Momentum SGD (PyTorch semantics, optional Nesterov); momentum=0 -> plain SGD."""

    def __init__(self, flat, lr, momentum=0.9, weight_decay=0.0, nesterov=False, wd_groups=("compute",)):
        super().__init__(flat, lr, weight_decay, wd_groups)
        self.momentum = momentum
        self.nesterov = nesterov

    def _apply(self, g, gscale, zero_grad):
        if self.momentum == 0.0:
            K.sgd(g.master, g.grad, self.hyper, g.mirror, self._wd(g), gscale, zero_grad)
        else:
            K.momentum(g.master, g.grad, g.state_buffer("momentum"), self.hyper, g.mirror, self.momentum,
                       self._wd(g), self.nesterov, gscale, zero_grad)


class FusedAdam(_FlatOptimizer):
    """AdamW with decoupled weight decay (BERT pre-training)."""

    def __init__(self, flat, lr, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01, wd_groups=("compute",)):
        super().__init__(flat, lr, weight_decay, wd_groups)
        self.betas = betas
        self.eps = eps

    def _apply(self, g, gscale, zero_grad):
        K.adam(g.master, g.grad, g.state_buffer("m"), g.state_buffer("v"), self.hyper, g.mirror, self.betas[0],
               self.betas[1], self.eps, self._wd(g), gscale, zero_grad)


class FusedAdagrad(_FlatOptimizer):
    """TF-style Adagrad (initial accumulator 0.1, no epsilon) -- DOWNPOUR's optimizer."""

    def __init__(self, flat, lr, initial_accumulator_value=0.1, eps=0.0):
        super().__init__(flat, lr, 0.0)
        self.init_acc = initial_accumulator_value
        self.eps = eps

    def new_slot(self, g, key):
        fresh = key not in g.state
        buf = g.state_buffer(key)
        if fresh and key == "acc":
            buf.fill_(self.init_acc)
        return buf

    def _acc(self, g):
        # the WHOLE group's accumulator is created and filled with the initial value on first use: DataParallel.step
        # applies a group slice by slice (_Slice shares the group's state dict), so a per-slice "fresh" test would
        # fill only the first slice and leave later slices at the allocator's zeros (lr * sign(g), or 0/0)
        full = g._g if isinstance(g, _Slice) else g
        if "acc" not in full.state:
            self.new_slot(full, "acc")
        return g.state_buffer("acc")

    def _apply(self, g, gscale, zero_grad):
        K.adagrad(g.master, g.grad, self._acc(g), self.hyper, g.mirror, self.eps, gscale, zero_grad)


def make_optimizer(kind, flat, lr, **kw):
    """A fused flat optimizer by name, for the CLI flags of the async-PS examples and bench (``--local_opt``,
    ``--ps_opt``): ``sgd`` plain SGD (TF GradientDescentOptimizer, ADAG's local and global rule), ``momentum``
    momentum 0.9 SGD, ``adagrad`` TF Adagrad with initial accumulator 0.1 (DOWNPOUR's local and global rule,
    /root/reference/DOWNPOUR/DOWNPOUR.py:57, :92), ``adam`` AdamW.  ``none`` returns None."""
    if kind in (None, "none"):
        return None
    if kind == "sgd":
        return FusedSGD(flat, lr=lr, momentum=0.0)
    if kind == "momentum":
        return FusedSGD(flat, lr=lr, momentum=kw.get("momentum", 0.9), weight_decay=kw.get("weight_decay", 0.0))
    if kind == "adagrad":
        return FusedAdagrad(flat, lr=lr)
    if kind == "adam":
        return FusedAdam(flat, lr=lr, weight_decay=kw.get("weight_decay", 0.01))
    raise ValueError("unknown optimizer %r (sgd, momentum, adagrad, adam, none)" % (kind,))
