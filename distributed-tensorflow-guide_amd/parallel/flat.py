"""Flat, HBM-resident parameter / gradient / optimizer-state buffers.

MI355X-first layout: instead of one tensor per parameter, every parameter of a dtype group lives
in ONE contiguous buffer (288 GB of HBM makes the fp32 master + bf16 compute copy + optimizer
state trivially affordable).  Consequences:

* the optimizer is a single vectorised kernel over the whole model (csrc/kernels/optim.hip);
* gradient buckets for RCCL all-reduce are plain slices of the flat grad buffer -- no
  flatten/unflatten copies (``param.grad`` is a view into it and autograd accumulates in place);
* parameters are laid out in REVERSE registration order, which is (approximately) the order in
  which backward produces their gradients, so every bucket is contiguous and becomes ready as
  a unit;
* PS push/pull and checkpoints move one buffer per group.

Groups: ``compute`` (weights of conv/linear/embedding: fp32 master + bf16 mirror that the model
reads, bf16 grads) and ``fp32`` (norm affine params and biases: the master IS the parameter,
fp32 grads).
"""
from collections import OrderedDict

import torch

from . import grad_sink

ALIGN = 64  # elements; keeps every view 128-byte aligned for 16-B vector access


def _align(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _view_like(flat, off, p):
    """A view of flat[off: off+numel] with p's shape and memory format."""
    n = p.numel()
    seg = flat[off:off + n]
    if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous():
        o, i, kh, kw = p.shape
        return seg.view(o, kh, kw, i).permute(0, 3, 1, 2)
    return seg.view(p.shape)


class FlatGroup:
    def __init__(self, name, params, names, compute_dtype, device):
        self.name = name
        self.params = params
        self.names = names
        self.compute_dtype = compute_dtype
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += _align(p.numel())
        self.numel = off
        self.device = device
        self.master = torch.zeros(off, dtype=torch.float32, device=device)
        self.mirror = torch.zeros(off, dtype=compute_dtype, device=device) if compute_dtype != torch.float32 else None
        self.grad = torch.zeros(off, dtype=compute_dtype, device=device)
        self.state = {}
        with torch.no_grad():
            for p, o in zip(params, self.offsets):
                _view_like(self.master, o, p).copy_(p.detach().float())
                store = self.mirror if self.mirror is not None else self.master
                v = _view_like(store, o, p)
                if self.mirror is not None:
                    v.copy_(p.detach().to(compute_dtype))
                p.data = v
                p.grad = _view_like(self.grad, o, p)
                grad_sink.mark(p)

    def state_buffer(self, key):
        """Lazily allocated fp32 optimizer state with the master's layout."""
        if key not in self.state:
            self.state[key] = torch.zeros_like(self.master)
        return self.state[key]

    def param_slices(self):
        for name, p, o in zip(self.names, self.params, self.offsets):
            yield name, p, o, p.numel()

    def master_view(self, i):
        return _view_like(self.master, self.offsets[i], self.params[i])

    def refresh_mirror(self):
        if self.mirror is not None:
            from ..ops import optim_kernels
            optim_kernels.refresh_mirror(self.master, self.mirror)

    def zero_grad(self):
        self.grad.zero_()


class FlatBuffers:
    """The module's floating-point buffers (BatchNorm running_mean / running_var) in ONE fp32 flat
    buffer; every module buffer is rebound to a view of it, so kernels that update the statistics in
    place write straight into the flat storage.  The async PS moves this buffer with the parameters
    (in TF's between-graph setup the BN moving averages are PS variables the workers update)."""

    def __init__(self, module, device=None):
        entries = []
        for mname, m in module.named_modules():
            for bname, b in m._buffers.items():
                if b is not None and b.dtype == torch.float32:
                    entries.append((f"{mname}.{bname}" if mname else bname, m, bname, b))
        self.names = [e[0] for e in entries]
        self.offsets = []
        off = 0
        for _, _, _, b in entries:
            self.offsets.append(off)
            off += _align(b.numel())
        self.numel = off
        device = device or (entries[0][3].device if entries else torch.device("cpu"))
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.views = []
        with torch.no_grad():
            for (_, m, bname, b), o in zip(entries, self.offsets):
                v = self.flat[o:o + b.numel()].view(b.shape)
                v.copy_(b)
                m._buffers[bname] = v
                self.views.append(v)

    def __len__(self):
        return len(self.names)

    def named(self):
        return zip(self.names, self.views)


class FlatParams:
    """Partition a module's parameters into flat groups (see module docstring)."""

    def __init__(self, module, compute_dtype=torch.bfloat16, keep_fp32=None, device=None):
        if keep_fp32 is None:
            keep_fp32 = lambda name, p: p.dim() <= 1  # noqa: E731 - norm params and biases
        named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        named.reverse()  # ~ backward order
        device = device or (named[0][1].device if named else torch.device("cpu"))
        comp = [(n, p) for n, p in named if not keep_fp32(n, p)]
        f32 = [(n, p) for n, p in named if keep_fp32(n, p)]
        self.groups = OrderedDict()
        if comp:
            self.groups["compute"] = FlatGroup("compute", [p for _, p in comp], [n for n, _ in comp],
                                               compute_dtype, device)
        if f32:
            self.groups["fp32"] = FlatGroup("fp32", [p for _, p in f32], [n for n, _ in f32], torch.float32, device)
        self.module = module
        fb = FlatBuffers(module, device)
        self.buffers = fb if len(fb) else None

    def __iter__(self):
        return iter(self.groups.values())

    def numel(self):
        return sum(g.numel for g in self.groups.values())

    def refresh_mirrors(self):
        for g in self:
            g.refresh_mirror()

    def zero_grad(self):
        for g in self:
            g.zero_grad()

    def named_masters(self):
        """(name, fp32 master view) for every parameter -- what checkpoints and the PS see."""
        for g in self:
            for i, n in enumerate(g.names):
                yield n, g.master_view(i)
