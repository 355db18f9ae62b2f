"""Direct gradient writes into the flat gradient buffer.

Parameters managed by :class:`FlatParams` have ``param.grad`` permanently bound to a view of the
group's flat grad buffer.  dtg's weight-gradient kernels (MFMA GEMM epilogue with beta=1) add
their result straight into that view instead of returning a tensor that autograd's
AccumulateGrad would then add (one extra read + write of every weight gradient, and one extra
launch per parameter).  Because AccumulateGrad is bypassed, its post-accumulate hooks do not fire;
the op calls :func:`notify` instead, which is what the all-reduce bucketing listens to.
"""
_listeners = []


def enabled(p):
    return p is not None and getattr(p, "_dtg_flat_grad", False)


def mark(p):
    p._dtg_flat_grad = True


def add_listener(fn):
    _listeners.append(fn)


def remove_listener(fn):
    if fn in _listeners:
        _listeners.remove(fn)


def notify(p):
    for fn in list(_listeners):
        fn(p)
