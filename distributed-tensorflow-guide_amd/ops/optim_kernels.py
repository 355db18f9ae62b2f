"""Flat-buffer optimizer applies (csrc/kernels/optim.hip) with a CPU reference path.

Every function updates ``master`` (fp32) in place from ``grad`` (fp32 or bf16), optionally
refreshes a bf16 ``mirror`` of the weights, scales the gradient by ``gscale`` and zeroes it.
``hyper`` is a float32 device tensor {lr, step} so the apply is graph-capturable.
"""
import torch

from ._native import lib


def _cpu_finish(master, mirror, grad, zero_grad):
    if mirror is not None:
        mirror.copy_(master)
    if zero_grad:
        grad.zero_()


def sgd(master, grad, hyper, mirror=None, wd=0.0, gscale=1.0, zero_grad=False):
    if master.is_cuda:
        return lib().sgd_apply(master, mirror, grad, hyper, wd, gscale, zero_grad)
    lr = float(hyper[0])
    g = grad.float() * gscale + wd * master
    master.add_(g, alpha=-lr)
    _cpu_finish(master, mirror, grad, zero_grad)


def momentum(master, grad, mom, hyper, mirror=None, mu=0.9, wd=0.0, nesterov=False, gscale=1.0, zero_grad=False):
    if master.is_cuda:
        return lib().momentum_apply(master, mirror, grad, mom, hyper, mu, wd, nesterov, gscale, zero_grad)
    lr = float(hyper[0])
    g = grad.float() * gscale + wd * master
    mom.mul_(mu).add_(g)
    master.add_(g + mu * mom if nesterov else mom, alpha=-lr)
    _cpu_finish(master, mirror, grad, zero_grad)


def adagrad(master, grad, acc, hyper, mirror=None, eps=0.0, gscale=1.0, zero_grad=False):
    """TF ApplyAdagrad: acc += g^2 ; w -= lr * g / sqrt(acc)  (SURVEY §2.5 N5)."""
    if master.is_cuda:
        return lib().adagrad_apply(master, mirror, grad, acc, hyper, eps, gscale, zero_grad)
    lr = float(hyper[0])
    g = grad.float() * gscale
    acc.add_(g * g)
    master.sub_(lr * g * torch.rsqrt(acc + eps))
    _cpu_finish(master, mirror, grad, zero_grad)


def adam(master, grad, m, v, hyper, mirror=None, b1=0.9, b2=0.999, eps=1e-8, wd=0.0, gscale=1.0,
         zero_grad=False):
    """AdamW (decoupled weight decay); hyper = {lr, step} with step already incremented."""
    if master.is_cuda:
        return lib().adam_apply(master, mirror, grad, m, v, hyper, b1, b2, eps, wd, gscale, zero_grad)
    lr, t = float(hyper[0]), float(hyper[1])
    g = grad.float() * gscale
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    mh = m / (1 - b1 ** t)
    vh = v / (1 - b2 ** t)
    master.sub_(lr * (mh / (vh.sqrt() + eps) + wd * master))
    _cpu_finish(master, mirror, grad, zero_grad)


def hyper_tick(hyper):
    """hyper[1] += 1 on the device (the step counter the fused applies read)."""
    lib().hyper_tick(hyper)


def axpby(acc, g, alpha, beta):
    """acc = alpha * acc + beta * g (window accumulate for DOWNPOUR / ADAG / SDAG)."""
    if acc.is_cuda:
        return lib().axpby(acc, g, alpha, beta)
    acc.mul_(alpha).add_(g.float(), alpha=beta)


def refresh_mirror(master, mirror):
    if master.is_cuda:
        return lib().f32_to_bf16(master, mirror)
    mirror.copy_(master)
