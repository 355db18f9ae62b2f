"""Eager GPU training steps behind the tf.train session surface.

The reference drives every model through ``sess.run(train_op)`` inside a MonitoredTrainingSession with a
StopAtStepHook and a checkpoint_dir (/root/reference/DOWNPOUR/DOWNPOUR.py:116-127,
/root/reference/Synchronous-SGD/ssgd.py:51-69).  dtg's north-star models (ResNet-50, BERT, the MNIST CNN) are
eager modules on flat HBM buffers (parallel/flat.py) running hand-written HIP kernels.  This module wraps one
of their training steps as two graph nodes, so the same session, hooks and Saver drive them::

    x, y = dtg.placeholder(name="images"), dtg.placeholder(name="labels")
    gs = dtg.train.get_or_create_global_step()
    opt = dtg.train.SyncReplicasOptimizer(FusedSGD(flat, lr=0.1), replicas_to_aggregate=world,
                                          total_num_replicas=world)          # all-reduce mode (no PS)
    train_op = opt.minimize(lambda x, y: ops.softmax_cross_entropy(model(x), y), global_step=gs, inputs=(x, y))
    hooks = [opt.make_session_run_hook(rank == 0), dtg.train.StopAtStepHook(last_step=1000)]
    with dtg.train.MonitoredTrainingSession(is_chief=rank == 0, checkpoint_dir=ck, hooks=hooks) as sess:
        while not sess.should_stop():
            sess.run(train_op, feed_dict={x: xb, y: yb})

* the gradients node (:class:`EagerGradients`) runs forward + backward; DataParallel's hooks launch each
  bucket's RCCL all-reduce from inside the backward (parallel/ddp.py);
* the apply node (:class:`EagerApply`) runs ``DataParallel.step(opt)`` -- each bucket's fused apply as soon as
  its collective has landed -- and adds 1 to ``global_step``, a host-side int64 variable, so a step costs no
  device synchronisation;
* ``train_op.loss`` is the step's loss: fetching it synchronises the device (as a TF fetch does); running the
  train op alone does not, so the host keeps queueing steps ahead of the GPU.

Checkpoints: the model is registered with the Saver (``register_flat_model``), so CheckpointSaverHook writes
one key per parameter name, the module buffers, the optimizer slots (``<param>/<slot>``), ``optimizer/step``
and ``global_step``; the chief restores the latest checkpoint, and the sync hook broadcasts the chief's state
to every rank before the first step (:func:`broadcast_training_state`).
"""
import torch

from .. import graph as G
from ..graph import Op, Tensor
from .saver import register_flat_model


def is_flat_optimizer(opt):
    """A fused flat-buffer optimizer (dtg.optim): one kernel per group over FlatParams buffers."""
    return hasattr(opt, "flat") and hasattr(opt, "_apply") and hasattr(opt, "step_count")


def fused_from_tf(opt, flat):
    """The fused flat optimizer implementing a tf.train optimizer's update rule on a FlatParams model
    (GradientDescent -> plain SGD, Momentum -> momentum SGD, Adagrad -> TF Adagrad, Adam -> Adam without decay)."""
    from ..optim import FusedAdagrad, FusedAdam, FusedSGD
    from .optimizer import AdagradOptimizer, AdamOptimizer, GradientDescentOptimizer, MomentumOptimizer
    lr = opt._lr
    if isinstance(lr, Tensor):
        lr = float(G.RunContext().eval(lr))
    lr = float(lr)
    if isinstance(opt, MomentumOptimizer):
        return FusedSGD(flat, lr=lr, momentum=opt._mu, nesterov=opt._nesterov)
    if isinstance(opt, AdagradOptimizer):
        return FusedAdagrad(flat, lr=lr, initial_accumulator_value=opt._init_acc)
    if isinstance(opt, AdamOptimizer):
        return FusedAdam(flat, lr=lr, betas=(opt._b1, opt._b2), eps=opt._eps, weight_decay=0.0)
    if isinstance(opt, GradientDescentOptimizer):
        return FusedSGD(flat, lr=lr, momentum=0.0)
    raise TypeError("no fused flat-buffer form of %s" % type(opt).__name__)


class EagerGradients(Tensor):
    """Forward + backward of ``loss_fn(*inputs)``; evaluates to the (detached) loss.  Parameter gradients land
    in the FlatParams gradient buffer, where the DataParallel hooks reduce them bucket by bucket."""

    def __init__(self, loss_fn, inputs=(), name="gradients"):
        self.loss_fn = loss_fn
        self._seed = None
        super().__init__(lambda c, *a: None, list(inputs), name)

    def _eval(self, ctx):
        loss = self.loss_fn(*[ctx.eval(i) for i in self.inputs])
        s = self._seed
        if s is None or s.shape != loss.shape or s.dtype != loss.dtype or s.device != loss.device:
            # backward seeded with a cached 1.0: loss.backward() would launch a fill kernel every step
            s = self._seed = torch.ones_like(loss)
        loss.backward(s)
        return loss.detach()


class EagerApply(Op):
    """Apply the reduced gradients (``DataParallel.step`` or, without data parallelism, ``opt.step``) and add 1
    to ``global_step``."""

    def __init__(self, grads, optimizer, dp=None, global_step=None, name="train"):
        self.grads, self.optimizer, self.dp, self.global_step = grads, optimizer, dp, global_step
        super().__init__(lambda c, *a: None, [grads], name)

    def _eval(self, ctx):
        ctx.eval(self.grads)
        if self.dp is not None:
            self.dp.step(self.optimizer)
        else:
            self.optimizer.step()
        gs = self.global_step
        if gs is not None:
            if getattr(gs, "remote", False):
                import numpy as np
                gs._client().assign_add(gs._name, np.ones(gs.shape, dtype=np.int64 if gs.dtype == torch.int64
                                                          else np.int32))
            else:
                with gs._lock:
                    gs._local.add_(1)
        return None

    @property
    def loss(self):
        """The step's loss as a fetchable tensor (fetching it synchronises the device)."""
        return self.grads


def minimize(optimizer, loss_fn, global_step=None, inputs=(), dp=None, name=None):
    """An eager train op: ``sess.run(op, feed_dict=...)`` = forward, backward, (bucketed all-reduce,) fused apply,
    global_step += 1.  ``optimizer`` is a fused flat optimizer; its model is registered with the Saver."""
    if not callable(loss_fn):
        raise TypeError("an eager train op needs a callable loss: loss_fn(*inputs) -> scalar tensor")
    register_flat_model(optimizer.flat, optimizer)
    grads = EagerGradients(loss_fn, inputs, (name or "train") + "/gradients")
    return EagerApply(grads, optimizer, dp, global_step, name or "train")


def broadcast_training_state(flat, optimizer=None, dp=None, global_step=None, src=0, group=None):
    """Make every rank start from rank ``src``'s state: parameters (masters + compute mirrors), module buffers,
    optimizer slots (allocated where the source has them -- it may have restored slots from a checkpoint that
    the other ranks never created) and step count, and the global step.  A no-op on one rank."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    if dp is not None:
        dp.broadcast_parameters(src)
    else:
        for g in flat:
            dist.broadcast(g.master, src, group=group)
            g.refresh_mirror()
        for buf in flat.module.buffers():
            if buf.is_floating_point() or buf.dtype in (torch.int64, torch.int32):
                dist.broadcast(buf, src, group=group)
    groups = list(flat)
    dev = groups[0].master.device if groups else torch.device("cpu")
    keys = [[sorted(g.state.keys()) for g in groups]]
    dist.broadcast_object_list(keys, src, group=group, device=dev if dev.type == "cuda" else None)
    for g, ks in zip(groups, keys[0]):
        for k in ks:
            dist.broadcast(g.state_buffer(k), src, group=group)
    gsv = 0
    if global_step is not None and global_step.is_initialized():
        gsv = int(global_step.read_value().item())
    scal = torch.tensor([getattr(optimizer, "step_count", 0) if optimizer is not None else 0, gsv],
                        dtype=torch.int64, device=dev)
    dist.broadcast(scal, src, group=group)
    if optimizer is not None and hasattr(optimizer, "step_count"):
        optimizer.step_count = int(scal[0].item())
        if hasattr(optimizer, "hyper"):
            optimizer.hyper[1].fill_(float(optimizer.step_count))
    if global_step is not None and not getattr(global_step, "remote", False):
        global_step.load(torch.tensor(int(scal[1].item()), dtype=global_step.dtype))
