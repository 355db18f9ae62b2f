"""``MirroredStrategy``-style front end over dtg's synchronous data parallelism.

BASELINE.json config 2 asks for a "single-replica MirroredStrategy-equiv"; SURVEY §2.3 notes the
reference has no in-graph replication.  MI355X-first this is one process per GPU (RCCL over xGMI
for N > 1, a no-op reducer for N = 1), exposed with the TF names a user of the guide expects:

    strategy = MirroredStrategy()
    with strategy.scope():
        model = MnistCNN().to(strategy.device)
    trainer = strategy.distribute(model, lambda flat: FusedSGD(flat, lr=0.05))
    for x, y in data:
        loss = trainer.step(lambda: loss_fn(model(x), y))

or, session-driven (hooks, checkpoints, resume -- train/eager.py)::

    x, y = dtg.placeholder(), dtg.placeholder()
    train_op = trainer.minimize(lambda x, y: loss_fn(model(x), y), global_step=gs, inputs=(x, y))
    with dtg.train.MonitoredTrainingSession(is_chief=strategy.rank == 0, checkpoint_dir=ck,
                                            hooks=[trainer.make_session_run_hook(strategy.rank == 0), ...]) as sess:
        while not sess.should_stop():
            sess.run(train_op, feed_dict={x: xb, y: yb})

Both run ``DataParallel.step``: each bucket's fused apply as soon as its all-reduce has landed.  The trainer
is the all-reduce mode of ``dtg.train.SyncReplicasOptimizer`` (replicas_to_aggregate = total = world).
"""
import contextlib

import torch

from . import comm
from .flat import FlatParams


class _Trainer:
    def __init__(self, flat, sro):
        self.flat, self.sro = flat, sro
        self.dp, self.opt = sro.dp, sro._flat_opt

    def step(self, loss_fn):
        loss = loss_fn()
        loss.backward()
        self.dp.step(self.opt)  # per-bucket apply overlapped with the collective tail
        return loss

    def minimize(self, loss_fn, global_step=None, inputs=(), name=None):
        return self.sro.minimize(loss_fn, global_step=global_step, inputs=inputs, name=name)

    def make_session_run_hook(self, is_chief):
        return self.sro.make_session_run_hook(is_chief)


class MirroredStrategy:
    def __init__(self, backend=None, bucket_mb=32.0, compute_dtype=torch.bfloat16):
        self.rank, self.local_rank, self.world, self.device = comm.init(backend)
        self.bucket_mb = bucket_mb
        self.compute_dtype = compute_dtype

    @property
    def num_replicas_in_sync(self):
        return self.world

    @contextlib.contextmanager
    def scope(self):
        """Variables created here live on this replica's device (one process per GPU)."""
        if self.device.type == "cuda":
            with torch.cuda.device(self.device):
                yield self
        else:
            yield self

    def distribute(self, model, optimizer_fn):
        from ..train.saver import register_flat_model
        from ..train.sync_replicas import SyncReplicasOptimizer
        flat = FlatParams(model, compute_dtype=self.compute_dtype)
        sro = SyncReplicasOptimizer(optimizer_fn(flat), self.world, self.world, bucket_mb=self.bucket_mb)
        sro._check_allreduce()
        sro._data_parallel().broadcast_parameters(0)
        register_flat_model(flat, sro._flat_opt)  # Saver / CheckpointSaverHook keys: the parameter names
        return _Trainer(flat, sro)

    def shard(self, t):
        """This replica's slice of a global batch (dim 0)."""
        n = t.shape[0] // self.world
        return t[self.rank * n:(self.rank + 1) * n]

    def reduce_mean(self, x):
        if self.world == 1:
            return x
        import torch.distributed as dist
        t = torch.as_tensor(x, dtype=torch.float32, device=self.device).clone()
        dist.all_reduce(t)
        return t / self.world
