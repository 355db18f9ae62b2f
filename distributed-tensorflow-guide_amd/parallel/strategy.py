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
"""
import contextlib

import torch

from . import comm
from .ddp import DataParallel
from .flat import FlatParams


class _Trainer:
    def __init__(self, flat, dp, opt):
        self.flat, self.dp, self.opt = flat, dp, opt

    def step(self, loss_fn):
        loss = loss_fn()
        loss.backward()
        self.dp.finish()
        self.opt.step(grad_scale=self.dp.grad_scale)
        return loss


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
        flat = FlatParams(model, compute_dtype=self.compute_dtype)
        dp = DataParallel(flat, bucket_mb=self.bucket_mb)
        dp.broadcast_parameters(0)
        return _Trainer(flat, dp, optimizer_fn(flat))

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
