"""ResNet-50 synchronous data-parallel training with checkpoint / resume (BASELINE.json config 3 as a
training job rather than a benchmark).

One process per GPU over RCCL (torchrun), the chief (rank 0) writes a TensorBundle checkpoint of the flat
parameters + optimizer state every ``--save_every`` steps (``dtg.train.save_flat``), and a (re)started job
restores the latest one and continues from its global step -- the reference's MonitoredTrainingSession /
Supervisor resume semantics (DOWNPOUR/DOWNPOUR.py:126-127, Hogwild/Hogwild.py:47-50) for the all-reduce
path.  A lost rank is fail-stop (parallel/comm.py Watchdog): restart the job and it resumes.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 resnet50_train.py \\
        --steps 1000 --ckpt_dir /path/to/ckpt [--save_every 100]
"""
import argparse
import os

import _path  # noqa: F401

import torch

import dtg  # noqa: F401
from dtg import fault, ops
from dtg.models import resnet
from dtg.optim import FusedSGD
from dtg.parallel import DataParallel, FlatParams, comm
from dtg.train import latest_checkpoint, restore_flat, save_flat


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100, help="last global step (absolute, like StopAtStepHook)")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--ckpt_dir", default="logdir")
    ap.add_argument("--save_every", type=int, default=100)
    ap.add_argument("--tiny", action="store_true", help="4-block narrow ResNet on 32x32 images (CPU tests)")
    a, _ = ap.parse_known_args()
    rank, _, world, device = comm.init()
    torch.manual_seed(1234)
    model = (resnet.resnet18_like_tiny(10) if a.tiny else resnet.resnet50()).to(device)
    model = model.to(memory_format=torch.channels_last)
    ncls = 10 if a.tiny else 1000
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    flat = FlatParams(model, compute_dtype=dtype)
    dp = DataParallel(flat, bucket_mb=8.0)
    opt = FusedSGD(flat, lr=a.lr * world, momentum=0.9, weight_decay=5e-5)
    step = 0
    ck = latest_checkpoint(a.ckpt_dir)
    if ck:
        step = restore_flat(flat, ck, optimizer=opt) or 0
        if rank == 0:
            print("resumed from %s (global step %d)" % (ck, step), flush=True)
    else:
        dp.broadcast_parameters(0)
    model.train()
    x, y = resnet.synthetic_batch(a.batch, device, dtype, 32 if a.tiny else a.image, ncls, seed=rank)
    prefix = os.path.join(a.ckpt_dir, "model.ckpt")
    while step < a.steps:
        fault.maybe_kill_rank(rank, step + 1)
        loss = ops.softmax_cross_entropy(model(x), y)
        loss.backward()
        dp.finish()
        opt.step(grad_scale=dp.grad_scale)
        step += 1
        if rank == 0 and (step % a.save_every == 0 or step == a.steps):
            os.makedirs(a.ckpt_dir, exist_ok=True)
            save_flat(flat, prefix, global_step=step, optimizer=opt)
        if rank == 0 and step % 10 == 0:
            print("step %d loss %.4f" % (step, loss.item()), flush=True)
    comm.barrier()
    if rank == 0:
        print("done at global step %d" % step, flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
