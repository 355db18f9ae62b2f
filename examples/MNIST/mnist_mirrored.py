"""MNIST CNN with the MirroredStrategy front end (BASELINE.json config 2).  Synthetic digits (no
dataset offline).  Single GPU by default; under torchrun every process is one replica.

    python mnist_mirrored.py [--steps 200] [--batch 256]
"""
import argparse
import time

import _path  # noqa: F401

import torch

import dtg  # noqa: F401
from dtg import ops
from dtg.models.mnist import MnistCNN, synthetic_mnist
from dtg.optim import FusedSGD
from dtg.parallel import MirroredStrategy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=256, help="global batch")
    ap.add_argument("--lr", type=float, default=0.01)
    a, _ = ap.parse_known_args()
    strategy = MirroredStrategy()
    dtype = torch.bfloat16 if strategy.device.type == "cuda" else torch.float32
    with strategy.scope():
        model = MnistCNN().to(strategy.device)
    trainer = strategy.distribute(model, lambda flat: FusedSGD(flat, lr=a.lr, momentum=0.9))
    per = a.batch // strategy.num_replicas_in_sync
    t0 = time.time()
    for i in range(a.steps):
        x, y = synthetic_mnist(per, strategy.device, dtype, seed=i * 1000 + strategy.rank)
        loss = trainer.step(lambda: ops.softmax_cross_entropy(model(x), y))
        if i % 50 == 0 and strategy.rank == 0:
            print(f"step {i} loss {loss.item():.4f}", flush=True)
    if strategy.device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.time() - t0
    x, y = synthetic_mnist(1024, strategy.device, dtype, seed=10 ** 6)
    with torch.no_grad():
        acc = (model(x).argmax(1) == y).float().mean().item()
    if strategy.rank == 0:
        print(f"accuracy {acc:.4f}  {a.steps * a.batch / dt:.0f} images/sec", flush=True)


if __name__ == "__main__":
    main()
