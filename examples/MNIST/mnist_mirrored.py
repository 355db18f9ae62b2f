"""MNIST CNN with the MirroredStrategy front end (BASELINE.json config 2), driven by a MonitoredTrainingSession
like the reference's scripts (/root/reference/DOWNPOUR/DOWNPOUR.py:116-127): StopAtStepHook, a checkpoint
directory (resume continues the global step), a StepCounterHook reporting images/sec per worker and for the
whole job.  Synthetic digits (no dataset offline).  Single GPU by default; under torchrun every process is one
replica (RCCL all-reduce, per-bucket fused apply).

    python mnist_mirrored.py [--steps 200] [--batch 256] [--ckpt_dir DIR]
"""
import argparse
import os

import _path  # noqa: F401

import torch

import dtg
from dtg import ops
from dtg.models.mnist import MnistCNN, synthetic_mnist
from dtg.optim import FusedSGD
from dtg.parallel import MirroredStrategy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200, help="last global step")
    ap.add_argument("--batch", type=int, default=256, help="global batch")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--ckpt_dir", default=None, help="checkpoint directory (resume from its latest checkpoint)")
    ap.add_argument("--save_every", type=int, default=100)
    a, _ = ap.parse_known_args()
    strategy = MirroredStrategy()
    is_chief = strategy.rank == 0
    dtype = torch.bfloat16 if strategy.device.type == "cuda" else torch.float32
    with strategy.scope():
        model = MnistCNN().to(strategy.device)
    trainer = strategy.distribute(model, lambda flat: FusedSGD(flat, lr=a.lr, momentum=0.9))
    per = a.batch // strategy.num_replicas_in_sync
    images, labels = dtg.placeholder(name="images"), dtg.placeholder(name="labels")
    global_step = dtg.train.get_or_create_global_step()
    train_op = trainer.minimize(lambda x, y: ops.softmax_cross_entropy(model(x), y), global_step=global_step,
                                inputs=(images, labels))
    counter = dtg.train.StepCounterHook(every_n_steps=50, batch_size=per, aggregate=True)
    hooks = [trainer.make_session_run_hook(is_chief), dtg.train.StopAtStepHook(last_step=a.steps), counter]
    with dtg.train.MonitoredTrainingSession(is_chief=is_chief, checkpoint_dir=a.ckpt_dir, hooks=hooks,
                                            save_checkpoint_secs=None,
                                            save_checkpoint_steps=a.save_every if a.ckpt_dir else None,
                                            log_step_count_steps=None, save_summaries_steps=None) as sess:
        step = int(sess.run(global_step))
        if is_chief and sess.restored_from:
            print("resumed from %s (global step %d)" % (sess.restored_from, step), flush=True)
        while not sess.should_stop():
            x, y = synthetic_mnist(per, strategy.device, dtype, seed=step * 1000 + strategy.rank)
            if step % 50 == 0:
                _, loss, step = sess.run([train_op, train_op.loss, global_step], feed_dict={images: x, labels: y})
                if is_chief:
                    print(f"step {step} loss {float(loss):.4f}", flush=True)
            else:
                _, step = sess.run([train_op, global_step], feed_dict={images: x, labels: y})
            step = int(step)
    x, y = synthetic_mnist(1024, strategy.device, dtype, seed=10 ** 6)
    with torch.no_grad():
        acc = (model(x).argmax(1) == y).float().mean().item()
    if is_chief:
        rate = counter.history[-1] if counter.history else {}
        node = rate.get("examples/sec/node", rate.get("examples/sec", float("nan")))
        print(f"accuracy {acc:.4f}  {node:.0f} images/sec (node), global step {step}", flush=True)
        if a.ckpt_dir:
            print("checkpoint", dtg.train.latest_checkpoint(a.ckpt_dir), flush=True)
    if os.environ.get("WORLD_SIZE"):
        from dtg.parallel import comm
        comm.shutdown()


if __name__ == "__main__":
    main()
