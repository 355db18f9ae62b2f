"""ResNet-50 synchronous data-parallel training on the reference's session surface (BASELINE.json config 3 as a
training job rather than a benchmark).

The same shape as /root/reference/Synchronous-SGD/ssgd.py:51-69 and /root/reference/DOWNPOUR/DOWNPOUR.py:116-127:
``SyncReplicasOptimizer(opt, replicas_to_aggregate, total_num_replicas)`` -> ``minimize`` -> hooks
(sync-replicas hook, StopAtStepHook, StepCounterHook) -> ``MonitoredTrainingSession(checkpoint_dir,
save_checkpoint_steps)`` -> ``while not sess.should_stop(): sess.run(train_op)``.  With no PS in the job the
optimizer runs in its all-reduce mode: one process per GPU over RCCL, bucketed all-reduces fired from inside
the backward, each bucket's fused momentum apply as soon as its collective lands (train/eager.py).

The chief's CheckpointSaverHook writes a TensorBundle keyed by parameter name (plus ``<param>/momentum``,
``optimizer/step``, ``global_step``); a (re)started job restores the latest one on the chief, broadcasts it to
every rank and continues from its global step up to the absolute ``--steps`` (StopAtStepHook(last_step)).  A
lost rank is fail-stop (parallel/comm.py Watchdog): restart the job and it resumes.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 resnet50_train.py \\
        --steps 1000 --ckpt_dir /path/to/ckpt [--save_every 100]
"""
import argparse

import _path  # noqa: F401

import torch

import dtg
from dtg import fault, ops
from dtg.models import resnet
from dtg.optim import FusedSGD
from dtg.parallel import FlatParams, comm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100, help="last global step (absolute, like StopAtStepHook)")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--ckpt_dir", default="logdir")
    ap.add_argument("--save_every", type=int, default=100)
    ap.add_argument("--log_every", type=int, default=10)
    ap.add_argument("--tiny", action="store_true", help="4-block narrow ResNet on 32x32 images (CPU tests)")
    a, _ = ap.parse_known_args()
    rank, _, world, device = comm.init()
    is_chief = rank == 0
    torch.manual_seed(1234)
    model = (resnet.resnet18_like_tiny(10) if a.tiny else resnet.resnet50()).to(device)
    model = model.to(memory_format=torch.channels_last)
    ncls = 10 if a.tiny else 1000
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    flat = FlatParams(model, compute_dtype=dtype)
    model.train()

    images = dtg.placeholder(name="images")
    labels = dtg.placeholder(name="labels")
    global_step = dtg.train.get_or_create_global_step()
    opt = dtg.train.SyncReplicasOptimizer(FusedSGD(flat, lr=a.lr * world, momentum=0.9, weight_decay=5e-5),
                                          replicas_to_aggregate=world, total_num_replicas=world, bucket_mb=8.0)
    train_op = opt.minimize(lambda x, y: ops.softmax_cross_entropy(model(x), y), global_step=global_step,
                            inputs=(images, labels))
    hooks = [opt.make_session_run_hook(is_chief), dtg.train.StopAtStepHook(last_step=a.steps),
             dtg.train.StepCounterHook(every_n_steps=a.log_every, batch_size=a.batch, aggregate=True,
                                       log=is_chief)]
    x, y = resnet.synthetic_batch(a.batch, device, dtype, 32 if a.tiny else a.image, ncls, seed=rank)
    with dtg.train.MonitoredTrainingSession(is_chief=is_chief, checkpoint_dir=a.ckpt_dir, hooks=hooks,
                                            save_checkpoint_secs=None, save_checkpoint_steps=a.save_every,
                                            log_step_count_steps=None, save_summaries_steps=None) as sess:
        step = int(sess.run(global_step))
        if is_chief and sess.restored_from:
            print("resumed from %s (global step %d)" % (sess.restored_from, step), flush=True)
        while not sess.should_stop():
            fault.maybe_kill_rank(rank, step + 1)
            if (step + 1) % a.log_every == 0:
                _, loss, step = sess.run([train_op, train_op.loss, global_step], feed_dict={images: x, labels: y})
                if is_chief:
                    print("step %d loss %.4f" % (step, float(loss)), flush=True)
            else:
                _, step = sess.run([train_op, global_step], feed_dict={images: x, labels: y})
            step = int(step)
    comm.barrier()
    if is_chief:
        print("done at global step %d" % step, flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
