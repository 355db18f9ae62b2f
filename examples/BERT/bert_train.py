"""BERT pre-training (MLM + NSP) as a training job on the reference's session surface (BASELINE.json config 5;
SURVEY §7.4).  Synthetic token batches of BERT's input signature (no dataset offline), random-init weights.

Same structure as /root/reference/Synchronous-SGD/ssgd.py:51-69 and /root/reference/DOWNPOUR/DOWNPOUR.py:116-127:
``SyncReplicasOptimizer`` (all-reduce mode: no PS, one process per GPU over RCCL) wrapping the fused AdamW
(dtg.optim.FusedAdam), a linear-warmup / linear-decay learning rate, ``MonitoredTrainingSession`` with
StopAtStepHook, a StepCounterHook reporting sequences/sec per worker and for the whole job, and a checkpoint
directory: the chief saves every ``--save_every`` steps (TensorBundle keyed by parameter name, AdamW slots
``<param>/m`` / ``<param>/v``, ``optimizer/step``, ``global_step``); a restarted job resumes from the latest
checkpoint at its global step, with the same learning-rate schedule position and dropout seeds.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bert_train.py \\
        --steps 1000 --ckpt_dir /path/to/ckpt
    python bert_train.py --tiny --steps 20 --ckpt_dir /tmp/bert_ck        # CPU, 2-layer model
"""
import argparse

import _path  # noqa: F401

import torch

import dtg
from dtg.models import bert
from dtg.optim import FusedAdam
from dtg.parallel import FlatParams, comm


def lr_at(step, base, warmup, total):
    """BERT's schedule: linear warmup to ``base`` over ``warmup`` steps, then linear decay to 0 at ``total``."""
    if step < warmup:
        return base * (step + 1) / warmup
    return base * max(0.0, (total - step) / max(1, total - warmup))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000, help="last global step (absolute, like StopAtStepHook)")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU sequences")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--ckpt_dir", default="bert_logdir")
    ap.add_argument("--save_every", type=int, default=200)
    ap.add_argument("--log_every", type=int, default=20)
    ap.add_argument("--tiny", action="store_true", help="2-layer, 64-wide BERT (CPU tests)")
    a, _ = ap.parse_known_args()
    rank, _, world, device = comm.init()
    is_chief = rank == 0
    cfg = bert.BertConfig.tiny() if a.tiny else bert.BertConfig.base()
    if a.tiny:
        a.seq = min(a.seq, 32)
    torch.manual_seed(1234)
    model = bert.BertForPreTraining(cfg).to(device)
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    flat = FlatParams(model, compute_dtype=dtype)
    model.train()

    batch_ph = [dtg.placeholder(name=n) for n in ("input_ids", "token_type_ids", "attention_mask",
                                                  "masked_lm_positions", "masked_lm_ids", "next_sentence_labels")]
    global_step = dtg.train.get_or_create_global_step()
    adam = FusedAdam(flat, lr=a.lr, weight_decay=0.01)
    opt = dtg.train.SyncReplicasOptimizer(adam, replicas_to_aggregate=world, total_num_replicas=world, bucket_mb=25.0)
    train_op = opt.minimize(lambda *b: model(*b), global_step=global_step, inputs=batch_ph)
    hooks = [opt.make_session_run_hook(is_chief), dtg.train.StopAtStepHook(last_step=a.steps),
             dtg.train.StepCounterHook(every_n_steps=a.log_every, batch_size=a.batch, aggregate=True, log=is_chief)]
    with dtg.train.MonitoredTrainingSession(is_chief=is_chief, checkpoint_dir=a.ckpt_dir, hooks=hooks,
                                            save_checkpoint_secs=None, save_checkpoint_steps=a.save_every,
                                            log_step_count_steps=None, save_summaries_steps=None) as sess:
        step = int(sess.run(global_step))
        model._step = step  # dropout seeds follow the global step across a resume
        if is_chief and sess.restored_from:
            print("resumed from %s (global step %d)" % (sess.restored_from, step), flush=True)
        while not sess.should_stop():
            adam.set_lr(lr_at(step, a.lr, a.warmup, a.steps))  # a device-side scalar: no sync
            b = bert.synthetic_batch(a.batch, a.seq, cfg, device, max_predictions=20, seed=step * 1000 + rank)
            feed = dict(zip(batch_ph, b))
            if (step + 1) % a.log_every == 0:
                _, loss, step = sess.run([train_op, train_op.loss, global_step], feed_dict=feed)
                if is_chief:
                    print("step %d loss %.4f lr %.3g" % (step, float(loss), adam.lr), flush=True)
            else:
                _, step = sess.run([train_op, global_step], feed_dict=feed)
            step = int(step)
    comm.barrier()
    if is_chief:
        print("done at global step %d" % step, flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
