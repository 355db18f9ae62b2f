"""ResNet-50 with an asynchronous parameter server on GPUs (BASELINE.json config 4: 1 PS + 7
workers intra-node, RCCL send/recv).  Same launch idiom as the reference's between-graph scripts
(``--job_name ps|worker --task_index i``, a hard-coded cluster dict; Hogwild/Hogwild.py:20-33),
but the PS owns a GPU and the parameters live in its HBM (dtg.parallel.async_ps).

    bash run_async.sh [--workers 7] [--steps 50] [--window 1]

--window T > 1 pushes every T local steps: --window_mode sum = DOWNPOUR, mean = ADAG.  --local_opt takes T - 1
worker-local optimizer steps inside the window and --ps_opt picks the PS's global rule, as in the reference:

    DOWNPOUR       --window 3 --window_mode sum  --local_opt adagrad --ps_opt adagrad   (DOWNPOUR/DOWNPOUR.py:57, :92)
    DOWNPOUR-Easy  --window 3 --window_mode sum  --local_opt sgd     --ps_opt adagrad   (DOWNPOUR-Easy/DOWNPOUR.py:53)
    ADAG           --window 3 --window_mode mean --local_opt sgd     --ps_opt sgd       (ADAG/ADAG.py:61-63)

Without --local_opt a window sums T gradients taken at the same parameters (SDAG's degenerate window).
"""
import argparse
import time

import _path  # noqa: F401

import torch

import dtg
from dtg import ops
from dtg.models import resnet
from dtg.optim import make_optimizer
from dtg.parallel import FlatParams
from dtg.parallel.async_ps import AsyncPSServer, AsyncPSWorker, init_from_cluster


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--job_name", default="")
    ap.add_argument("--task_index", type=int, default=0)
    ap.add_argument("--workers", type=int, default=7)
    ap.add_argument("--base_port", type=int, default=2222)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--window", type=int, default=1)
    ap.add_argument("--window_mode", default="sum", choices=("sum", "mean"))
    ap.add_argument("--local_opt", default="none", choices=("none", "sgd", "adagrad", "momentum"),
                    help="worker-local optimizer inside the window (T - 1 local steps)")
    ap.add_argument("--local_lr", type=float, default=None, help="local optimizer learning rate (default --lr)")
    ap.add_argument("--ps_opt", default="momentum", choices=("sgd", "adagrad", "momentum"),
                    help="the PS's global optimizer")
    ap.add_argument("--dyn_sgd", action="store_true",
                    help="Dynamic SGD: scale each PS update by 1/(staleness+1) (reference README TODO)")
    ap.add_argument("--overlap_pull", action="store_true",
                    help="pull overlapped with the next step (one extra step of staleness, Hogwild allows it)")
    ap.add_argument("--tiny", action="store_true", help="narrow 4-block ResNet, 32x32 images (CPU smoke tests)")
    a, _ = ap.parse_known_args()
    cluster = {"ps": [f"localhost:{a.base_port}"],
               "worker": [f"localhost:{a.base_port + 1 + i}" for i in range(a.workers)]}
    rank, world, device = init_from_cluster(cluster, a.job_name, a.task_index)
    torch.manual_seed(1234)
    model = (resnet.resnet18_like_tiny(10) if a.tiny else resnet.resnet50()).to(device)
    model = model.to(memory_format=torch.channels_last)
    ncls = 10 if a.tiny else 1000
    flat = FlatParams(model)
    if a.job_name == "ps":
        opt = make_optimizer(a.ps_opt, flat, a.lr, momentum=0.9, weight_decay=5e-5)
        ps = AsyncPSServer(flat, opt, workers=range(1, world), window=a.window, window_mode=a.window_mode,
                           staleness_log=True, staleness_scaling="dyn" if a.dyn_sgd else None)
        t0 = time.time()
        n = ps.serve()
        dt = time.time() - t0
        st = ps.staleness
        print(f"[ps] {n} updates in {dt:.1f}s, per worker {ps.per_worker}, mean staleness "
              f"{sum(st) / max(1, len(st)):.2f}", flush=True)
    else:
        # the reference's worker loop (Hogwild/Hogwild.py:44-57): a train op run under a session until the stop
        # hook fires; the session's hook does the initial pull and tells the PS when this worker is done
        local = make_optimizer(a.local_opt, flat, a.local_lr or a.lr) if a.window > 1 else None
        w = AsyncPSWorker(flat, ps_rank=0, window=a.window, window_mode=a.window_mode, local_optimizer=local,
                          overlap_pull=a.overlap_pull)
        dt_ = torch.bfloat16 if device.type == "cuda" else torch.float32
        x, y = resnet.synthetic_batch(a.batch, device, dt_, a.image, ncls, seed=rank)
        images, labels = dtg.placeholder(name="images"), dtg.placeholder(name="labels")
        global_step = dtg.train.get_or_create_global_step()
        train_op = w.minimize(lambda xb, yb: ops.softmax_cross_entropy(model(xb), yb), global_step=global_step,
                              inputs=(images, labels))
        counter = dtg.train.StepCounterHook(every_n_steps=10, batch_size=a.batch)
        hooks = [w.make_session_run_hook(), dtg.train.StopAtStepHook(last_step=a.steps), counter]
        t0 = time.time()
        with dtg.train.MonitoredTrainingSession(is_chief=False, hooks=hooks, log_step_count_steps=None,
                                                save_summaries_steps=None, save_checkpoint_secs=None) as sess:
            step = 0
            while not sess.should_stop():
                if step % 10 == 0:
                    _, loss, step = sess.run([train_op, train_op.loss, global_step], feed_dict={images: x, labels: y})
                    print(f"[worker {a.task_index}] step {int(step) - 1} loss {float(loss):.4f}", flush=True)
                else:
                    _, step = sess.run([train_op, global_step], feed_dict={images: x, labels: y})
                step = int(step)
            if device.type == "cuda":
                torch.cuda.synchronize()
            dt = time.time() - t0
        print(f"[worker {a.task_index}] {a.steps * a.batch / dt:.1f} images/sec, {w.pushes} pushes", flush=True)


if __name__ == "__main__":
    main()
