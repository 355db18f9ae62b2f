#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): ResNet-50 bf16 synchronous all-reduce data parallelism,
images/sec for the whole job, one process per MI355X (RCCL over xGMI).

    python bench.py --gpus N --steps K --warmup W            (N=1 runs in-process)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K --warmup W

Weak scaling: every GPU trains a fixed per-GPU batch (default 1024 images of 224x224, synthetic
data, random-init weights).  ``--model bert`` measures BASELINE.json config 5 instead (BERT-base
pre-training, MLM + NSP, seq 128, per-GPU batch 256, fused Adam; sequences/sec).

Per-GPU batch: sized for 288 GB of HBM3E rather than for an 80 GB part.  A bigger shard amortises
the per-launch and per-tile fixed costs of every kernel, and it halves the gradient bytes
all-reduced per image (one model's gradients per step, whatever the batch).  Measured on one MI355X
(profiles/r02_batch):

- ResNet-50: 10.5k img/s at 128, 12.1k at 256, 12.9k at 384, 13.4k at 512 (round 2);
  14.56k at 512, 14.87k at 768, 15.05k at 1024 (round 3, one box, profiles/r03_bn2_prologue).  1024 per GPU
  (74 GB peak) is the default: at 8 GPUs that is the global batch of 8192 of large-minibatch SGD
  (linear learning-rate scaling with warmup, Goyal et al. 2017).
- BERT-base: 6.2k seq/s at 64, 7.6k at 128, 8.2k at 256.

``--mode async_ps --gpus N`` measures BASELINE.json config 4 (1 PS + N-1 ResNet-50 workers, RCCL
point-to-point; see ``_async_ps``).  ``--model mnist`` measures BASELINE.json config 2 (MNIST CNN, per-GPU batch 512; a launch-bound step,
so it replays as one hipGraph by default).  ``--batch`` overrides the default.  A timed step is the full training step: forward, fused softmax-xent,
backward with bucketed RCCL all-reduce overlapped, and the fused momentum-SGD apply.  W untimed
warmup steps, then K steps bracketed by barrier + device synchronize on both sides; the job time
is the MAX over ranks; rank 0 prints one JSON line.  With N > 1 the line also carries ``allreduce_probe``:
the all-reduce of the whole gradient and of one bucket timed alone AFTER the timed steps (bus bandwidth
of this job's xGMI links), and the same training step re-timed with the collectives switched off
(``compute_only_ms_per_step``; ``exposed_comm_ms_per_step`` = ms_per_step minus it) -- the scaling curve's
communication side, measured in the driver's own multi-GPU runs.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "images/sec (whole node) ResNet-50 sync DP at 1/2/4/8 MI355X; scaling efficiency"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default 1024 resnet / 256 bert)")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--image", type=int, default=224)
    # all-reduce bucket size: ResNet-50's 51 MB of bf16 gradients in 8 MB buckets (backward order) leaves
    # only the last ~3 MB (layer2/layer1/stem) exposed after backward ends; 32 MB buckets would leave
    # ~20 MB (layer3 onwards) to reduce after the last gradient lands.  BERT (220 MB) uses 25 MB.
    ap.add_argument("--bucket_mb", type=float, default=0.0, help="0: 8 (resnet50) / 25 (bert)")
    ap.add_argument("--lr", type=float, default=0.0)
    ap.add_argument("--model", default="resnet50")
    # whole-step hipGraph replay (parallel/graphs.py; one rank only, multi-rank steps keep their RCCL
    # all-reduce hooks eager).  auto (-1): on for the launch-bound MNIST step; off for ResNet-50 and
    # BERT, which are GPU-bound (>= 99 % kernel-busy): replay measured equal for ResNet-50 (11.93k vs
    # 11.97k img/s) and 2 % slower for BERT (profiles/r02_baselines)
    ap.add_argument("--graph", type=int, default=-1, help="-1 auto, 0 eager, 1 capture")
    # BASELINE.json config 4: ResNet-50 asynchronous parameter server, rank 0 = PS, ranks 1..N-1 = workers
    ap.add_argument("--mode", default="sync", choices=("sync", "async_ps"))
    ap.add_argument("--window", type=int, default=1, help="async_ps: local steps per push (DOWNPOUR/ADAG window)")
    ap.add_argument("--overlap_pull", type=int, default=1, help="async_ps: pull overlapped with the next step")
    ap.add_argument("--window_mode", default="sum", choices=("sum", "mean"),
                    help="async_ps: push the window's sum (DOWNPOUR) or mean (ADAG)")
    ap.add_argument("--local_opt", default="none", choices=("none", "sgd", "adagrad", "momentum"),
                    help="async_ps: worker-local optimizer inside the window (DOWNPOUR: adagrad, ADAG: sgd)")
    ap.add_argument("--local_lr", type=float, default=None, help="async_ps: local optimizer lr (default: --lr)")
    ap.add_argument("--ps_opt", default="momentum", choices=("sgd", "adagrad", "momentum"),
                    help="async_ps: the PS's global optimizer (DOWNPOUR: adagrad, ADAG: sgd)")
    return ap.parse_known_args(argv)[0]


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _self_launch(n, argv):
    """``python bench.py --gpus N`` (N > 1) outside torchrun: start the N rank processes here, one per GPU,
    through torch.distributed.run on 127.0.0.1, before this process touches the GPU (nothing above has
    imported torch).  Rank 0's JSON line reaches our stdout unchanged; the exit code is torchrun's, which is
    non-zero when any rank fails.  Reference semantics: one process per replica, all replicas aggregated
    every step (Synchronous-SGD/ssgd.py:51-55)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def _backend_name():
    """'rccl' for the production path (torch's "nccl" backend is RCCL on ROCm), else the backend."""
    import torch.distributed as dist
    b = dist.get_backend() if dist.is_initialized() else (os.environ.get("DTG_BACKEND") or "nccl")
    return "rccl" if b == "nccl" else b


def main(argv=None):
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(a.gpus, sys.argv[1:] if argv is None else argv))
    import torch
    import dtg  # noqa: F401
    from dtg.models import resnet
    from dtg.parallel import FlatParams, DataParallel, comm
    from dtg.optim import FusedSGD
    from dtg import ops
    from dtg.utils import StepTimer, trace_range

    def train_step(forward_loss, dp, opt):
        """forward -> backward (bucketed all-reduce fired from inside) -> join + fused apply per bucket, with roctx
        ranges around each phase when DTG_TRACE=1 (dtg.utils.trace).  The backward is seeded with a cached
        1.0 (``loss.backward()`` would launch a framework fill kernel for it every step)."""
        seed = []

        def step():
            with trace_range("dtg.forward"):
                loss = forward_loss()
            if not seed:
                seed.append(torch.ones_like(loss))
            with trace_range("dtg.backward"):
                loss.backward(seed[0])
            with trace_range("dtg.allreduce.join"):
                # finish + apply, each bucket's slice applied as soon as its all-reduce has landed (parallel/ddp.py
                # DataParallel.step): the applies overlap the collective tail
                dp.step(opt)
            return loss
        return step

    # async PS survives a lost worker on its own: no fail-stop rank watchdog there
    rank, local, world, device = comm.init("nccl" if torch.cuda.is_available() else "gloo",
                                           watchdog=a.mode != "async_ps")
    if world != a.gpus:
        # a mislabelled point on the scaling curve is worse than no point
        comm.shutdown()
        sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if a.mode == "async_ps":
        return _async_ps(a, rank, world, device)
    a.bucket_mb = a.bucket_mb or (25.0 if a.model == "bert" else 8.0)
    torch.manual_seed(1234)
    if device.type == "cuda":
        ops.lib()  # fail loudly if the HIP kernels are missing
    dtype = torch.bfloat16
    if a.model == "mnist":
        from dtg.models.mnist import MnistCNN, synthetic_mnist
        a.batch = a.batch or 512
        model = MnistCNN().to(device)
        flat = FlatParams(model, compute_dtype=dtype)
        dp = DataParallel(flat, bucket_mb=a.bucket_mb)
        dp.broadcast_parameters(0)
        opt = FusedSGD(flat, lr=(a.lr or 0.01) * world, momentum=0.9)
        x, y = synthetic_mnist(a.batch, device, dtype, seed=rank)
        model.train()

        step = train_step(lambda: ops.softmax_cross_entropy(model(x), y), dp, opt)
        metric, unit = "images/sec (whole node) MNIST CNN sync DP", "images/sec"
        conf = {"model": "MNIST CNN (conv5x5-32, conv5x5-64, fc1024, fc10)", "seq_len": None, "image_size": 28,
                "optimizer": "momentum-sgd (fused)"}
    elif a.model == "bert":
        from dtg.models import bert
        from dtg.optim import FusedAdam
        a.batch = a.batch or 256
        cfg = bert.BertConfig.base()
        model = bert.BertForPreTraining(cfg).to(device)
        flat = FlatParams(model, compute_dtype=dtype)
        dp = DataParallel(flat, bucket_mb=a.bucket_mb)
        dp.broadcast_parameters(0)
        opt = FusedAdam(flat, lr=a.lr or 1e-4, weight_decay=0.01)
        batch = bert.synthetic_batch(a.batch, a.seq, cfg, device, max_predictions=20, seed=rank)
        model.train()

        step = train_step(lambda: model(*batch), dp, opt)
        metric, unit = "sequences/sec (whole node) BERT-base pre-training sync DP", "sequences/sec"
        conf = {"model": "BERT-base (MLM+NSP)", "seq_len": a.seq, "optimizer": "adam-wd (fused)"}
    else:
        a.batch = a.batch or 1024
        model = resnet.resnet50().to(device)
        model = model.to(memory_format=torch.channels_last)
        flat = FlatParams(model, compute_dtype=dtype)
        dp = DataParallel(flat, bucket_mb=a.bucket_mb)
        dp.broadcast_parameters(0)
        opt = FusedSGD(flat, lr=(a.lr or 0.1) * world, momentum=0.9, weight_decay=5e-5)
        x, y = resnet.synthetic_batch(a.batch, device, dtype, a.image, 1000, seed=rank)
        model.train()

        step = train_step(lambda: ops.softmax_cross_entropy(model(x), y), dp, opt)
        metric, unit = METRIC, "images/sec"
        conf = {"model": "ResNet-50", "seq_len": None, "image_size": a.image, "optimizer": "momentum-sgd (fused)"}

    from dtg.parallel import GraphedStep, capture_supported
    use_graph = (a.graph == 1 or (a.graph == -1 and a.model == "mnist" and capture_supported(world))) \
        and device.type == "cuda"
    if use_graph:
        # warmup = eager steps on a side stream + the capture; the rest of the warmup replays
        step = GraphedStep(step, warmup=min(2, max(a.warmup - 1, 1)))
    main_prio = os.environ.get("DTG_MAIN_PRIO")
    if (main_prio is None and a.model == "bert" and world == 1 and os.environ.get("DTG_DDP_FORCE") != "1"
            and "DTG_SIDE_PRIO" not in os.environ and not use_graph):
        # BERT on one rank (no collective stream): the main stream (data gradients, LayerNorm, attention -- the
        # critical path) on the high-priority queue and the weight-gradient side stream at normal priority, so
        # the side stream's compute-bound GEMMs fill in around the main stream instead of taking CUs from it:
        # 9,466 vs 9,345 seq/s (profiles/r05_stream_prio/ab_bert_prio.log).  ResNet-50 measured the opposite
        # (its side stream must keep pace with a memory-bound main stream), and with ranks > 1 the process
        # group's high-priority stream needs its own queue, so both keep the default order.  Not under a graph
        # replay (--graph 1): the main stream is not re-created there, so only the side stream would move.
        from dtg.parallel import overlap as _ov
        _ov.set_side_priority(0)
        main_prio = "-1"
    if main_prio is not None and device.type == "cuda" and not use_graph:
        # the whole step on a stream of this priority (A/B of the main / side stream priorities, DTG_SIDE_PRIO)
        ms = torch.cuda.Stream(device=device, priority=int(main_prio))
        ms.wait_stream(torch.cuda.current_stream(device))
        step0 = step

        def step():
            with torch.cuda.stream(ms):
                return step0()
        print(f"main stream priority {int(main_prio)}, range {torch.cuda.Stream.priority_range()}", file=sys.stderr)
    for _ in range(a.warmup):
        loss = step()
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    sync()
    comm.barrier()
    sync()
    # per-step GPU times from HIP events (dtg.utils.StepTimer: read back after the loop, no sync inside)
    diag = StepTimer(batch_size=a.batch, device=device) if os.environ.get("DTG_BENCH_DIAG") == "1" else None
    if device.type == "cuda":
        torch.cuda.reset_peak_memory_stats(device)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if diag:
            diag.start()
        loss = step()
        if diag:
            diag.stop()
    sync()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt = comm.all_reduce_max(dt, device)
    final_loss = float(loss.float().item())
    if diag:
        print(f"rank {rank} step times: {diag.times_ms()}  {diag.summary()}", file=sys.stderr, flush=True)
    if device.type == "cuda":  # allocator health (a cudaMalloc retry inside the timed loop synchronises it)
        ms = torch.cuda.memory_stats(device)
        print(f"rank {rank} memory: peak reserved {ms.get('reserved_bytes.all.peak', 0) / 2**30:.1f} GiB, "
              f"peak allocated {ms.get('allocated_bytes.all.peak', 0) / 2**30:.1f} GiB, "
              f"alloc retries {ms.get('num_alloc_retries', 0)}, device mallocs {ms.get('num_device_alloc', 0)}",
              file=sys.stderr, flush=True)
    gb = a.batch * world
    ips = gb * a.steps / dt
    probe = None
    if world > 1:
        probe = _allreduce_probe(dp, a.bucket_mb, world, device, sync)
    emu = dp.emulate  # DTG_COMM_EMULATE (parallel/ddp.py): one-card stand-in for an N-rank all-reduce
    if (world > 1 or emu) and not use_graph:
        probe = probe or ({"comm_emulate": emu} if emu else {})
        # the same step with the collectives switched off, timed like the real one (after it, outside it):
        # ms_per_step - compute_only_ms = communication the overlap did not hide
        n_co = min(a.steps, 10)
        dp.set_comm(False)
        step()
        sync()
        comm.barrier()
        sync()
        t1 = time.perf_counter()
        for _ in range(n_co):
            step()
        sync()
        comm.barrier()
        sync()
        co = comm.all_reduce_max(time.perf_counter() - t1, device) / n_co
        dp.set_comm(True)
        probe["compute_only_ms_per_step"] = round(co * 1e3, 3)
        probe["exposed_comm_ms_per_step"] = round(dt / a.steps * 1e3 - co * 1e3, 3)
    if rank == 0:
        config = {"model": conf["model"], "global_batch": gb, "per_gpu_batch": a.batch, "seq_len": conf["seq_len"]}
        config.update({k: v for k, v in conf.items() if k not in config})
        config.update({"parallelism": f"dp{world}", "allreduce": f"{_backend_name()} bf16, {a.bucket_mb:g} MB buckets, overlapped",
                       "step_launch": "hipGraph replay" if use_graph else "eager"})
        print(json.dumps({
            "metric": metric, "value": round(ips, 2), "unit": unit, "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init weights)", "config": config,
            "final_loss": final_loss, **({"allreduce_probe": probe} if probe else {})}), flush=True)
    comm.shutdown()


def _allreduce_probe(dp, bucket_mb, world, device, sync):
    """After the timed steps (outside them): the collective alone, on this job's links -- one all-reduce of
    the whole gradient (its bytes and dtype) and one of a single bucket, each the median of 5 after 2
    warm-ups, as algorithm time and bus bandwidth (algbw x 2(N-1)/N, the ring-equivalent per-link rate;
    SURVEY §7.5 item 7: report busbw next to images/sec, since 2-, 4- and 8-GPU subsets of the xGMI mesh
    have 1, 3 and 7 links per GPU)."""
    import torch
    import torch.distributed as dist
    from dtg.parallel import comm
    grads = [g.grad for g in dp.flat]
    nbytes = sum(t.numel() * t.element_size() for t in grads)
    dt_ = grads[0].dtype
    out = {"grad_bytes": nbytes, "dtype": str(dt_).replace("torch.", "")}
    for name, n in (("full", nbytes), ("bucket", min(nbytes, int(bucket_mb * (1 << 20))))):
        buf = torch.zeros(max(1, n // grads[0].element_size()), dtype=dt_, device=device)
        times = []
        for i in range(7):
            sync()
            comm.barrier()
            t0 = time.perf_counter()
            dist.all_reduce(buf)
            sync()
            if i >= 2:
                times.append(time.perf_counter() - t0)
        t = comm.all_reduce_max(sorted(times)[len(times) // 2], device)
        out[f"{name}_ms"] = round(t * 1e3, 3)
        out[f"{name}_busbw_GBps"] = round(n / t / 1e9 * 2 * (world - 1) / world, 1)
        del buf
    return out


def _async_ps(a, rank, world, device):
    """BASELINE.json config 4: 1 PS + (N-1) ResNet-50 workers, Hogwild by default
    (``--window T``: sum (DOWNPOUR) or ``--window_mode mean`` (ADAG) of T local gradients per push, with
    ``--local_opt adagrad|sgd`` taking T - 1 worker-local optimizer steps inside the window and ``--ps_opt`` the
    PS's global rule -- DOWNPOUR = ``--local_opt adagrad --ps_opt adagrad``).  The PS rank owns a GPU and the
    parameters; workers push gradients and pull parameters over RCCL point-to-point (parallel/async_ps.py).
    Whole-node images/sec = PS-applied updates x images per update / wall time, counted on the PS from the
    moment every worker has finished its W warm-up steps (a device synchronize on the PS brackets both
    ends), so PS queueing and transfer stalls are inside the number.  Reference semantics: Hogwild/Hogwild.py:44-57,
    DOWNPOUR/DOWNPOUR.py:96-102."""
    import torch
    from dtg import ops
    from dtg.models import resnet
    from dtg.optim import make_optimizer
    from dtg.parallel import FlatParams, comm
    from dtg.parallel.async_ps import AsyncPSServer, AsyncPSWorker
    if world < 2:
        comm.shutdown()
        sys.exit("bench.py --mode async_ps needs --gpus >= 2 (one PS rank + workers)")
    if device.type == "cuda":
        from dtg import ops as _ops
        _ops.lib()
    a.batch = a.batch or 512
    torch.manual_seed(1234)
    model = resnet.resnet50().to(device).to(memory_format=torch.channels_last)
    flat = FlatParams(model)
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    lr = a.lr or 0.1
    if rank == 0:
        opt = make_optimizer(a.ps_opt, flat, lr, momentum=0.9, weight_decay=5e-5)
        ps = AsyncPSServer(flat, opt, workers=range(1, world), window=a.window, window_mode=a.window_mode,
                           staleness_log=True)
        ps.serve()
        (u0, t0), (u1, t1) = ps.timed or ps.timed_end, ps.timed_end
        imgs = (u1 - u0) * a.batch * a.window
        ips = imgs / max(t1 - t0, 1e-9)
        st = ps.staleness[u0:] or [0]
        print(json.dumps({
            "metric": "images/sec (whole node) ResNet-50 async PS, 1 PS + %d workers" % (world - 1),
            "value": round(ips, 2), "unit": "images/sec", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round((t1 - t0) / max(1, (u1 - u0) / (world - 1)) * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic (random-init weights)",
            "config": {"model": "ResNet-50", "per_gpu_batch": a.batch, "global_batch": a.batch * (world - 1),
                       "image_size": a.image, "parallelism": "ps1+w%d" % (world - 1),
                       "transport": "rccl p2p" if _backend_name() == "rccl" else _backend_name(),
                       "window": a.window, "window_mode": a.window_mode, "local_opt": a.local_opt,
                       "overlap_pull": bool(a.overlap_pull), "optimizer": "%s (fused, on PS)" % a.ps_opt},
            "updates_timed": u1 - u0, "per_worker": {str(k): v for k, v in ps.per_worker.items()},
            "mean_staleness": round(sum(st) / len(st), 3), "lost_workers": ps.lost}), flush=True)
        ps.close()
    else:
        local = make_optimizer(a.local_opt, flat, a.local_lr or lr) if a.window > 1 else None
        w = AsyncPSWorker(flat, ps_rank=0, window=a.window, window_mode=a.window_mode, local_optimizer=local,
                          overlap_pull=bool(a.overlap_pull))
        x, y = resnet.synthetic_batch(a.batch, device, dtype, a.image, 1000, seed=rank)
        model.train()
        w.begin()
        for i in range(a.warmup + a.steps):
            if i == a.warmup:
                w.warm()
            ops.softmax_cross_entropy(model(x), y).backward()
            w.step_done()
        w.finish()
    comm.shutdown()


if __name__ == "__main__":
    main()
