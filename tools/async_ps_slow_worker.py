#!/usr/bin/env python3
"""Async PS with one slowed worker (parallel/async_ps.py GPU-ready request order, verdict r4 item 4).

1 PS + W workers as processes on one machine; the workers train a small MLP for ``--seconds``; worker k of
``DTG_APS_TEST_SLOW="k:secs"`` delays each of its gradients by a device spin of ``secs`` (comm_spin on its
compute stream: the gradient exists on the device only that much later, its host is not blocked).  The PS
prints one JSON line with its per-worker update counts: under Hogwild the fast workers should take
proportionally more updates, not wait for the slow one.

    DTG_BACKEND=gloo DTG_GLOO_DEVICE=cuda python tools/async_ps_slow_worker.py --workers 3 --seconds 6
    (RCCL, one GPU per rank: DTG_BACKEND=nccl on a node with >= W+1 GPUs)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, port, seconds, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import torch
        import dtg  # noqa: F401
        from dtg import ops
        from dtg.models.layers import Linear
        from dtg.ops import lib
        from dtg.optim import FusedSGD
        from dtg.parallel import FlatParams, comm
        from dtg.parallel.async_ps import AsyncPSServer, AsyncPSWorker
        _, _, _, device = comm.init()
        torch.set_num_threads(1)  # W+1 ranks share the host's cores
        torch.manual_seed(0)
        model = torch.nn.Sequential(Linear(256, 512, act="relu"), Linear(512, 10)).to(device)
        flat = FlatParams(model, compute_dtype=torch.bfloat16 if device.type == "cuda" else torch.float32)
        slow = os.environ.get("DTG_APS_TEST_SLOW", "")
        slow_rank, slow_s = (int(slow.split(":")[0]), float(slow.split(":")[1])) if slow else (-1, 0.0)
        if rank == 0:
            ps = AsyncPSServer(flat, FusedSGD(flat, lr=0.01, momentum=0.0), workers=range(1, world),
                               staleness_log=True)
            n = ps.serve()
            q.put((rank, "ok", {"updates": n, "per_worker": ps.per_worker, "lost": ps.lost,
                                "mean_staleness": sum(ps.staleness) / max(1, len(ps.staleness))}))
            ps.close()
        else:
            w = AsyncPSWorker(flat, ps_rank=0)
            g = torch.Generator().manual_seed(rank)
            dt = torch.bfloat16 if device.type == "cuda" else torch.float32
            x = torch.randn(64, 256, generator=g).to(device, dt)
            y = torch.randint(0, 10, (64,), generator=g).to(device)
            w.begin()
            t_end = time.time() + seconds
            while time.time() < t_end:
                ops.softmax_cross_entropy(model(x), y).backward()
                if rank == slow_rank and device.type == "cuda":
                    lib().comm_spin(slow_s, 1, 0)  # this gradient "exists" slow_s later on the device
                elif rank == slow_rank:
                    time.sleep(slow_s)
                w.step_done()
            w.finish()
            q.put((rank, "ok", {"pushes": w.pushes}))
        comm.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None))
        raise


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=6.0)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    world = 1 + args.workers
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, args.seconds, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, status, payload = q.get(timeout=180)
        if status != "ok":
            print(status, file=sys.stderr)
            sys.exit(1)
        out[r] = payload
    for p in procs:
        p.join(timeout=60)
    ps = out[0]
    assert sum(out[r]["pushes"] for r in range(1, world)) == ps["updates"], out
    print(json.dumps({"per_worker": ps["per_worker"], "lost": ps["lost"], "updates": ps["updates"],
                      "mean_staleness": ps["mean_staleness"], "slow": os.environ.get("DTG_APS_TEST_SLOW", "")}))


if __name__ == "__main__":
    main()
