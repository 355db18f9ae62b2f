#!/usr/bin/env python3
"""Multi-rank correctness checks of the distributed paths, one process per rank (SURVEY §4.2 "Distributed
(GPU)"; reference: data parallelism, README.md:10; async PS, Hogwild/Hogwild.py:44-57):

* allreduce  -- the collective's sum equals the host sum of every rank's tensor (several sizes);
* dp_resnet  -- DataParallel over a 4-block ResNet (fused bottlenecks, BN per replica): N ranks x batch B
                give the mean of the N per-shard gradients, computed here on one process shard by shard;
* dp_bert    -- DataParallel over a 2-layer BERT (dropout off): N ranks x B equals ONE process on the
                full N*B batch;
* async_ps   -- 1 PS + (N-1) workers: every pushed gradient is applied exactly once, and the PS parameters
                equal a replay of the pushed gradients in the PS's logged order.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/multigpu_checks.py
    (RCCL, one GPU per rank; DTG_BACKEND=gloo DTG_GLOO_DEVICE=cuda rehearses it with N ranks on one card)

Rank 0 prints one JSON line {"ok": bool, "world": N, "backend": ..., "checks": {...}}; exit code 1 on failure.
"""
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dtg  # noqa: E402,F401
from dtg import ops  # noqa: E402
from dtg.parallel import DataParallel, FlatParams, comm  # noqa: E402


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def check_allreduce(rank, world, device):
    worst = 0.0
    for n in (1, 1000, 1 << 20, 5_000_001):
        g = torch.Generator().manual_seed(100 + n)
        full = torch.randn(world, n, generator=g)
        t = full[rank].clone().to(device)
        dist.all_reduce(t)
        worst = max(worst, (t.cpu() - full.sum(0)).abs().max().item())
    assert worst < 1e-4, worst
    return {"max_abs_err": worst}


def _resnet(device):
    from dtg.models.resnet import ResNet
    torch.manual_seed(0)
    m = ResNet((1, 1, 1, 1), 10, width=64).to(device).to(memory_format=torch.channels_last)
    for mod in m.modules():
        if isinstance(mod, dtg.models.layers.BatchNorm2d):
            mod.weight.data.fill_(1.0)  # c3's zero init would leave the residual branches without gradient
    return m.train()


def check_dp_resnet(rank, world, device, B=8):
    from dtg.models import resnet
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    x, y = resnet.synthetic_batch(B * world, device, dtype, 32, 10, seed=5)
    model = _resnet(device)
    flat = FlatParams(model, compute_dtype=dtype)
    dp = DataParallel(flat, bucket_mb=0.25)  # several buckets in flight
    dp.broadcast_parameters(0)
    sl = slice(B * rank, B * (rank + 1))
    ops.softmax_cross_entropy(model(x[sl]), y[sl]).backward()
    dp.finish()
    got = {n: p.grad.float() * dp.grad_scale for n, p in model.named_parameters()}
    dp.remove_hooks()
    ref = _resnet(device)
    FlatParams(ref, compute_dtype=dtype)
    for r in range(world):  # the same N shards, one after another, gradients accumulated
        s = slice(B * r, B * (r + 1))
        ops.softmax_cross_entropy(ref(x[s]), y[s]).backward()
    errs = {n: _rel(got[n], p.grad.float() / world) for n, p in ref.named_parameters()}
    worst = max(errs.values())
    assert worst < 3e-2, sorted(errs.items(), key=lambda kv: -kv[1])[:4]
    return {"max_rel_err": worst, "buckets": len(dp.buckets)}


def check_dp_bert(rank, world, device, B=4, S=64):
    from dtg.models import bert
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    cfg = bert.BertConfig(vocab_size=1024, hidden=128, layers=2, heads=2, intermediate=512, max_position=S,
                          dropout=0.0, attn_dropout=0.0)

    def build():
        torch.manual_seed(0)
        return bert.BertForPreTraining(cfg).to(device).train()

    full = bert.synthetic_batch(B * world, S, cfg, device, max_predictions=8, seed=9)
    model = build()
    flat = FlatParams(model, compute_dtype=dtype)
    dp = DataParallel(flat, bucket_mb=0.5)
    dp.broadcast_parameters(0)
    sl = slice(B * rank, B * (rank + 1))
    model(*[t[sl] for t in full]).backward()
    dp.finish()
    got = {n: p.grad.float() * dp.grad_scale for n, p in model.named_parameters()}
    dp.remove_hooks()
    ref = build()
    FlatParams(ref, compute_dtype=dtype)
    ref(*full).backward()
    errs = {n: _rel(got[n], p.grad) for n, p in ref.named_parameters() if p.grad.float().norm() > 0}
    worst = max(errs.values())
    assert worst < 5e-2, sorted(errs.items(), key=lambda kv: -kv[1])[:4]
    return {"max_rel_err": worst}


def check_async_ps(rank, world, device, steps=5):
    """1 PS + (N-1) workers: every push applied once, AND the PS parameters equal a replay of the pushed
    gradients in the order the PS logged (AsyncPSServer.order): each worker records what it pushed and
    sends it to the PS after the run, the PS re-applies them to its initial parameters with the same SGD."""
    from dtg.models.layers import Linear
    from dtg.optim import FusedSGD
    from dtg.parallel.async_ps import AsyncPSServer, AsyncPSWorker, _irecv, _isend, _wait_all
    torch.manual_seed(0)
    model = torch.nn.Sequential(Linear(64, 128, act="relu"), Linear(128, 10)).to(device)
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    flat = FlatParams(model, compute_dtype=dtype)
    lr = 0.05
    if rank == 0:
        init = [g.master.clone() for g in flat]
        ps = AsyncPSServer(flat, FusedSGD(flat, lr=lr, momentum=0.0), workers=range(1, world))
        n = ps.serve()
        ps.close()
        expect = {w: steps for w in range(1, world)}
        assert n == steps * (world - 1) and ps.per_worker == expect and not ps.lost, (n, ps.per_worker, ps.lost)
        pushed = {w: [[torch.empty_like(g.grad) for g in flat] for _ in range(steps)] for w in range(1, world)}
        _wait_all([_irecv(t, w, None) for w in pushed for gs in pushed[w] for t in gs])
        rep = [m.clone() for m in init]
        for w, i in ps.order:  # the PS's applied order
            for m, gr in zip(rep, pushed[w][i]):
                m.sub_(lr * gr.float())
        err = max(((m - r).abs().max() / (r.abs().max() + 1e-12)).item() for m, r in
                  zip([g.master for g in flat], rep))
        assert err < 1e-5, err
        return {"updates": n, "replay_max_rel_err": err, "order_head": ps.order[:8]}
    w = AsyncPSWorker(flat, ps_rank=0, overlap_pull=rank % 2 == 0)
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(32, 64, generator=g).to(device, dtype)
    y = torch.randint(0, 10, (32,), generator=g).to(device)
    w.begin()
    pushed = []
    for _ in range(steps):
        ops.softmax_cross_entropy(model(x), y).backward()
        pushed.append([gr.grad.clone() for gr in flat])  # what step_done pushes (window 1)
        w.step_done()
    w.finish()
    _wait_all([_isend(t, 0, None) for gs in pushed for t in gs])
    return {"pushes": w.pushes}


CHECKS = {"allreduce": check_allreduce, "dp_resnet": check_dp_resnet, "dp_bert": check_dp_bert,
          "async_ps": check_async_ps}


def main():
    names = [a for a in sys.argv[1:] if not a.startswith("-")] or list(CHECKS)
    rank, _, world, device = comm.init()
    res, ok = {}, True
    for name in names:
        try:
            res[name] = CHECKS[name](rank, world, device)
        except Exception:
            ok = False
            res[name] = {"error": traceback.format_exc()[-1500:]}
        if device.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()
    flags = torch.tensor([0.0 if ok else 1.0], device=device)
    dist.all_reduce(flags)
    ok = flags.item() == 0
    if not all("error" not in v for v in res.values()):
        print(json.dumps({"rank": rank, "checks": res}), file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps({"ok": ok, "world": world, "backend": dist.get_backend(), "device": str(device),
                          "checks": res}), flush=True)
    comm.shutdown()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
