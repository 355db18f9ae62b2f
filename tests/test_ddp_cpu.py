"""All-reduce data parallelism (parallel/ddp.py) with 2 gloo ranks on the CPU: bucketed,
hook-driven all-reduce must give exactly the full-batch gradient (DP equivalence), and the fused
flat optimizer must keep replicas bit-identical."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mlp():
    import dtg  # noqa: F401
    from dtg.models.layers import Linear

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = Linear(16, 32, act="relu")
            self.b = Linear(32, 32, act="relu")
            self.c = Linear(32, 4)

        def forward(self, x):
            return self.c(self.b(self.a(x)))
    return M()


def _rank(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import dtg  # noqa: F401
        from dtg import ops
        from dtg.optim import FusedSGD
        from dtg.parallel import DataParallel, FlatParams, comm
        comm.init("gloo")
        torch.manual_seed(0)
        ref = _mlp()
        torch.manual_seed(0)
        model = _mlp()
        flat = FlatParams(model, compute_dtype=torch.float32)
        dp = DataParallel(flat, bucket_mb=0.001)  # tiny buckets: several all-reduces in flight
        assert len(dp.buckets) > 2
        dp.broadcast_parameters(0)
        opt = FusedSGD(flat, lr=0.1, momentum=0.9)
        g = torch.Generator().manual_seed(1)
        x = torch.randn(8 * world, 16, generator=g)
        y = torch.randint(0, 4, (8 * world,), generator=g)
        shard = slice(8 * rank, 8 * (rank + 1))
        loss = ops.softmax_cross_entropy(model(x[shard]), y[shard])
        loss.backward()
        dp.finish()
        # reference: full batch, single process
        full = ops.softmax_cross_entropy(ref(x), y)
        full.backward()
        for (n, p), (_, pr) in zip(model.named_parameters(), ref.named_parameters()):
            got = p.grad * dp.grad_scale
            assert torch.allclose(got, pr.grad, atol=1e-5, rtol=1e-4), (n, (got - pr.grad).abs().max())
        opt.step(dp.grad_scale)
        # replicas stay identical after the step
        w = flat.groups["compute"].master.clone()
        ws = [torch.empty_like(w) for _ in range(world)]
        dist.all_gather(ws, w)
        assert all(torch.equal(ws[0], v) for v in ws)
        assert flat.groups["compute"].grad.abs().sum() == 0  # zeroed by the fused apply
        comm.shutdown()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_allreduce_dp_equivalence_two_ranks():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: "ok", 1: "ok"}, res


class _DirectMul(__import__("torch").autograd.Function):
    """y = x * w with w's gradient written straight into its flat view + grad_sink.notify (the
    fused GPU ops' contract); returns None for w, so autograd still runs w's AccumulateGrad."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x * w

    @staticmethod
    def backward(ctx, dy):
        from dtg.parallel import grad_sink
        x, w = ctx.saved_tensors
        w.grad.add_((dy * x).sum(0))
        grad_sink.notify(w)
        return dy * w, None


def _rank_direct(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import dtg  # noqa: F401
        from dtg.parallel import DataParallel, FlatParams, comm
        comm.init("gloo")

        class M(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.ws = torch.nn.ParameterList([torch.nn.Parameter(torch.full((64,), 1.0 + i)) for i in range(4)])

            def forward(self, x):
                for w in self.ws:
                    x = _DirectMul.apply(x, w)
                return x

        model = M()
        flat = FlatParams(model, compute_dtype=torch.float32, keep_fp32=lambda n, p: False)
        dp = DataParallel(flat, bucket_mb=1.0)  # ONE bucket holding all four parameters
        assert len(dp.buckets) == 1
        launched_with = []
        real_launch = dp._launch

        def spy(b):
            launched_with.append(len(dp._done))
            real_launch(b)
        dp._launch = spy
        x = torch.ones(2, 64) * (rank + 1)
        for _ in range(2):  # twice: the per-step bookkeeping must reset
            flat.zero_grad()
            model(x).sum().backward()
            dp.finish()
        # the bucket's all-reduce may only start once all four gradients are written
        assert launched_with == [4, 4], launched_with
        comm.shutdown()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_direct_write_params_count_once():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_direct, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: "ok", 1: "ok"}, res


def test_allreduce_bw_tool_gloo(tmp_path):
    """tools/allreduce_bw.py runs end to end on 2 gloo ranks and reports sane bandwidth rows."""
    import json as _json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "bw.jsonl"
    sys.path.insert(0, os.path.join(root, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(root, "tools", "allreduce_bw.py"), "--min_kb", "4",
           "--max_mb", "0.25", "--iters", "3", "--warmup", "1", "--bucket_mb", "40", "--json", str(out)]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = [_json.loads(line) for line in out.read_text().splitlines()]
    assert len(rows) >= 7 and all(x["n_ranks"] == 2 and x["us"] > 0 and x["busbw_GBs"] > 0 for x in rows)
    assert rows[-1]["tag"].startswith("resnet50_bucket")


def _rank_step(rank, world, port, q):
    """DataParallel.step (apply per bucket as each all-reduce lands) == finish() + opt.step(), bit for bit, over
    two steps with momentum / Adam / Adagrad (several buckets, the fp32 and compute groups; Adagrad's accumulator
    must start at 0.1 in every bucket slice, not only the first)."""
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import dtg  # noqa: F401
        from dtg import ops
        from dtg.optim import FusedAdagrad, FusedAdam, FusedSGD
        from dtg.parallel import DataParallel, FlatParams, comm
        comm.init("gloo")
        for Opt in (FusedSGD, FusedAdam, FusedAdagrad):
            runs = []
            for mode in ("step", "finish"):
                torch.manual_seed(0)
                model = _mlp()
                flat = FlatParams(model, compute_dtype=torch.float32)
                dp = DataParallel(flat, bucket_mb=0.001)
                assert len(dp.buckets) > 2
                dp.broadcast_parameters(0)
                opt = Opt(flat, lr=0.05)
                g = torch.Generator().manual_seed(1 + rank)
                for _ in range(2):
                    x = torch.randn(8, 16, generator=g)
                    y = torch.randint(0, 4, (8,), generator=g)
                    ops.softmax_cross_entropy(model(x), y).backward()
                    if mode == "step":
                        dp.step(opt)
                    else:
                        dp.finish()
                        opt.step(grad_scale=dp.grad_scale)
                runs.append([p.detach().clone() for p in model.parameters()] +
                            [grp.master.clone() for grp in flat])
                dp.remove_hooks()
            assert all(torch.equal(a, b) for a, b in zip(*runs)), Opt.__name__
            assert all(torch.isfinite(t).all() for t in runs[0]), Opt.__name__
        comm.shutdown()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_dp_step_overlapped_apply_equals_finish_then_step():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_step, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: "ok", 1: "ok"}, res
