"""GPU-style async parameter server (parallel/async_ps.py) exercised with gloo ranks on the CPU.

* 1 PS + 1 worker: asynchronous == sequential, so the PS parameters must equal a local replay;
* 1 PS + 2 workers (Hogwild): every pushed gradient is applied exactly once, both workers learn;
* window=3, mean (ADAG-style): the PS applies steps/3 updates of the averaged gradient.
"""
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model(bn=False):
    import dtg  # noqa: F401
    from dtg.models.layers import BatchNorm2d, Linear

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = Linear(8, 16, act=None if bn else "relu")
            self.n = BatchNorm2d(16) if bn else None
            self.b = Linear(16, 3)

        def forward(self, x):
            h = self.a(x)
            return self.b(self.n(h) if self.n is not None else h)
    torch.manual_seed(0)
    return M()


def _data(seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(32, 8, generator=g), torch.randint(0, 3, (32,), generator=g)


def _rank(rank, world, port, steps, window, mode, q, dyn=False, bn=False):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import dtg  # noqa: F401
        from dtg import ops
        from dtg.optim import FusedSGD
        from dtg.parallel import FlatParams, comm
        from dtg.parallel.async_ps import AsyncPSServer, AsyncPSWorker
        comm.init("gloo")
        model = _model(bn)
        flat = FlatParams(model, compute_dtype=torch.float32)
        # numpy payloads: torch CPU tensors would travel by fd-sharing, which races the child's exit
        bufs = lambda: {n: b.clone().numpy() for n, b in model.named_buffers()}  # noqa: E731
        if rank == 0:
            opt = FusedSGD(flat, lr=0.1, momentum=0.0)
            ps = AsyncPSServer(flat, opt, workers=range(1, world), window=window, window_mode=mode,
                               staleness_log=True, staleness_scaling="dyn" if dyn else None)
            n = ps.serve()
            q.put((rank, "ok", {"updates": n, "per_worker": dict(ps.per_worker),
                                "w": [g.master.clone().numpy() for g in flat],
                                "staleness": list(ps.staleness), "scales": list(ps.scales), "bufs": bufs()}))
        else:
            w = AsyncPSWorker(flat, ps_rank=0, window=window, window_mode=mode)
            w.begin()
            x, y = _data(rank)
            losses = []
            for _ in range(steps):
                loss = ops.softmax_cross_entropy(model(x), y)
                loss.backward()
                w.step_done()
                losses.append(loss.item())
            w.finish()
            q.put((rank, "ok", {"losses": losses, "pushes": w.pushes, "bufs": bufs()}))
        comm.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None))
        raise


def _run(world, steps, window=1, mode="sum", dyn=False, bn=False):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, steps, window, mode, q, dyn, bn)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, status, payload = q.get(timeout=240)
        assert status == "ok", status
        out[r] = payload
    for p in procs:
        p.join(timeout=60)
    return out


def _replay(steps, window, mode, seed=1):
    """Sequential single-worker SGD with the same window rule."""
    import dtg  # noqa: F401
    from dtg import ops
    model = _model()
    x, y = _data(seed)
    params = list(model.parameters())
    acc = [torch.zeros_like(p) for p in params]
    for i in range(steps):
        loss = ops.softmax_cross_entropy(model(x), y)
        grads = torch.autograd.grad(loss, params)
        for a, g in zip(acc, grads):
            a.add_(g)
        if (i + 1) % window == 0:
            scale = 1.0 / window if mode == "mean" else 1.0
            with torch.no_grad():
                for p, a in zip(params, acc):
                    p.sub_(0.1 * scale * a)
                    a.zero_()
    return {n: p.detach() for n, p in model.named_parameters()}


def _ps_params_by_name(out):
    import dtg  # noqa: F401
    from dtg.parallel import FlatParams
    model = _model()
    flat = FlatParams(model, compute_dtype=torch.float32)
    for g, w in zip(flat, out[0]["w"]):
        g.master.copy_(torch.as_tensor(w))
    return dict(flat.named_masters())


def test_async_ps_single_worker_equals_sequential():
    out = _run(2, steps=12)
    assert out[0]["updates"] == 12 and out[1]["pushes"] == 12
    assert all(s == 0 for s in out[0]["staleness"])
    got = _ps_params_by_name(out)
    ref = _replay(12, 1, "sum")
    for n, v in ref.items():
        assert torch.allclose(got[n], v, atol=1e-5), n


def test_async_ps_window_mean_equals_sequential():
    out = _run(2, steps=12, window=3, mode="mean")
    assert out[0]["updates"] == 4
    got = _ps_params_by_name(out)
    ref = _replay(12, 3, "mean")
    for n, v in ref.items():
        assert torch.allclose(got[n], v, atol=1e-5), n


def test_async_ps_two_workers_hogwild():
    out = _run(3, steps=30)
    assert out[0]["updates"] == 60
    assert out[0]["per_worker"] == {1: 30, 2: 30}
    for r in (1, 2):
        ls = out[r]["losses"]
        assert ls[-1] < ls[0], ls


def _elastic_rank(rank, world, port, steps, tau, alpha, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import dtg  # noqa: F401
        from dtg import ops
        from dtg.optim import FusedSGD
        from dtg.parallel import FlatParams, comm
        from dtg.parallel.async_ps import AsyncPSServer, ElasticWorker
        comm.init("gloo")
        model = _model()
        flat = FlatParams(model, compute_dtype=torch.float32)
        if rank == 0:
            ps = AsyncPSServer(flat, None, workers=range(1, world)).enable_elastic(alpha)
            n = ps.serve()
            q.put((rank, "ok", {"updates": n, "w": [g.master.clone().numpy() for g in flat]}))
        else:
            w = ElasticWorker(flat, FusedSGD(flat, lr=0.1, momentum=0.0), tau=tau)
            w.begin()
            x, y = _data(rank)
            losses = []
            for _ in range(steps):
                loss = ops.softmax_cross_entropy(model(x), y)
                loss.backward()
                w.step_done()
                losses.append(loss.item())
            w.finish()
            q.put((rank, "ok", {"losses": losses, "exchanges": w.exchanges}))
        comm.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None))
        raise


def _run_elastic(world, steps, tau, alpha):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_elastic_rank, args=(r, world, port, steps, tau, alpha, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, status, payload = q.get(timeout=240)
        assert status == "ok", status
        out[r] = payload
    for p in procs:
        p.join(timeout=60)
    return out


def test_easgd_single_worker_matches_replay():
    """AEASGD (reference README TODO): with one worker the exchanges are sequential -> exact replay."""
    steps, tau, alpha = 12, 3, 0.5
    out = _run_elastic(2, steps, tau, alpha)
    assert out[0]["updates"] == steps // tau and out[1]["exchanges"] == steps // tau
    import dtg  # noqa: F401
    from dtg import ops
    model = _model()
    center = {n: p.detach().clone() for n, p in model.named_parameters()}
    x, y = _data(1)
    params = dict(model.named_parameters())
    for i in range(steps):
        loss = ops.softmax_cross_entropy(model(x), y)
        grads = torch.autograd.grad(loss, list(params.values()))
        with torch.no_grad():
            for p, g in zip(params.values(), grads):
                p.sub_(0.1 * g)
            if (i + 1) % tau == 0:
                for n, p in params.items():
                    d = alpha * (p - center[n])
                    p.sub_(d)
                    center[n].add_(d)
    got = _ps_params_by_name(out)
    for n, v in center.items():
        assert torch.allclose(got[n], v, atol=1e-5), n


def test_easgd_two_workers_learn():
    out = _run_elastic(3, 24, 4, 0.3)
    assert out[0]["updates"] == 2 * (24 // 4)
    for r in (1, 2):
        assert out[r]["losses"][-1] < out[r]["losses"][0]


def test_dynsgd_scales_updates_by_staleness():
    """Dynamic SGD (reference README TODO): every PS update is scaled by 1/(staleness+1); with one
    worker the staleness is always 0, so it equals the sequential replay; with three workers stale
    pushes occur and are damped accordingly."""
    out = _run(2, steps=8, dyn=True)
    assert set(out[0]["staleness"]) == {0} and all(s == 1.0 for s in out[0]["scales"])
    ref = _replay(8, 1, "sum")
    got = _ps_params_by_name(out)
    for n, p in ref.items():
        assert torch.allclose(got[n], p, atol=1e-5), n
    out = _run(4, steps=10, dyn=True)
    assert out[0]["updates"] == 30
    assert max(out[0]["staleness"]) > 0
    for tau, sc in zip(out[0]["staleness"], out[0]["scales"]):
        assert abs(sc - 1.0 / (tau + 1)) < 1e-12
    # (per-worker losses are not asserted: each worker sees its own shard, so a worker's loss on its
    # shard can rise while the shared model improves on the union)


def test_async_ps_carries_bn_running_stats():
    """BatchNorm running statistics are PS state: the workers' running-mean/var updates
    reach the PS.  One worker: the PS statistics equal the worker's after every step is pushed; two
    workers: the PS statistics move away from their initial (0, 1) values."""
    out = _run(2, steps=6, bn=True)
    ps = {n: torch.as_tensor(v) for n, v in out[0]["bufs"].items()}
    wk = {n: torch.as_tensor(v) for n, v in out[1]["bufs"].items()}
    assert set(ps) == {"n.running_mean", "n.running_var"}
    for n in ps:
        assert torch.allclose(ps[n], wk[n], atol=1e-6), n
    assert ps["n.running_mean"].abs().max() > 1e-3
    out = _run(3, steps=6, bn=True)
    assert out[0]["updates"] == 12
    ps = {n: torch.as_tensor(v) for n, v in out[0]["bufs"].items()}
    assert ps["n.running_mean"].abs().max() > 1e-3
    assert (ps["n.running_var"] - 1).abs().max() > 1e-3


def _rank_opts(rank, world, port, steps, q, overlap=False, die_after=None, timeout=None, stall=None, env=None,
               step_sleep=0.0, duration=None, slow=None):
    """Hogwild ranks with the worker-side options: overlapped pulls, a worker that dies (os._exit, no
    finish) after ``die_after`` steps, a PS ``worker_timeout`` with a worker that stalls; ``env`` extra
    environment (e.g. a short rank-liveness timeout), ``step_sleep`` seconds per worker step; ``duration``: the
    workers step until that many seconds have passed (``steps`` ignored); ``slow`` = (rank, seconds): that
    worker takes that much longer to produce each gradient."""
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        os.environ.update(env or {})
        import time
        import dtg  # noqa: F401
        from dtg import ops
        from dtg.optim import FusedSGD
        from dtg.parallel import FlatParams, comm
        from dtg.parallel.async_ps import AsyncPSServer, AsyncPSWorker
        comm.init("gloo")
        model = _model()
        flat = FlatParams(model, compute_dtype=torch.float32)
        if rank == 0:
            ps = AsyncPSServer(flat, FusedSGD(flat, lr=0.1, momentum=0.0), workers=range(1, world),
                               staleness_log=True, worker_timeout=timeout)
            try:
                n = ps.serve()
            except TimeoutError as e:
                q.put((rank, "ok", {"timeout": str(e)}))
                q.close()
                q.join_thread()  # flush before the hard exit
                os._exit(0)
            q.put((rank, "ok", {"updates": n, "per_worker": dict(ps.per_worker), "lost": list(ps.lost),
                                "w": [g.master.clone().numpy() for g in flat], "staleness": list(ps.staleness)}))
        else:
            w = AsyncPSWorker(flat, ps_rank=0, overlap_pull=overlap)
            w.begin()
            x, y = _data(rank)
            t_end = time.time() + duration if duration else None
            i = 0
            while (i < steps) if t_end is None else (time.time() < t_end):
                loss = ops.softmax_cross_entropy(model(x), y)
                loss.backward()
                if slow is not None and rank == slow[0]:
                    time.sleep(slow[1])  # a slow worker: its gradient takes this much longer to exist
                w.step_done()
                if step_sleep:
                    time.sleep(step_sleep)
                if die_after is not None and rank == world - 1 and i + 1 == die_after:
                    q.put((rank, "ok", {"died": True}))
                    q.close()
                    q.join_thread()
                    os._exit(3)  # no finish(), no shutdown: the process just disappears
                if stall is not None and rank == world - 1 and i + 1 == stall:
                    q.put((rank, "ok", {"stalled": True}))
                    q.close()
                    q.join_thread()
                    time.sleep(60)
                    os._exit(0)
                i += 1
            w.finish()
            q.put((rank, "ok", {"pushes": w.pushes}))
        comm.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None))
        raise


def _run_opts(world, steps, **kw):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_opts, args=(r, world, port, steps, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, status, payload = q.get(timeout=240)
        assert status == "ok", status
        out[r] = payload
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    return out


def test_async_ps_overlapped_pull_equals_lagged_replay():
    """overlap_pull: the worker's step t gradient is computed on the PS parameters after update t-2 (one
    extra step of staleness, the pull lands at the next exchange); with one worker that is deterministic."""
    steps = 10
    out = _run_opts(2, steps, overlap=True)
    assert out[0]["updates"] == steps and out[1]["pushes"] == steps
    import dtg  # noqa: F401
    from dtg import ops
    model = _model()
    x, y = _data(1)
    params = list(model.parameters())
    hist = [[p.detach().clone() for p in params]]  # PS states P_0, P_1, ...
    for t in range(1, steps + 1):
        used = hist[max(0, t - 2)]
        with torch.no_grad():
            for p, v in zip(params, used):
                p.copy_(v)
        loss = ops.softmax_cross_entropy(model(x), y)
        grads = torch.autograd.grad(loss, params)
        hist.append([h - 0.1 * g for h, g in zip(hist[-1], grads)])
    got = _ps_params_by_name(out)
    for (n, _), v in zip(model.named_parameters(), hist[-1]):
        assert torch.allclose(got[n], v, atol=1e-5), n


def test_async_ps_survives_a_dead_worker():
    """A worker process that vanishes mid-run (SURVEY §4.2 fault injection): its control connection drops,
    the PS drops it and finishes with the survivor, every update it did push counted once."""
    out = _run_opts(3, 12, die_after=4)
    assert out[2] == {"died": True}
    assert out[0]["lost"] == [2]
    assert out[0]["per_worker"] == {1: 12, 2: 4} and out[0]["updates"] == 16


def test_async_ps_dead_worker_outlives_rank_watchdog_timeout():
    """comm.init starts the fail-stop rank watchdog (parallel/comm.py) for multi-rank jobs; an async-PS job
    must not inherit it, or the PS and every survivor would exit (status 75) DTG_RANK_TIMEOUT after a
    worker died.  Here the timeout is 1 s and the survivor keeps training ~4 s after the death."""
    env = {"DTG_RANK_TIMEOUT": "1", "DTG_HEARTBEAT_S": "0.2"}
    out = _run_opts(3, 24, die_after=2, env=env, step_sleep=0.2)
    assert out[2] == {"died": True}
    assert out[0]["lost"] == [2]
    assert out[0]["per_worker"] == {1: 24, 2: 2} and out[1] == {"pushes": 24}


@pytest.mark.parametrize("overlap", [False, True])
def test_async_ps_one_ps_seven_workers(overlap):
    """BASELINE.json config 4's topology, 1 PS + 7 workers (gloo on the CPU): every worker's pushes are all
    applied (equal per-worker counts), nobody is lost, and the staleness stays within what a round-robin of 7
    workers implies: a worker's pull is followed by at most the other 6 workers' updates before its push
    (one exchange more with overlapped pulls)."""
    steps = 6
    out = _run_opts(8, steps, overlap=overlap)
    ps = out[0]
    assert ps["lost"] == []
    assert ps["per_worker"] == {w: steps for w in range(1, 8)}
    assert ps["updates"] == 7 * steps
    st = ps["staleness"]
    bound = 6 + (7 if overlap else 0)
    assert max(st) <= 7 * 2 - 1 + (7 if overlap else 0)
    assert sum(st) / len(st) <= bound, st


def test_async_ps_worker_timeout_names_silent_workers():
    out = _run_opts(2, 6, timeout=3.0, stall=2)
    assert "no request from workers [1]" in out[0]["timeout"]


def test_async_ps_slow_worker_does_not_hold_back_fast_ones():
    """1 PS + 3 workers for 4 s, worker 3 taking 0.25 s longer per gradient: the PS serves gradients in the
    order they exist, so the two fast workers take proportionally more updates instead of waiting for it
    (Hogwild semantics, /root/reference/Hogwild/Hogwild.py:44-57), and every push is applied once."""
    out = _run_opts(4, 0, duration=4.0, slow=(3, 0.25))
    ps = out[0]
    assert ps["lost"] == []
    pw = ps["per_worker"]
    assert pw[3] <= 17, pw
    # a fast worker is not held to the slow one's pace (lock-step would give equal counts); 1.5x leaves room for a
    # loaded CI host (pytest -n 4 measured 10 / 11 vs 6), where the fast workers' own compute slows too
    assert 2 * min(pw[1], pw[2]) >= 3 * pw[3], pw
    assert sum(out[r]["pushes"] for r in (1, 2, 3)) == ps["updates"]


def test_announcer_sends_tokens_only_after_their_events_in_order():
    """The worker-side announcer (parallel/async_ps.py::_Announcer): submit() returns at once, each token is
    sent only after its event completes, and tokens keep their submission order."""
    import threading
    import time
    import dtg  # noqa: F401
    from dtg.parallel.async_ps import _Announcer

    class Ev:
        def __init__(self, delay):
            self.delay, self.done = delay, threading.Event()

        def synchronize(self):
            time.sleep(self.delay)
            self.done.set()

    sent = []

    class Ctl:
        def request(self, rank, kind):
            sent.append((rank, kind, time.perf_counter()))

    a = _Announcer(Ctl())
    e1, e2 = Ev(0.3), Ev(0.0)
    t0 = time.perf_counter()
    a.submit(1, 1, e1)
    a.submit(1, 4, e2)
    a.submit(1, 2)
    assert time.perf_counter() - t0 < 0.1  # the host never waits for the device here
    a.close()
    assert [k for _, k, _ in sent] == [1, 4, 2]
    assert sent[0][2] - t0 >= 0.3 and e1.done.is_set()


# ---- DOWNPOUR / ADAG with a worker-local optimizer (/root/reference/DOWNPOUR/DOWNPOUR.py:54-102,
# /root/reference/ADAG/ADAG.py:61-90): pull, T gradient evaluations with T - 1 local optimizer updates between them,
# push the window's sum (DOWNPOUR) or mean (ADAG), global optimizer on the PS, pull.

_LR_G, _LR_L = 0.05, 0.02


def _make_opt(kind, flat, lr):
    from dtg.optim import FusedAdagrad, FusedSGD
    return FusedAdagrad(flat, lr=lr) if kind == "adagrad" else FusedSGD(flat, lr=lr, momentum=0.0)


def _rank_local(rank, world, port, steps, window, mode, local, glob, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import dtg  # noqa: F401
        from dtg import ops
        from dtg.parallel import FlatParams, comm
        from dtg.parallel.async_ps import AsyncPSServer, AsyncPSWorker
        comm.init("gloo")
        model = _model()
        flat = FlatParams(model, compute_dtype=torch.float32)
        if rank == 0:
            ps = AsyncPSServer(flat, _make_opt(glob, flat, _LR_G), workers=range(1, world), window=window,
                               window_mode=mode)
            n = ps.serve()
            q.put((rank, "ok", {"updates": n, "order": list(ps.order), "w": [g.master.clone().numpy() for g in flat]}))
        else:
            w = AsyncPSWorker(flat, ps_rank=0, window=window, window_mode=mode,
                              local_optimizer=_make_opt(local, flat, _LR_L))
            w.begin()
            x, y = _data(rank)
            for _ in range(steps):
                ops.softmax_cross_entropy(model(x), y).backward()
                w.step_done()
            w.finish()
            q.put((rank, "ok", {"pushes": w.pushes}))
        comm.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None))
        raise


def _run_local(world, steps, window, mode, local, glob):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_local, args=(r, world, port, steps, window, mode, local, glob, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, status, payload = q.get(timeout=240)
        assert status == "ok", status
        out[r] = payload
    for p in procs:
        p.join(timeout=60)
    return out


class _Rule:
    """TF ApplyAdagrad (initial accumulator 0.1) or ApplyGradientDescent on a dict of named tensors."""

    def __init__(self, kind, lr, like):
        self.kind, self.lr = kind, lr
        self.acc = {n: torch.full_like(v, 0.1) for n, v in like.items()} if kind == "adagrad" else None

    def apply(self, params, grads):
        for n in params:
            g = grads[n]
            if self.acc is not None:
                self.acc[n].add_(g * g)
                params[n] = params[n] - self.lr * g * torch.rsqrt(self.acc[n])
            else:
                params[n] = params[n] - self.lr * g


def _window_replay(order, window, mode, local, glob):
    """Sequential replay of the reference rule in the PS's applied order: worker w's window k starts from the PS
    state its previous pull returned (the state right after ITS previous update; the initial state for k = 0)."""
    import dtg  # noqa: F401
    from dtg import ops
    model = _model()
    names = [n for n, _ in model.named_parameters()]
    state = {n: p.detach().clone() for n, p in model.named_parameters()}
    gopt = _Rule(glob, _LR_G, state)
    pulled, lopt = {}, {}
    for w, k in order:
        start = pulled.get(w, {n: v.clone() for n, v in _model().named_parameters()})
        lopt.setdefault(w, _Rule(local, _LR_L, state))
        x, y = _data(w)
        loc = {n: v.detach().clone() for n, v in start.items()}
        total = {n: torch.zeros_like(v) for n, v in loc.items()}
        for t in range(window):
            with torch.no_grad():
                for n, p in model.named_parameters():
                    p.copy_(loc[n])
            loss = ops.softmax_cross_entropy(model(x), y)
            grads = dict(zip(names, torch.autograd.grad(loss, list(model.parameters()))))
            for n in names:
                total[n] += grads[n]
            if t < window - 1:  # T - 1 local updates (DOWNPOUR/DOWNPOUR.py:65-75)
                lopt[w].apply(loc, grads)
        push = {n: v / window for n, v in total.items()} if mode == "mean" else total
        gopt.apply(state, push)
        pulled[w] = {n: v.clone() for n, v in state.items()}
    return state


@pytest.mark.parametrize("local,glob,mode", [("adagrad", "adagrad", "sum"),  # DOWNPOUR
                                             ("sgd", "adagrad", "sum"),      # DOWNPOUR-Easy
                                             ("sgd", "sgd", "mean")])        # ADAG
def test_async_ps_local_optimizer_window_equals_reference_rule(local, glob, mode):
    """1 PS + 1 worker, window 3 with a local optimizer: the PS parameters equal a sequential replay of the
    reference's rule (T gradients, T - 1 local applies, summed / averaged push, global apply on the PS)."""
    out = _run_local(2, steps=12, window=3, mode=mode, local=local, glob=glob)
    assert out[0]["updates"] == 4 and out[1]["pushes"] == 4
    ref = _window_replay(out[0]["order"], 3, mode, local, glob)
    got = _ps_params_by_name(out)
    for n, v in ref.items():
        assert torch.allclose(got[n], v, atol=1e-5), (n, (got[n] - v).abs().max())


def test_async_ps_downpour_two_workers_follow_logged_order():
    """1 PS + 2 workers, DOWNPOUR (local Adagrad, window 3, global Adagrad): whatever order the PS applied the
    pushes in, replaying that logged order with each worker's window starting from the state its own previous pull
    returned gives the PS's final parameters."""
    out = _run_local(3, steps=9, window=3, mode="sum", local="adagrad", glob="adagrad")
    order = out[0]["order"]
    assert out[0]["updates"] == 6 and sorted(order) == [(1, 0), (1, 1), (1, 2), (2, 0), (2, 1), (2, 2)]
    ref = _window_replay(order, 3, "sum", "adagrad", "adagrad")
    got = _ps_params_by_name(out)
    for n, v in ref.items():
        assert torch.allclose(got[n], v, atol=1e-5), (n, (got[n] - v).abs().max())


def test_bound_inflight_times_out_naming_the_worker(monkeypatch):
    """the PS host's wait for its oldest in-flight request polls against worker_timeout and raises a
    TimeoutError naming the worker (a receive from a worker that died mid-transfer never completes), instead of
    blocking forever in Event.synchronize()."""
    import types
    import dtg  # noqa: F401
    from dtg.parallel import async_ps

    class NeverDone:
        def record(self, stream):
            pass

        def query(self):
            return False

        def synchronize(self):  # pragma: no cover - the old, unbounded wait
            raise AssertionError("blocking synchronize() on an in-flight request")

    monkeypatch.setattr(torch.cuda, "Event", NeverDone)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda dev=None: None)
    ps = object.__new__(async_ps.AsyncPSServer)
    ps.dev = types.SimpleNamespace(type="cuda")
    ps.max_inflight, ps.worker_timeout, ps._inflight = 1, 0.3, []
    ps._bound_inflight(3)
    with pytest.raises(TimeoutError, match="worker rank 3"):
        ps._bound_inflight(5)


def test_resnet_async_ps_example_session_driven(tmp_path):
    """examples/ResNet50/resnet50_async_ps.py (tiny ResNet, gloo): 1 PS + 2 workers, the workers' loop is a
    MonitoredTrainingSession running AsyncPSWorker.minimize's train op until StopAtStepHook; the session's hook
    pulls first and finishes the worker, and the PS's serve() returns after 2 x 4 updates."""
    import subprocess
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    base = free_ports(1)[0]
    script = os.path.join(ROOT, "examples", "ResNet50", "resnet50_async_ps.py")
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", DTG_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    args = ["--tiny", "--workers", "2", "--steps", "4", "--batch", "2", "--image", "32", "--base_port", str(base)]
    procs = [subprocess.Popen([sys.executable, script, "--job_name", "ps", "--task_index", "0"] + args, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)]
    procs += [subprocess.Popen([sys.executable, script, "--job_name", "worker", "--task_index", str(i)] + args,
                               env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for i in range(2)]
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            outs.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, o, e in outs:
        assert rc == 0, o + e[-3000:]
    assert "[ps] 8 updates" in outs[0][1], outs[0][1]
    for rc, o, e in outs[1:]:
        assert "step 0 loss" in o and "4 pushes" in o, o
