"""Asynchronous parameter server on GPUs: one PS rank keeps the parameters in HBM, workers push
gradients and pull parameters with point-to-point RCCL send/recv (``torch.distributed`` "nccl"
backend = RCCL over xGMI; "gloo" on the CPU for tests).

This is the GPU-scale form of the reference's between-graph async training (SURVEY §2.3 Hogwild,
DOWNPOUR, ADAG; §2.4 (b); BASELINE.json config 4 "ResNet-50 async parameter-server, 1 PS + 7
workers intra-node (RCCL send/recv)").  Reference semantics kept:

* Hogwild (``Hogwild/Hogwild.py:44-57``): every worker gradient is applied on the PS as soon as it
  arrives, no locking across workers; a worker computes on whatever parameters it last pulled.
* DOWNPOUR / ADAG window (``DOWNPOUR/DOWNPOUR.py:63-102``, ``ADAG/ADAG.py:69-90``): a worker runs
  ``window`` local steps (optionally applying a local optimizer), accumulates their gradients and
  pushes the sum (DOWNPOUR) or the mean (ADAG); the PS applies it with the global optimizer.
* Dynamic SGD (the reference README's TODO list, ``README.md:40``): ``staleness_scaling="dyn"``
  scales every update by 1/(tau+1), tau = the number of PS updates since the pushing worker last
  pulled (DynSGD, Jiang et al., SIGMOD 2017), so stale gradients from slow workers move the
  parameters less.

MI355X design: parameters and optimizer state live in the PS GPU's flat buffers (FlatParams); a
push is one RCCL send per dtype group (bf16 compute grads + fp32 norm/bias grads), a pull is one
send of the bf16 compute mirror + fp32 group.  The PS serves all workers concurrently: it keeps
one receive posted per worker (RCCL runs each PS<->worker pair on its own communicator/stream),
applies whichever gradient lands first with the fused HIP optimizer kernel, snapshots the updated
parameters into that worker's send buffer (so later applies cannot tear an in-flight send) and
sends them back.
"""
import time

import torch
import torch.distributed as dist

_GRAD, _DONE, _ELASTIC = 1, 2, 3


# gloo moves CPU tensors only for point-to-point; with DTG_BACKEND=gloo DTG_GLOO_DEVICE=cuda (the
# one-card rehearsal of this GPU path, see parallel/comm.py) device tensors are staged through host
# memory.  RCCL sends/receives HBM buffers directly; these helpers are then plain dist calls.
def _staged(t, group):
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _send(t, dst, group=None):
    dist.send(t.cpu() if _staged(t, group) else t, dst=dst, group=group)


def _recv(t, src=None, group=None):
    if not _staged(t, group):
        return dist.recv(t, src=src, group=group)
    h = torch.empty_like(t, device="cpu")
    peer = dist.recv(h, src=src, group=group)
    t.copy_(h)
    return peer


from ..utils.trace import traced


class _HostSend:
    """isend of a host copy; keeps the copy alive until wait()."""

    def __init__(self, t, dst, group):
        self._h = t.cpu()
        self._w = dist.isend(self._h, dst=dst, group=group)

    def wait(self):
        self._w.wait()
        self._h = None

    def is_completed(self):
        return self._w.is_completed()


def _isend(t, dst, group=None):
    return _HostSend(t, dst, group) if _staged(t, group) else dist.isend(t, dst=dst, group=group)


def _group_payload_grads(flat):
    return [g.grad for g in flat]


def _buffers(flat):
    fb = getattr(flat, "buffers", None)
    return [fb.flat] if fb is not None else []


def _group_payload_params(flat):
    # what the model reads: the bf16 mirror of the compute group, the fp32 master of the fp32 group,
    # and the module buffers (BN running statistics: PS variables in the reference's TF setup)
    return [g.mirror if g.mirror is not None else g.master for g in flat] + _buffers(flat)


def _elastic_state(flat):
    return [g.master for g in flat] + _buffers(flat)


class AsyncPSWorker:
    """Worker side.  ``begin()`` pulls the current parameters, ``step_done()`` after every backward
    pushes/pulls every ``window`` steps, ``finish()`` tells the PS this worker is done (the PS's
    ``serve()`` returns when all workers finished; a new begin()/serve() round may follow)."""

    def __init__(self, flat, ps_rank=0, window=1, window_mode="sum", local_optimizer=None, group=None):
        assert window_mode in ("sum", "mean")
        self.flat = flat
        self.ps = ps_rank
        self.pg = group
        self.window = max(1, int(window))
        self.window_mode = window_mode
        self.local_opt = local_optimizer
        dev = next(iter(flat)).master.device
        self.dev = dev
        self._hdr = torch.zeros(2, dtype=torch.int64, device=dev)
        self._acc = [torch.zeros_like(g.grad) for g in flat] if (self.window > 1 and local_optimizer) else None
        # module buffers as pulled: the push carries (current - pulled), the worker's running-statistics
        # update since the pull, which the PS adds to its own copy
        self._buf0 = [torch.empty_like(b) for b in _buffers(flat)]
        self._bufd = [torch.empty_like(b) for b in _buffers(flat)]
        self.local_step = 0
        self.pushes = 0

    def begin(self):
        """Initial pull (replaces the chief's assign_global + sleep(10) bootstrap,
        DOWNPOUR/DOWNPOUR.py:129-135)."""
        self.pull()

    @traced("dtg.ps.pull")
    def pull(self):
        for buf in _group_payload_params(self.flat):
            _recv(buf, src=self.ps, group=self.pg)
        for b0, b in zip(self._buf0, _buffers(self.flat)):
            b0.copy_(b)
        if self.local_opt is not None:
            # the local optimizer updates the fp32 master: re-seed it from the pulled parameters
            for g in self.flat:
                if g.mirror is not None:
                    g.master.copy_(g.mirror)

    @traced("dtg.ps.push")
    def step_done(self):
        """Call once per local step after backward.  Pushes/pulls every ``window`` steps; returns
        True when an exchange with the PS happened."""
        self.local_step += 1
        if self._acc is not None:
            # DOWNPOUR-style: accumulate this step's gradient, then take a local optimizer step
            for a, g in zip(self._acc, self.flat):
                a.add_(g.grad.to(a.dtype))
            self.local_opt.step()
        if self.local_step % self.window:
            return False
        grads = self._acc if self._acc is not None else _group_payload_grads(self.flat)
        for d, b, b0 in zip(self._bufd, _buffers(self.flat), self._buf0):
            torch.sub(b, b0, out=d)
        self._hdr[0] = _GRAD
        self._hdr[1] = self.local_step
        _send(self._hdr, dst=self.ps, group=self.pg)
        works = [_isend(t, dst=self.ps, group=self.pg) for t in list(grads) + self._bufd]
        for w in works:
            w.wait()
        for t in grads:
            t.zero_()
        if self._acc is not None:
            self.flat.zero_grad()
        self.pull()
        self.pushes += 1
        return True

    def finish(self):
        self._hdr[0] = _DONE
        self._hdr[1] = self.local_step
        _send(self._hdr, dst=self.ps, group=self.pg)


class AsyncPSServer:
    """PS side: ``serve()`` runs until every worker sent DONE; returns the number of updates."""

    def __init__(self, flat, optimizer, workers, window=1, window_mode="sum", group=None, staleness_log=False,
                 staleness_scaling=None):
        assert staleness_scaling in (None, "dyn")
        self.dyn = staleness_scaling == "dyn"
        self.flat = flat
        self.opt = optimizer
        self.workers = list(workers)
        self.pg = group
        self.gscale = 1.0 / window if window_mode == "mean" else 1.0
        dev = next(iter(flat)).master.device
        self.dev = dev
        self._recv = {w: [torch.empty_like(g.grad) for g in flat] for w in self.workers}
        self._recv_buf = {w: [torch.empty_like(b) for b in _buffers(flat)] for w in self.workers}
        self._snap = {w: [torch.empty_like(t) for t in _group_payload_params(flat)] for w in self.workers}
        self._hdr = {w: torch.zeros(2, dtype=torch.int64, device=dev) for w in self.workers}
        self._send_works = {w: [] for w in self.workers}
        self.updates = 0
        self.version = 0
        self._pulled_version = {w: 0 for w in self.workers}
        self.staleness = [] if staleness_log else None
        self.scales = [] if staleness_log else None
        self.per_worker = {w: 0 for w in self.workers}

    def _send_params(self, w):
        for prev in self._send_works[w]:
            prev.wait()  # the snapshot buffer is about to be overwritten
        snap = self._snap[w]
        for s, p in zip(snap, _group_payload_params(self.flat)):
            s.copy_(p)
        self._send_works[w] = [_isend(s, dst=w, group=self.pg) for s in snap]
        self._pulled_version[w] = self.version

    @traced("dtg.ps.apply")
    def _apply(self, w):
        bufs = self._recv[w]
        saved = [g.grad for g in self.flat]
        tau = self.version - self._pulled_version[w]
        scale = self.gscale / (tau + 1) if self.dyn else self.gscale
        try:
            for g, b in zip(self.flat, bufs):
                g.grad = b
            self.opt.step(grad_scale=scale, zero_grad=False)
        finally:
            for g, s in zip(self.flat, saved):
                g.grad = s
        # running statistics: add the worker's update since its pull (lock-free, Hogwild-style, like the
        # reference's unlocked assign_moving_average on PS variables)
        for b, d in zip(_buffers(self.flat), self._recv_buf[w]):
            b.add_(d)
        if self.staleness is not None:
            self.staleness.append(tau)
            self.scales.append(scale)
        self.version += 1
        self.updates += 1
        self.per_worker[w] += 1

    def _handle(self, w):
        """Header from worker w has landed: DONE -> False; else receive, apply, reply -> True."""
        kind = int(self._hdr[w][0].item())
        if kind == _DONE:
            return False
        if kind == _ELASTIC:
            self._elastic(w)
            return True
        for b in self._recv[w] + self._recv_buf[w]:
            _recv(b, src=w, group=self.pg)
        self._apply(w)
        self._send_params(w)
        return True

    def _elastic(self, w):
        """EASGD exchange (Zhang, Choromanska, LeCun 2015): receive the worker's parameters x_i,
        d = alpha * (x_i - x~), x~ += d, send d back (the worker applies x_i -= d)."""
        bufs = self._recv_elastic[w]
        for b in bufs:
            _recv(b, src=w, group=self.pg)
        with torch.no_grad():
            for c, b in zip(_elastic_state(self.flat), bufs):
                b.sub_(c).mul_(self.elastic_alpha)
                c.add_(b)
            for g in self.flat:
                g.refresh_mirror()
        for prev in self._send_works[w]:
            prev.wait()
        snap = self._snap_elastic[w]
        for s_, b in zip(snap, bufs):
            s_.copy_(b)
        self._send_works[w] = [_isend(s_, dst=w, group=self.pg) for s_ in snap]
        self.version += 1
        self.updates += 1
        self.per_worker[w] += 1

    def enable_elastic(self, alpha):
        """Serve EASGD exchanges: the PS parameters are the elastic center variable x~."""
        self.elastic_alpha = float(alpha)
        self._recv_elastic = {w: [torch.empty_like(t) for t in _elastic_state(self.flat)] for w in self.workers}
        self._snap_elastic = {w: [torch.empty_like(t) for t in _elastic_state(self.flat)] for w in self.workers}
        return self

    def serve(self, poll_sleep=0.0):
        for w in self.workers:
            self._send_params(w)
        if dist.get_backend(self.pg) == "gloo":
            self._serve_any_source()
        else:
            self._serve_polling(poll_sleep)
        for w in self.workers:
            for s in self._send_works[w]:
                s.wait()
        return self.updates

    def _serve_polling(self, poll_sleep):
        # RCCL: one header receive posted per worker (each on its pair communicator); serve
        # whichever completes first
        pending = {w: dist.irecv(self._hdr[w], src=w, group=self.pg) for w in self.workers}
        while pending:
            progressed = False
            for w in list(pending):
                if not pending[w].is_completed():
                    continue
                pending[w].wait()
                progressed = True
                if self._handle(w):
                    pending[w] = dist.irecv(self._hdr[w], src=w, group=self.pg)
                else:
                    del pending[w]
            if not progressed and poll_sleep:
                time.sleep(poll_sleep)

    def _serve_any_source(self):
        # gloo: receive-from-any-source gives arrival order directly
        live = set(self.workers)
        hdr = torch.zeros(2, dtype=torch.int64, device=self.dev)
        while live:
            w = _recv(hdr, group=self.pg)  # returns the sender's global rank
            self._hdr[w].copy_(hdr)
            if not self._handle(w):
                live.discard(w)


class ElasticWorker:
    """Asynchronous elastic-averaging SGD worker (AEASGD; AEAMSGD with a momentum local optimizer) --
    the algorithms the reference lists as TODO (README.md:40-42, paper link README.md:99).

    The worker trains its own replica x_i with ``local_optimizer`` every step; every ``tau`` steps it
    exchanges with the PS center x~:  d = alpha (x_i - x~);  x_i -= d;  x~ += d  (moving-average
    coupling instead of gradient pushes; the PS must call ``AsyncPSServer.enable_elastic(alpha)``).
    """

    def __init__(self, flat, local_optimizer, tau=4, ps_rank=0, group=None):
        self.flat = flat
        self.opt = local_optimizer
        self.tau = max(1, int(tau))
        self.ps = ps_rank
        self.pg = group
        dev = next(iter(flat)).master.device
        self._hdr = torch.zeros(2, dtype=torch.int64, device=dev)
        self._d = [torch.empty_like(t) for t in _elastic_state(flat)]
        self.local_step = 0
        self.exchanges = 0

    def begin(self):
        """Start from the center: receive the PS parameters (mirror / fp32 group) into the replica."""
        for buf in _group_payload_params(self.flat):
            _recv(buf, src=self.ps, group=self.pg)
        with torch.no_grad():
            for g in self.flat:
                if g.mirror is not None:
                    g.master.copy_(g.mirror)

    def step_done(self):
        """After backward: local optimizer step; every tau steps an elastic exchange."""
        self.local_step += 1
        self.opt.step()
        if self.local_step % self.tau:
            return False
        self._hdr[0] = _ELASTIC
        self._hdr[1] = self.local_step
        _send(self._hdr, dst=self.ps, group=self.pg)
        works = [_isend(t, dst=self.ps, group=self.pg) for t in _elastic_state(self.flat)]
        for w in works:
            w.wait()
        for d in self._d:
            _recv(d, src=self.ps, group=self.pg)
        with torch.no_grad():
            for t, d in zip(_elastic_state(self.flat), self._d):
                t.sub_(d)
            for g in self.flat:
                g.refresh_mirror()
        self.exchanges += 1
        return True

    def finish(self):
        self._hdr[0] = _DONE
        self._hdr[1] = self.local_step
        _send(self._hdr, dst=self.ps, group=self.pg)


def init_from_cluster(cluster, job_name, task_index, backend=None, port_offset=1):
    """Bootstrap the RCCL/gloo process group from a TF-style ClusterSpec: the PS task 0 is rank 0
    (its ``host:port`` + ``port_offset`` is the rendezvous), worker i is rank 1 + i.  One process per
    GPU: pin each process to its GPU with HIP_VISIBLE_DEVICES (see examples/ResNet50/run_async.sh).
    Returns (rank, world, device)."""
    import datetime
    import os

    spec = cluster.as_dict() if hasattr(cluster, "as_dict") else dict(cluster)
    ps_host, ps_port = spec["ps"][0].rsplit(":", 1)
    n_workers = len(spec["worker"])
    rank = 0 if job_name == "ps" else 1 + int(task_index)
    world = 1 + n_workers
    backend = os.environ.get("DTG_BACKEND") or backend
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    gloo_cuda = backend == "gloo" and os.environ.get("DTG_GLOO_DEVICE") == "cuda" and torch.cuda.is_available()
    device = torch.device("cuda", 0) if backend == "nccl" or gloo_cuda else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    os.environ["MASTER_ADDR"] = "127.0.0.1" if ps_host in ("localhost", "") else ps_host
    os.environ["MASTER_PORT"] = str(int(ps_port) + port_offset)
    kw = {"device_id": device} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600), **kw)
    return rank, world, device
