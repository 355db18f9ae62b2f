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

MI355X design:

* **payloads** go over RCCL point-to-point: torch's RCCL process group gives every PS<->worker pair its
  own 2-rank communicator and HIP stream, so the pairs move gradients and parameters concurrently.  With
  one process per GPU and every device visible to every process (examples/ResNet50/run_async.sh,
  ``bench.py --mode async_ps``) each pair is a distinct GPU pair, which on MI355X's fully connected xGMI
  mesh has a direct link of its own (7 per GPU); that the 7 transfers then run link-parallel has not been
  traced on an 8-GPU node yet (the one-card rehearsals stage through host memory over gloo).  A push is one
  send per dtype group (bf16 compute grads, fp32 norm/bias grads, the BN running-statistics delta); a pull
  is the bf16 compute mirror, the fp32 group and the module buffers.
* **request framing** goes over dtg's native TCP service (csrc/ps/server.cc, the same one the CPU PS
  uses): a worker enqueues a (rank, kind) token on one queue and the PS blocks in ``q_dequeue`` with
  the GIL released.  So the PS serves requests in arrival order with no busy spin and no device
  synchronisation: its host loop only enqueues GPU work (post the receive, make the apply stream wait
  for it, apply with the fused HIP optimizer kernel, snapshot, send), all ordered by streams and events.
* **failure detection**: each worker's control connection carries a watch (``PSClient.watch``); if the
  worker process dies, the service enqueues its "lost" token and ``serve()`` finishes with the
  survivors (``lost`` lists who dropped out).  ``worker_timeout`` bounds how long the PS waits with no
  request from any live worker (TimeoutError naming them).  A worker that dies in the middle of a
  transfer leaves an RCCL kernel waiting on its pair stream; RCCL communicators cannot shrink, so that
  case is fail-stop (the other workers' pulls stall and the PS times out), like sync DP.
* **GPU-ready request order**: a worker's host enqueues a step long before its GPU has the gradient.  Its
  request token therefore goes out from a small announcer thread only once a device event recorded after the
  gradient has completed (:class:`_Announcer`), so the PS -- which posts the receive and makes its apply stream
  wait for it as soon as it dequeues a token -- serves workers in the order their gradients EXIST, never
  stalls its apply stream behind a worker that is still in backward, and fast workers take proportionally
  more updates than a slow one (``test_async_ps_slow_worker_does_not_hold_back_fast_ones``).  The PS also
  bounds how many requests' device work it has queued (``max_inflight``; the host waits on the oldest
  request's completion event beyond it), so its pair streams cannot pile up.
* **staleness** tau of an update = the number of PS updates applied between the pushing worker's last pull
  (the parameter snapshot its gradient was computed on) and this update.  With W workers in round-robin tau is
  about W - 1; ``overlap_pull`` adds one exchange (about W more): the one-card 1 PS + 7 worker rehearsal with
  overlapped pulls measured a mean of 6.0 (``profiles/r04_async_ps``).
* **overlap** (``overlap_pull=True``): the worker snapshots its gradients into a send buffer, posts the
  push and the pull, and goes on with its next step on the parameters it already has; the pulled ones
  are swapped in (a device copy) at its next exchange.  That adds one step of staleness, which Hogwild
  semantics allow, and takes the push -> PS apply -> pull round trip off the worker's critical path.
  Without it the worker's GPU waits for the pull (its host does not).
"""
import os
import sys

import torch
import torch.distributed as dist

_GRAD, _DONE, _ELASTIC, _WARM = 1, 2, 3, 4
_KINDS = 16
_REQ = "dtg.aps.req"
_instances = [0]  # per-process count of async-PS objects: the same on every rank (construction order)


# gloo moves CPU tensors only for point-to-point; with DTG_BACKEND=gloo DTG_GLOO_DEVICE=cuda (the
# one-card rehearsal of this GPU path, see parallel/comm.py) device tensors are staged through host
# memory.  RCCL sends/receives HBM buffers directly; these helpers are then plain dist calls.
def _staged(t, group):
    return t.is_cuda and dist.get_backend(group) == "gloo"


class _Done:
    def wait(self):
        pass


class _HostSend:
    """isend of a host copy; keeps the copy alive until wait()."""

    def __init__(self, t, dst, group):
        self._h = t.cpu()
        self._w = dist.isend(self._h, dst=dst, group=group)

    def wait(self):
        self._w.wait()
        self._h = None


class _HostRecv:
    """irecv into a host buffer; wait() lands it in the device tensor."""

    def __init__(self, t, src, group):
        self._t = t
        self._h = torch.empty_like(t, device="cpu")
        self._w = dist.irecv(self._h, src=src, group=group)

    def wait(self):
        self._w.wait()
        self._t.copy_(self._h)
        self._h = None


def _isend(t, dst, group=None):
    return _HostSend(t, dst, group) if _staged(t, group) else dist.isend(t, dst=dst, group=group)


def _irecv(t, src, group=None):
    """Post a receive.  RCCL: ``wait()`` makes the CURRENT stream wait for it (no host block)."""
    return _HostRecv(t, src, group) if _staged(t, group) else dist.irecv(t, src=src, group=group)


def _wait_all(works):
    for w in works:
        w.wait()


from ..utils.trace import traced  # noqa: E402
from ..graph import Op  # noqa: E402
from ..train.hooks import SessionRunHook  # noqa: E402


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


class _Control:
    """Request framing between the PS rank and its workers over the native TCP service.  The PS hosts it
    and publishes its address in the process group's store; workers connect and watch their connection."""

    def __init__(self, is_ps, rank):
        from .. import _runtime
        from . import comm
        # a lost worker is survivable here (serve() continues with the rest): the fail-stop rank watchdog that
        # comm.init starts for multi-rank jobs would instead end every rank DTG_RANK_TIMEOUT after the loss
        comm.stop_watchdog()
        _instances[0] += 1
        key = "dtg.aps.ctl.%d" % _instances[0]
        store = dist.distributed_c10d._get_default_store()
        self.svc = None
        if is_ps:
            host = os.environ.get("MASTER_ADDR", "127.0.0.1")
            bind = "127.0.0.1" if host in ("127.0.0.1", "localhost") else "0.0.0.0"
            self.svc = _runtime.PSServer(bind, 0, 0)
            self.svc.start()
            self.cli = _runtime.PSClient("127.0.0.1", self.svc.port, 60.0)
            store.set(key, "%s:%d" % ("127.0.0.1" if bind == "127.0.0.1" else host, self.svc.port))
        else:
            addr = store.get(key).decode()
            h, p = addr.rsplit(":", 1)
            self.cli = _runtime.PSClient(h, int(p), 60.0)
            self.cli.watch(_REQ, -(rank + 1))  # dies with the process -> the PS sees a lost token

    def request(self, rank, kind):
        self.cli.q_enqueue(_REQ, [rank * _KINDS + kind])

    def next(self, timeout):
        return self.cli.q_dequeue(_REQ, -1.0 if timeout is None else float(timeout))

    def unwatch(self):
        self.cli.unwatch()

    def close(self):
        if self.cli is not None:
            self.cli.close()
            self.cli = None
        if self.svc is not None:
            self.svc.stop()
            self.svc = None


class _Announcer:
    """Sends a worker's request tokens from a background thread, each only after the device event it carries
    has completed (None: at once), in submission order.  The worker's host thread never blocks on its own GPU
    for this, and the PS sees a gradient's token only when the gradient is on the device."""

    def __init__(self, ctl):
        import queue
        import threading
        self._ctl = ctl
        self._q = queue.Queue()
        self.error = None
        self._t = threading.Thread(target=self._run, name="dtg-aps-announce", daemon=True)
        self._t.start()

    def _run(self):
        while True:
            item = self._q.get()
            if item is None:
                return
            rank, kind, ev = item
            try:
                if ev is not None:
                    ev.synchronize()
                self._ctl.request(rank, kind)
            except Exception as e:  # surfaced by the next submit()/close()
                self.error = e
                return

    def _check(self):
        if self.error is not None:
            raise RuntimeError("async PS request announcer failed") from self.error

    def submit(self, rank, kind, event=None):
        self._check()
        self._q.put((rank, kind, event))

    def close(self):
        """Flush every queued token (in order) and stop the thread."""
        self._q.put(None)
        self._t.join()
        self._check()


def _ready_event(tensors):
    """A device event after the work that produces ``tensors`` (None for host tensors)."""
    t = next((t for t in tensors if t.is_cuda), None)
    if t is None:
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    return ev


class AsyncPSWorker:
    """Worker side.  ``begin()`` pulls the current parameters, ``step_done()`` after every backward
    pushes/pulls every ``window`` steps, ``warm()`` marks the end of a warm-up phase (benchmarks),
    ``finish()`` tells the PS this worker is done (the PS's ``serve()`` returns when all workers finished)."""

    def __init__(self, flat, ps_rank=0, window=1, window_mode="sum", local_optimizer=None, group=None,
                 overlap_pull=False):
        assert window_mode in ("sum", "mean")
        self.flat = flat
        self.ps = ps_rank
        self.pg = group
        self.rank = dist.get_rank()
        self.window = max(1, int(window))
        self.window_mode = window_mode
        self.local_opt = local_optimizer
        self.overlap = bool(overlap_pull)
        self._ctl = _Control(False, self.rank)
        self._ann = _Announcer(self._ctl)
        self._acc = [torch.zeros_like(g.grad) for g in flat] if (self.window > 1 and local_optimizer) else None
        # module buffers as pulled: the push carries (current - pulled), the worker's running-statistics
        # update since the pull, which the PS adds to its own copy
        self._buf0 = [torch.empty_like(b) for b in _buffers(flat)]
        self._bufd = [torch.empty_like(b) for b in _buffers(flat)]
        # overlap: gradient snapshot being sent, parameters being received (double buffers)
        self._gsnap = [torch.empty_like(g.grad) for g in flat] if self.overlap else None
        self._pbuf = [torch.empty_like(t) for t in _group_payload_params(flat)] if self.overlap else None
        self._sends = []
        self._pull = None
        self.local_step = 0
        self.pushes = 0

    def begin(self):
        """Initial pull (replaces the chief's assign_global + sleep(10) bootstrap,
        DOWNPOUR/DOWNPOUR.py:129-135)."""
        _wait_all([_irecv(t, self.ps, self.pg) for t in _group_payload_params(self.flat)])
        self._pulled()

    def _pulled(self):
        for b0, b in zip(self._buf0, _buffers(self.flat)):
            b0.copy_(b)
        if self.local_opt is not None:
            # the local optimizer updates the fp32 master: re-seed it from the pulled parameters
            for g in self.flat:
                if g.mirror is not None:
                    g.master.copy_(g.mirror)

    @traced("dtg.ps.pull")
    def _land_pull(self):
        """Overlap mode: the previous exchange's parameters -> the model (stream-ordered device copy)."""
        if self._pull is None:
            return
        _wait_all(self._pull)
        self._pull = None
        for dst, src in zip(_group_payload_params(self.flat), self._pbuf):
            dst.copy_(src)
        self._pulled()

    @traced("dtg.ps.push")
    def step_done(self):
        """Call once per local step after backward.  Pushes/pulls every ``window`` steps; returns
        True when an exchange with the PS happened."""
        self.local_step += 1
        if self._acc is not None:
            # DOWNPOUR-style: accumulate this step's gradient, then take a local optimizer step -- on the first T - 1
            # steps of the window only, as the reference's graph runs it (DOWNPOUR/DOWNPOUR.py:65-75: the t-th
            # compute_gradients waits for opt_local of step t - 1, and nothing waits for the last one, so a window
            # of T gradient evaluations applies T - 1 local updates).  The last local update
            # would be overwritten by the pull anyway, but it would still feed the local optimizer's state (an
            # Adagrad accumulator, a momentum buffer) a gradient the reference never applies locally.
            for a, g in zip(self._acc, self.flat):
                a.add_(g.grad.to(a.dtype))
            if self.local_step % self.window:
                self.local_opt.step()
        if self.local_step % self.window:
            return False
        self._land_pull()
        grads = self._acc if self._acc is not None else _group_payload_grads(self.flat)
        for d, b, b0 in zip(self._bufd, _buffers(self.flat), self._buf0):
            torch.sub(b, b0, out=d)
        _wait_all(self._sends)  # the previous push's buffers are free again
        if self.overlap:
            for s, g in zip(self._gsnap, grads):
                s.copy_(g)
            grads_out = self._gsnap
        else:
            grads_out = grads
        # the token goes out when the gradient exists on the device (announcer thread), the sends are posted now
        self._ann.submit(self.rank, _GRAD, _ready_event(list(grads_out) + self._bufd))
        self._sends = [_isend(t, self.ps, self.pg) for t in list(grads_out) + self._bufd]
        if self.overlap:
            self._pull = [_irecv(t, self.ps, self.pg) for t in self._pbuf]
        else:
            _wait_all(self._sends)  # (stream-ordered) before the gradients are zeroed below
            self._sends = []
        for t in grads:
            t.zero_()
        if self._acc is not None:
            self.flat.zero_grad()
        if not self.overlap:
            _wait_all([_irecv(t, self.ps, self.pg) for t in _group_payload_params(self.flat)])
            self._pulled()
        self.pushes += 1
        return True

    # ---- session surface (train/eager.py): the reference's worker loop, sess.run(train_op) under a session ----------
    def minimize(self, loss_fn, global_step=None, inputs=(), name="async_ps_train"):
        """A train op for ``sess.run``: forward + backward of ``loss_fn(*inputs)``, then :meth:`step_done` (the
        window's local optimizer step, and the push / pull every ``window`` steps) and ``global_step += 1`` -- the
        worker loop of /root/reference/Hogwild/Hogwild.py:44-57 and DOWNPOUR/DOWNPOUR.py:116-140 with the
        parameters in the PS's HBM.  ``global_step`` counts this worker's local steps (the PS counts updates)."""
        from ..train.eager import EagerGradients
        return _AsyncPSApply(EagerGradients(loss_fn, inputs, name + "/gradients"), self, global_step, name)

    def make_session_run_hook(self):
        """after_create_session: the initial pull (:meth:`begin`); end: :meth:`finish` (the PS's ``serve()``
        returns once every worker finished, the ``Server.join()`` of the reference's PS task)."""
        return _AsyncPSHook(self)

    def warm(self):
        """Tell the PS this worker has finished its warm-up (``AsyncPSServer.timed`` starts when all have)."""
        self._ann.submit(self.rank, _WARM)

    def finish(self):
        self._land_pull()
        _wait_all(self._sends)
        self._sends = []
        self._ann.close()  # every GRAD / WARM token is out before DONE
        self._ctl.unwatch()
        try:
            self._ctl.request(self.rank, _DONE)
        except RuntimeError as e:
            # the last worker's DONE lets the PS leave serve() and close its control service; the service can go
            # down before the reply to that enqueue is flushed.  A lost connection here loses nothing: this worker
            # has no further requests, and a PS that died earlier already failed the pushes above.
            if "connection lost" not in str(e):
                raise
        self._ctl.close()


class _AsyncPSApply(Op):
    """The worker's train op (AsyncPSWorker.minimize)."""

    def __init__(self, grads, worker, global_step, name):
        self.grads, self.worker, self.global_step = grads, worker, global_step
        super().__init__(lambda c, *a: None, [grads], name)

    def _eval(self, ctx):
        ctx.eval(self.grads)
        self.worker.step_done()
        gs = self.global_step
        if gs is not None:
            with gs._lock:
                gs._local.add_(1)
        return None

    @property
    def loss(self):
        """The step's loss as a fetchable tensor (fetching it synchronises the device)."""
        return self.grads


class _AsyncPSHook(SessionRunHook):
    """AsyncPSWorker.make_session_run_hook: initial pull once the session exists, finish() at its end."""

    def __init__(self, worker):
        self.worker = worker
        self._begun = False

    def after_create_session(self, session, coord):
        if not self._begun:
            self.worker.begin()
            self._begun = True

    def end(self, session):
        if self._begun:
            self.worker.finish()
            self._begun = False


class AsyncPSServer:
    """PS side: ``serve()`` runs until every worker sent DONE (or was lost); returns the number of updates."""

    def __init__(self, flat, optimizer, workers, window=1, window_mode="sum", group=None, staleness_log=False,
                 staleness_scaling=None, worker_timeout=None, max_inflight=None):
        assert staleness_scaling in (None, "dyn")
        self.dyn = staleness_scaling == "dyn"
        self.flat = flat
        self.opt = optimizer
        self.workers = list(workers)
        self.pg = group
        self.gscale = 1.0 / window if window_mode == "mean" else 1.0
        self.worker_timeout = worker_timeout if worker_timeout is not None else float(
            os.environ.get("DTG_PS_WORKER_TIMEOUT", "600"))
        dev = next(iter(flat)).master.device
        self.dev = dev
        self._ctl = _Control(True, dist.get_rank())
        self._recv = {w: [torch.empty_like(g.grad) for g in flat] for w in self.workers}
        self._recv_buf = {w: [torch.empty_like(b) for b in _buffers(flat)] for w in self.workers}
        self._snap = {w: [torch.empty_like(t) for t in _group_payload_params(flat)] for w in self.workers}
        self._send_works = {w: [] for w in self.workers}
        self.updates = 0
        self.version = 0
        self._pulled_version = {w: 0 for w in self.workers}
        self.staleness = [] if staleness_log else None
        self.scales = [] if staleness_log else None
        self.per_worker = {w: 0 for w in self.workers}
        self.lost = []
        self._warm = set()
        self.timed = None  # (updates, time) when every worker reported warm; serve() fills timed_end
        # applied order: (worker, that worker's push index) per update -- what a replay of the PS must follow
        self.order = []
        self._push_idx = {w: 0 for w in self.workers}
        # requests whose device work (receive, apply, snapshot, send) may be queued at once; beyond that the host
        # waits for the oldest one's completion event (one outstanding request per worker by default)
        self.max_inflight = int(max_inflight if max_inflight is not None else
                                os.environ.get("DTG_PS_MAX_INFLIGHT", str(max(1, len(self.workers)))))
        self._inflight = []

    def _send_params(self, w):
        _wait_all(self._send_works[w])  # the snapshot buffer is about to be overwritten (stream wait)
        snap = self._snap[w]
        for s, p in zip(snap, _group_payload_params(self.flat)):
            s.copy_(p)
        self._send_works[w] = [_isend(s, w, self.pg) for s in snap]
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
        self.order.append((w, self._push_idx[w]))
        self._push_idx[w] += 1

    def _bound_inflight(self, w):
        """Record this request's completion on the apply stream; wait for the oldest beyond max_inflight.

        The wait polls the event against ``worker_timeout`` instead of blocking in ``synchronize()``: a worker that
        died mid-transfer leaves its receive (and so the apply stream behind it) pending forever, and the host must
        still fail-stop with a TimeoutError naming that worker, as the module docstring promises."""
        if self.dev.type != "cuda":
            return
        import time
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        self._inflight.append((ev, w))
        while len(self._inflight) > self.max_inflight:
            ev0, w0 = self._inflight.pop(0)
            deadline = time.monotonic() + self.worker_timeout
            nap = 5e-5
            while not ev0.query():
                if time.monotonic() > deadline:
                    raise TimeoutError("async PS: the request of worker rank %d has not completed on the device in "
                                       "%.0f s (worker lost mid-transfer?)" % (w0, self.worker_timeout))
                time.sleep(nap)
                nap = min(nap * 2, 2e-3)

    def _grad(self, w):
        # the receive is posted from the apply (current) stream, so RCCL's pair stream first waits for the
        # previous apply that read these buffers; the apply then waits for the receive (stream events only).
        # The worker sent this token only once its gradient was on its device (_Announcer), so the receive
        # completes as soon as the pair's transfer does.
        _wait_all([_irecv(b, w, self.pg) for b in self._recv[w] + self._recv_buf[w]])
        self._apply(w)
        self._send_params(w)
        self._bound_inflight(w)

    def _elastic(self, w):
        """EASGD exchange (Zhang, Choromanska, LeCun 2015): receive the worker's parameters x_i,
        d = alpha * (x_i - x~), x~ += d, send d back (the worker applies x_i -= d)."""
        bufs = self._recv_elastic[w]
        _wait_all([_irecv(b, w, self.pg) for b in bufs])
        with torch.no_grad():
            for c, b in zip(_elastic_state(self.flat), bufs):
                b.sub_(c).mul_(self.elastic_alpha)
                c.add_(b)
            for g in self.flat:
                g.refresh_mirror()
        _wait_all(self._send_works[w])
        snap = self._snap_elastic[w]
        for s_, b in zip(snap, bufs):
            s_.copy_(b)
        self._send_works[w] = [_isend(s_, w, self.pg) for s_ in snap]
        self.version += 1
        self.updates += 1
        self.per_worker[w] += 1

    def enable_elastic(self, alpha):
        """Serve EASGD exchanges: the PS parameters are the elastic center variable x~."""
        self.elastic_alpha = float(alpha)
        self._recv_elastic = {w: [torch.empty_like(t) for t in _elastic_state(self.flat)] for w in self.workers}
        self._snap_elastic = {w: [torch.empty_like(t) for t in _elastic_state(self.flat)] for w in self.workers}
        return self

    def _sync(self):
        """Wait for the apply stream only: a device-wide synchronize would also wait on every pair stream,
        and a parameter send to a worker that was lost mid-run never completes with RCCL (those sends are
        deliberately left unjoined)."""
        if self.dev.type == "cuda":
            torch.cuda.current_stream(self.dev).synchronize()

    def serve(self, poll_sleep=None):
        """Serve requests in arrival order until every worker is done or lost.  (``poll_sleep`` is
        accepted for compatibility; the loop blocks in the native queue and never polls.)"""
        import time
        live = set(self.workers)
        for w in self.workers:
            self._send_params(w)
        while live:
            tok = self._ctl.next(self.worker_timeout)
            if tok is None:
                raise TimeoutError("async PS: no request from workers %s in %.0f s" % (sorted(live),
                                                                                       self.worker_timeout))
            if tok < 0:
                w = -tok - 1
                if w in live:
                    live.discard(w)
                    self.lost.append(w)
                    print("[dtg.async_ps] worker rank %d lost (its control connection closed); continuing with %s"
                          % (w, sorted(live)), file=sys.stderr, flush=True)
                continue
            w, kind = divmod(tok, _KINDS)
            if kind == _DONE:
                live.discard(w)
            elif kind == _WARM:
                self._warm.add(w)
                if self._warm >= set(self.workers) - set(self.lost) and self.timed is None:
                    self._sync()
                    self.timed = (self.updates, time.perf_counter())
            elif kind == _ELASTIC:
                self._elastic(w)
            else:
                self._grad(w)
        for w in self.workers:
            if w not in self.lost:
                _wait_all(self._send_works[w])
            self._send_works[w] = []
        self._sync()
        self.timed_end = (self.updates, time.perf_counter())
        return self.updates

    def close(self):
        self._ctl.close()


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
        self.rank = dist.get_rank()
        self._ctl = _Control(False, self.rank)
        self._d = [torch.empty_like(t) for t in _elastic_state(flat)]
        self.local_step = 0
        self.exchanges = 0

    def begin(self):
        """Start from the center: receive the PS parameters (mirror / fp32 group) into the replica."""
        _wait_all([_irecv(t, self.ps, self.pg) for t in _group_payload_params(self.flat)])
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
        self._ctl.request(self.rank, _ELASTIC)
        _wait_all([_isend(t, self.ps, self.pg) for t in _elastic_state(self.flat)])
        _wait_all([_irecv(d, self.ps, self.pg) for d in self._d])
        with torch.no_grad():
            for t, d in zip(_elastic_state(self.flat), self._d):
                t.sub_(d)
            for g in self.flat:
                g.refresh_mirror()
        self.exchanges += 1
        return True

    def finish(self):
        self._ctl.unwatch()
        try:
            self._ctl.request(self.rank, _DONE)
        except RuntimeError as e:
            # the last worker's DONE lets the PS leave serve() and close its control service; the service can go
            # down before the reply to that enqueue is flushed.  A lost connection here loses nothing: this worker
            # has no further requests, and a PS that died earlier already failed the pushes above.
            if "connection lost" not in str(e):
                raise
        self._ctl.close()


def init_from_cluster(cluster, job_name, task_index, backend=None, port_offset=1):
    """Bootstrap the RCCL/gloo process group from a TF-style ClusterSpec: the PS task 0 is rank 0
    (its ``host:port`` + ``port_offset`` is the rendezvous), worker i is rank 1 + i.  One process per
    GPU: rank r uses device r % (visible devices), with every device left visible to every process
    (examples/ResNet50/run_async.sh) -- RCCL can only use the direct xGMI peer links between GPUs a process
    can see, so pinning each process to one device with HIP_VISIBLE_DEVICES would hide its peers.  On one
    card (the gloo rehearsal) every rank lands on device 0.  Returns (rank, world, device)."""
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
    if backend == "nccl" or gloo_cuda:
        device = torch.device("cuda", rank % max(1, torch.cuda.device_count()))
    else:
        device = torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    os.environ["MASTER_ADDR"] = "127.0.0.1" if ps_host in ("localhost", "") else ps_host
    os.environ["MASTER_PORT"] = str(int(ps_port) + port_offset)
    kw = {"device_id": device} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600), **kw)
    return rank, world, device
