"""Synchronous data parallelism: bucketed RCCL all-reduce overlapped with backward.

This is the fast path of ``SyncReplicasOptimizer`` (replicas_to_aggregate == total_num_replicas,
no PS) and the BASELINE north-star config ("ResNet-50 bf16 sync all-reduce DP
on 8x MI355X").  One process per GPU, ``torch.distributed`` backend "nccl" (= RCCL on ROCm) over
xGMI; "gloo" for CPU tests.

Design:
* gradients live in the flat buffers of :class:`FlatParams`; a bucket is a contiguous slice of a
  group's flat grad buffer (no flatten copies) -- the buffer is laid out in backward order;
* a post-accumulate-grad hook per parameter counts down its bucket; when the last gradient of a
  bucket lands, its all-reduce (SUM) is issued asynchronously.  RCCL runs on its own stream and
  waits on the compute stream's event at launch, so it overlaps the rest of backward;
* ``finish()`` joins all outstanding collectives into the compute stream; the 1/world averaging is
  folded into the optimizer's gradient scale (no separate divide kernel);
* bucket size (constructor default 32 MB; bench.py passes 8 MB for ResNet-50 and 25 MB for BERT): large
  enough to amortise the ~tens-of-µs RCCL launch against the xGMI link rate, small enough that the
  last bucket -- the only one left to reduce after backward ends -- is short (sweep with
  ``tools/allreduce_bw.py`` and ``bench.py --bucket_mb``).
"""
import os

import torch
import torch.distributed as dist

from . import grad_sink, overlap
from ..utils.trace import trace_range



_EMU_MODES = {"busy": 1, "traffic": 2, "data": 4}


def _parse_emulate(spec):
    """DTG_COMM_EMULATE="<busbw GB/s>[,<ranks>[,<workgroups>[,<latency us>[,<modes>]]]]" (defaults 8 ranks, 32
    workgroups, 10 us, no modes); modes = "+"-joined subset of busy, traffic, data (csrc/kernels/comm_emu.hip):
    busy-polling waves, the ring's HBM traffic, and the bucket multiplied by the rank count (N identical
    replicas summed).  See :meth:`DataParallel._emulate`."""
    if not spec:
        return None
    parts = spec.split(",")
    modes = 0
    if len(parts) >= 5:
        for m in filter(None, parts[4].split("+")):
            if m not in _EMU_MODES:
                raise ValueError("DTG_COMM_EMULATE: unknown mode %r (busy, traffic, data)" % m)
            modes |= _EMU_MODES[m]
        parts = parts[:4]
    f = [float(v) for v in parts]
    f += [8, 32, 10][len(f) - 1:]
    return {"busbw_GBps": f[0], "ranks": int(f[1]), "wgs": int(f[2]), "latency_us": f[3], "modes": modes}


EMULATE = _parse_emulate(os.environ.get("DTG_COMM_EMULATE", ""))


class _Bucket:
    __slots__ = ("group", "start", "end", "params", "pending", "work", "index", "seq", "emu_event")

    def __init__(self, group, start, index):
        self.group = group
        self.start = start
        self.end = start
        self.params = []
        self.pending = 0
        self.work = None
        self.index = index
        self.seq = 0            # launch order within the step (DataParallel.step applies in that order)
        self.emu_event = None   # DTG_COMM_EMULATE: the emulated collective of this bucket done

    def view(self):
        return self.group.grad[self.start:self.end]


class DataParallel:
    def __init__(self, flat, process_group=None, bucket_mb=32.0, overlap=True):
        self.flat = flat
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        forced = os.environ.get("DTG_DDP_FORCE") == "1" and dist.is_available() and dist.is_initialized()
        self.overlap = overlap and (self.world > 1 or forced)
        self._force = forced
        self._comm = True  # set_comm(False): gradients stay rank-local (bench.py's compute-only timing)
        self._estreams = {}
        self._escratch = {}  # device index -> [scratch buffer, window offset] (traffic mode)
        self._qprobe = {}    # device index -> out-of-place all-gather target (DTG_COMM_QUEUE_PROBE)
        # the emulated collective stands in for peers a one-rank run does not have: with real peers it would
        # add spin kernels on top of the real collectives and skew the scaling numbers, so it is refused there
        if EMULATE is not None and self.world > 1:
            import warnings
            warnings.warn("DTG_COMM_EMULATE is ignored at world size %d (one-rank rehearsals only)" % self.world)
        self.emulate = EMULATE if (self.overlap and self.world == 1) else None
        self.buckets = []
        self._hooks = []
        cap = int(bucket_mb * (1 << 20))
        for g in flat:
            esz = g.grad.element_size()
            b = None
            for i, (name, p, off, n) in enumerate(g.param_slices()):
                if b is None or (b.end - b.start) * esz >= cap:
                    b = _Bucket(g, off, len(self.buckets))
                    self.buckets.append(b)
                b.params.append(p)
                nxt = g.offsets[i + 1] if i + 1 < len(g.offsets) else g.numel
                b.end = nxt
        self._param_bucket = {}
        for b in self.buckets:
            for p in b.params:
                self._param_bucket[p] = b
        if self.overlap:
            for p in self._param_bucket:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
            grad_sink.add_listener(self._on_direct)
        self._reset()

    # -- hooks ---------------------------------------------------------------------------------
    # A parameter counts towards its bucket exactly once per backward.  Direct-write ops
    # (grad_sink.notify) report from inside their backward; autograd ALSO runs the parameter's
    # AccumulateGrad node afterwards (with an undefined gradient, since the op returned None) and
    # that fires the post-accumulate hook a second time -- it must not count again, or a bucket
    # would launch its all-reduce while some of its gradients are still being computed.
    def _reset(self):
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
            b.emu_event = None
        self._done = set()
        self._nlaunched = 0

    def _launch(self, b):
        b.seq = self._nlaunched
        self._nlaunched += 1
        v = b.view()
        side = overlap.pending_stream(v)
        with trace_range("dtg.allreduce.bucket%d" % b.index):  # roctx range (DTG_TRACE=1)
            if side is not None and dist.get_backend(self.pg) == "nccl":
                # weight gradients of this bucket may still be running on the side stream (parallel/overlap.py),
                # its BN-parameter gradients come from main-stream kernels.  The side stream waits for the
                # main stream's event at this point and the collective is enqueued FROM the side stream, so
                # RCCL's stream waits for both.  No third stream: main + side + RCCL's own stream fit the four
                # hardware queues a HIP process gets by default (GPU_MAX_HW_QUEUES=4), where a separate
                # launch stream made two streams share a queue and serialise (profiles/r03_streams).  The
                # side stream's later wgrads need the main stream's later dgrads anyway, so the wait costs
                # it nothing.
                main = torch.cuda.current_stream(v.device)
                ls = side
                ls.wait_stream(main)
                with torch.cuda.stream(ls):
                    b.work = dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
                    if os.environ.get("DTG_COMM_QUEUE_PROBE") == "1" and self.world == 1:
                        # one-rank out-of-place all-gather: RCCL copies on the process group's own stream, so a
                        # kernel trace shows that stream's hardware queue (the in-place all-reduce issues nothing)
                        out = self._qprobe.get(v.device.index)
                        if out is None or out.numel() < v.numel() or out.dtype != v.dtype:
                            out = self._qprobe[v.device.index] = torch.empty_like(v)
                        dist.all_gather_into_tensor(out[:v.numel()], v, group=self.pg, async_op=True).wait()
                b.emu_event = self._emulate(v, ls)
                return
            if side is not None:
                # host-staged backends (gloo): the main stream waits for the side stream (an event, no host
                # sync) and the collective is enqueued from the main stream exactly as without it
                torch.cuda.current_stream(v.device).wait_stream(side)
            b.work = dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            b.emu_event = self._emulate(v, torch.cuda.current_stream(v.device) if v.is_cuda else None)

    def _emulate(self, v, after):
        """DTG_COMM_EMULATE: make a one-card run pay what an N-rank RCCL all-reduce of this bucket costs the
        chip.  A one-rank collective is a local copy that never waits on a peer, so it cannot show whether the
        real one -- RCCL channel workgroups resident on CUs for the whole bus time, blocked on peers -- delays
        the backward's remaining weight gradients (the overlap that decides 1->8 scaling).  After the real
        collective is enqueued, an emulation kernel (csrc/kernels/comm_emu.hip) holding ``wgs`` workgroups for
        ``bytes * 2(N-1)/N / busbw + latency`` runs on a high-priority pool stream -- drawn from the same
        torch stream pool, at the same priority, as the process group's collective stream -- after everything
        the launching stream has queued; :meth:`finish` makes the main stream wait for it, as for the real
        work.  Successive buckets serialise on that stream like collectives on RCCL's.

        Modes (round 5, the pessimistic forms): ``busy`` -- every wave busy-polls, as RCCL's primitives do;
        ``traffic`` -- the workgroups stream 2 x 2(N-1)/N x bucket bytes (read + written) through a 1 GiB scratch
        buffer over the emulated time, the HBM traffic the ring adds next to the HBM-bound backward; ``data``
        -- after the wait the bucket is read and written back times N (N identical replicas summed), so a test
        sees every gradient of the bucket final when the collective read it (the optimizer then scales by
        1/N, :attr:`grad_scale`)."""
        e = self.emulate
        if e is None or after is None:
            return
        from ..ops._native import lib
        idx = v.device.index
        es = self._estreams.get(idx)
        if es is None:
            es = self._estreams[idx] = torch.cuda.Stream(device=v.device, priority=-1)
        n = e["ranks"]
        nbytes = v.numel() * v.element_size()
        secs = nbytes * 2.0 * (n - 1) / n / (e["busbw_GBps"] * 1e9) + e["latency_us"] * 1e-6
        es.wait_stream(after)
        modes = e.get("modes", 0)
        ev = torch.cuda.Event()
        with torch.cuda.stream(es):
            if modes == 0:
                lib().comm_spin(secs, e["wgs"], 0)
                ev.record(es)
                return ev
            scratch = None
            traffic = 0
            if modes & 2:
                sc = self._escratch.get(idx)
                if sc is None:
                    sc = self._escratch[idx] = [torch.empty(1 << 30, dtype=torch.uint8, device=v.device), 0]
                scratch = sc[0]
                traffic = int(2 * nbytes * 2.0 * (n - 1) / n)
            used = lib().comm_emu(secs, e["wgs"], modes, scratch, sc[1] if scratch is not None else 0, traffic,
                                  v if modes & 4 else None, float(n))
            if scratch is not None:
                sc[1] += used
            ev.record(es)
        return ev

    def _on_direct(self, p):
        if p in self._param_bucket:
            self._count(p)

    def _on_grad(self, p):
        self._count(p)

    def _count(self, p):
        if p in self._done:
            return
        self._done.add(p)
        b = self._param_bucket[p]
        b.pending -= 1
        if b.pending == 0 and self._comm:
            self._launch(b)

    # -- step ------------------------------------------------------------------------------------
    @property
    def grad_scale(self):
        """Factor the optimizer applies to the summed gradients (1/world: mean; the emulated data mode sums
        ``ranks`` identical replicas, so 1/ranks there)."""
        if self.emulate is not None and self.emulate.get("modes", 0) & 4:
            return 1.0 / self.emulate["ranks"]
        return 1.0 / self.world

    def finish(self):
        """Wait for every bucket's all-reduce (launching any that did not fire)."""
        overlap.join()  # (normally already joined at the end of backward)
        if not self._comm:
            self._reset()
            return
        if self.world == 1 and not self._force:
            return
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        for b in self.buckets:
            b.work.wait()
        for es in self._estreams.values():
            torch.cuda.current_stream(es.device).wait_stream(es)
        self._reset()

    def step(self, opt, zero_grad=True):
        """finish() + opt.step(), with the apply overlapped with the collective tail: every bucket's slice of the
        flat buffers is applied as soon as ITS all-reduce has landed (the main stream waits per bucket, in
        launch order), so the applies of the buckets reduced during backward run while the last buckets -- the
        layers backward reaches last, e.g. BERT's word embeddings -- are still on the wire.  Bit-identical to
        finish() + opt.step(grad_scale=self.grad_scale) (the fused applies are elementwise)."""
        if not (self.overlap and self._comm) or (self.world == 1 and not self._force):
            self.finish()
            return opt.step(grad_scale=self.grad_scale, zero_grad=zero_grad)
        overlap.join()
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        order = sorted(self.buckets, key=lambda b: b.seq)
        estreams = list(self._estreams.values())

        def ready_fn(b):
            def ready():
                b.work.wait()
                if b.emu_event is not None:
                    torch.cuda.current_stream().wait_event(b.emu_event)
            return ready
        ranges = [(b.group, b.start, b.end, ready_fn(b)) for b in order]
        # zero-width gaps are impossible (buckets tile each group), but a group with no bucket would be missed
        covered = {id(b.group) for b in self.buckets}
        for g in self.flat:
            if id(g) not in covered:
                ranges.append((g, 0, g.numel, lambda: None))
        out = opt.step(grad_scale=self.grad_scale, zero_grad=zero_grad, ranges=ranges)
        for es in estreams:
            torch.cuda.current_stream(es.device).wait_stream(es)
        self._reset()
        return out

    def set_comm(self, on):
        """Turn the gradient collectives off (on=False: every rank steps on its own gradients) or back on.
        bench.py times a few steps this way after the timed region, so its JSON line can split a multi-GPU
        step into compute and exposed communication."""
        self._comm = bool(on)
        self._reset()

    def broadcast_parameters(self, src=0):
        """Chief broadcast of initial weights and module buffers (replaces the reference's
        ``assign_global`` + ``sleep(10)`` bootstrap, DOWNPOUR/DOWNPOUR.py:129-135)."""
        if self.world == 1:
            return
        for g in self.flat:
            dist.broadcast(g.master, src, group=self.pg)
            g.refresh_mirror()
        for buf in self.flat.module.buffers():
            if buf.is_floating_point() or buf.dtype in (torch.int64, torch.int32):
                dist.broadcast(buf, src, group=self.pg)

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        grad_sink.remove_listener(self._on_direct)
