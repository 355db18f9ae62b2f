"""SyncReplicasOptimizer (SURVEY §2.3 "Synchronous SGD", §2.5 N6/N7, §7.5 item 4).

Two execution modes behind one API:

* **PS-accumulator mode** (the reference's semantics; used whenever the variables live on a PS or
  ``replicas_to_aggregate < total_num_replicas``): every worker pushes its gradients into a
  per-variable ConditionalAccumulator on the PS (stale gradients, whose ``local_step`` is behind the
  accumulator's global step, are dropped), then blocks on the sync-token queue.  The chief runs an
  aggregation thread (TF's chief QueueRunner): take ``replicas_to_aggregate`` gradients per
  variable (their mean), apply them with the wrapped optimizer on the PS, bump ``global_step``,
  advance the accumulators and enqueue one token per replica.  With M workers aggregating N < M,
  M - N gradients per step are backups and get dropped (Synchronous-SGD/README.md:3).
  Native pieces: csrc/ps/server.cc ACC_* and Q_* ops.

* **All-reduce mode** (no PS and ``replicas_to_aggregate == total_num_replicas`` == the process-group size): one
  gradient per rank, summed by RCCL (gloo on CPU) and averaged, so every replica applies the same update --
  what the accumulator computes when nobody is stale, without the PS round trips.  Two forms:

  - eager GPU models: the wrapped optimizer is a fused flat optimizer (``dtg.optim``) -- or a tf.train
    optimizer plus ``var_list=<FlatParams>`` -- and ``minimize(loss_fn, global_step, inputs=...)`` takes a
    callable.  The train op is forward + backward with bucketed all-reduces fired from inside the backward,
    then ``DataParallel.step`` (each bucket applied as its collective lands; train/eager.py);
  - graph variables that are not on a PS (the toy graph): ``apply_gradients`` all-reduces each gradient and
    applies the wrapped optimizer locally on every replica.

  ``make_session_run_hook`` broadcasts the chief's state (restored from a checkpoint, or freshly initialised)
  to every rank once the session exists.  Backup workers (R < M) need the accumulator: all-reduce has no
  stale gradient to drop, so that combination is refused.
"""
import os
import threading
import time

import numpy as np
import torch

from .. import graph as G
from ..graph import Op, Tensor
from ..variables import Variable, _as_np
from .hooks import SessionRunHook
from .optimizer import Optimizer

TOKEN_QUEUE = "sync_token_q"


class SyncReplicasOptimizer(Optimizer):
    def __init__(self, opt, replicas_to_aggregate, total_num_replicas=None, variable_averages=None,
                 variables_to_average=None, use_locking=False, name="sync_replicas", bucket_mb=25.0,
                 process_group=None):
        from .eager import is_flat_optimizer
        super().__init__(opt.lr if is_flat_optimizer(opt) else opt._lr, use_locking, name)
        self._opt = opt
        self._bucket_mb = float(bucket_mb)
        self._pg = process_group
        self.dp = None              # all-reduce mode over a FlatParams model: its DataParallel
        self.mode = None            # "ps" | "allreduce" (decided when the train op is built)
        self._flat_opt = opt if is_flat_optimizer(opt) else None
        self._replicas_to_aggregate = int(replicas_to_aggregate)
        self._total_num_replicas = int(total_num_replicas or replicas_to_aggregate)
        self._tokens_per_step = max(self._total_num_replicas, self._replicas_to_aggregate)
        self._gv = None
        self._global_step = None
        self.local_step = 0
        self._stop_check = None
        self._chief_thread = None
        self._chief_stop = threading.Event()
        self.dropped = 0
        # strict lock-step (dtg extension, enabled by num_tokens == 0 in the hook): one token queue
        # per worker, so every replica contributes exactly one fresh gradient per global step
        self.strict = False
        # seconds a worker waits for the chief's next token before failing (a lost worker without backups)
        self.sync_timeout = float(os.environ.get("DTG_SYNC_TIMEOUT", "600"))

    def _token_queue(self, task=None):
        if not self.strict:
            return TOKEN_QUEUE
        if task is None:
            from ..variables import _this_server
            s = _this_server()
            task = s.task_index if s is not None else 0
        return "%s/%d" % (TOKEN_QUEUE, task)

    # ---- all-reduce mode ------------------------------------------------------------------------
    def _world(self):
        import torch.distributed as dist
        return dist.get_world_size(self._pg) if dist.is_available() and dist.is_initialized() else 1

    def _check_allreduce(self):
        if self._replicas_to_aggregate != self._total_num_replicas:
            raise ValueError(
                "replicas_to_aggregate=%d < total_num_replicas=%d (backup workers) needs the PS-accumulator mode: "
                "all-reduce has no stale gradient to drop -- place the variables on a PS (replica_device_setter)"
                % (self._replicas_to_aggregate, self._total_num_replicas))
        w = self._world()
        if self._total_num_replicas != w:
            raise ValueError("all-reduce mode: total_num_replicas=%d but the process group has %d rank(s) (one "
                             "replica per process)" % (self._total_num_replicas, w))
        self.mode = "allreduce"

    def _flat_for(self, var_list):
        from ..parallel.flat import FlatParams
        from .eager import fused_from_tf
        if self._flat_opt is None:
            if not isinstance(var_list, FlatParams):
                raise TypeError("an eager train op wraps a fused flat optimizer (dtg.optim) or gets "
                                "var_list=<FlatParams> for a tf.train optimizer")
            self._flat_opt = fused_from_tf(self._opt, var_list)
        return self._flat_opt

    def _data_parallel(self):
        if self.dp is None:
            from ..parallel.ddp import DataParallel
            self.dp = DataParallel(self._flat_opt.flat, process_group=self._pg, bucket_mb=self._bucket_mb)
        return self.dp

    def minimize(self, loss, global_step=None, var_list=None, name=None, inputs=()):
        """``loss`` callable (an eager model's ``loss_fn(*inputs)``): the all-reduce train op of train/eager.py.
        Otherwise the graph form: compute_gradients + apply_gradients."""
        if not callable(loss) or isinstance(loss, G.Node):
            return super().minimize(loss, global_step=global_step, var_list=var_list, name=name)
        self._flat_for(var_list)
        self._check_allreduce()
        self._global_step = global_step
        from .eager import minimize as eager_minimize
        return eager_minimize(self._flat_opt, loss, global_step, inputs, self._data_parallel(),
                              name or "sync_replicas_train")

    # ------------------------------------------------------------------------------------------
    def compute_gradients(self, *args, **kwargs):
        return self._opt.compute_gradients(*args, **kwargs)

    def apply_gradients(self, grads_and_vars, global_step=None, name=None):
        if global_step is None:
            raise ValueError("SyncReplicasOptimizer.apply_gradients needs global_step")
        self._gv = [(g, v) for g, v in grads_and_vars]
        self._global_step = global_step
        remote = [isinstance(v, Variable) and v.remote for _, v in self._gv]
        if not any(remote):
            self._check_allreduce()
            return _AllReduceTrainOp(self, name or "sync_replicas_train")
        if not all(remote):
            raise ValueError("SyncReplicasOptimizer: some variables are on a parameter server and some are not")
        self.mode = "ps"
        self.chief_init_op = Op(lambda c: self._init_local_step(), [], "sync_rep_local_step_init")
        self.local_step_init_op = self.chief_init_op
        self.ready_for_local_init_op = _ReadyForLocalInit(self)
        return _SyncTrainOp(self, name or "sync_replicas_train")

    # ------------------------------------------------------------------------------------------
    def _acc_name(self, v):
        return v._name + "/grad_accum"

    def _gs_client(self):
        return self._global_step._client()

    def _read_gs(self):
        return int(self._global_step.read_value().item())

    def _ensure_accumulators(self, step=None):
        step = self._read_gs() if step is None else step
        for _, v in self._gv:
            v._client().acc_create(self._acc_name(v), np.zeros(v.shape, np.float32), int(step))

    def _init_local_step(self):
        self.local_step = self._read_gs()
        self._ensure_accumulators(self.local_step)

    def get_init_tokens_op(self, num_tokens=-1):
        tokens_needed = self._replicas_to_aggregate - self._total_num_replicas
        if num_tokens == -1:
            num_tokens = self._replicas_to_aggregate
        elif num_tokens < tokens_needed:
            raise ValueError("Too few tokens to finish the first step: %d (given) vs %d (needed)"
                             % (num_tokens, tokens_needed))

        def run(ctx):
            if num_tokens > 0:
                gs = self._read_gs()
                self._gs_client().q_enqueue(TOKEN_QUEUE, [gs] * num_tokens)
        return Op(run, [], "sync_replicas/init_tokens")

    def make_session_run_hook(self, is_chief, num_tokens=-1):
        if self.mode == "allreduce":
            return _AllReduceSyncHook(self, is_chief)
        return _SyncReplicasHook(self, is_chief, num_tokens)

    # ---- chief aggregation loop (TF: get_chief_queue_runner) ---------------------------------
    def _chief_loop(self):
        from ..variables import new_client
        opt = self._opt
        gv = self._gv
        gs = self._global_step
        conns = {}

        def cl(v):  # this thread's own connections: its blocking acc_take must not starve the training thread
            c = conns.get(v.ps_task)
            if c is None:
                c = conns[v.ps_task] = new_client(*v.ps_task)
            return c
        try:
            self._chief_steps(opt, gv, gs, cl)
        finally:
            for c in conns.values():
                c.close()

    def _chief_steps(self, opt, gv, gs, cl):
        while not self._chief_stop.is_set():
            grads = []
            for _, v in gv:
                g = None
                while g is None and not self._chief_stop.is_set():
                    g = cl(v).acc_take(self._acc_name(v), self._replicas_to_aggregate, 0.25)
                if g is None:
                    return
                grads.append(g)
            lr = float(opt._lr) if not isinstance(opt._lr, Tensor) else float(G.RunContext().eval(opt._lr))
            opt._t += 1
            by_task = {}
            for g, (_, v) in zip(grads, gv):
                by_task.setdefault(v.ps_task, []).append((v._name, np.array(g, dtype=np.float32, order="C")))
            new_step = None
            for task, items in by_task.items():
                gs_name = gs._name if (gs.remote and gs.ps_task == task and new_step is None) else ""
                client = cl([v for _, v in gv if v.ps_task == task][0])
                step, _ = client.apply(opt.PS_KIND, opt._hyper(lr), bool(opt._use_locking), gs_name, items, False)
                if gs_name:
                    new_step = step
            if new_step is None:
                new_step = int(cl(gs).assign_add(gs._name, np.ones((), _np(gs.dtype))))
            for _, v in gv:
                cl(v).acc_set_step(self._acc_name(v), int(new_step))
            if self.strict:
                for t in range(self._total_num_replicas):
                    cl(gs).q_enqueue(self._token_queue(t), [int(new_step)])
            else:
                cl(gs).q_enqueue(TOKEN_QUEUE, [int(new_step)] * self._tokens_per_step)

    def start_chief(self):
        if self._chief_thread is None:
            self._chief_stop.clear()
            self._chief_thread = threading.Thread(target=self._chief_loop, name="sync_replicas_chief", daemon=True)
            self._chief_thread.start()

    def stop_chief(self):
        self._chief_stop.set()
        if self._chief_thread is not None:
            self._chief_thread.join(timeout=5)
            self._chief_thread = None


def _np(dt):
    return {torch.int32: np.int32, torch.int64: np.int64}.get(dt, np.float32)


class SyncTimeoutError(RuntimeError):
    """A synchronous step could not be aggregated in time (TF: DeadlineExceededError)."""


class _ReadyForLocalInit(Tensor):
    def __init__(self, opt):
        self._opt = opt
        super().__init__(lambda c: None, [], "report_uninitialized_variables_1")

    def _eval(self, ctx):
        names = [v._name for _, v in self._opt._gv if not v.is_initialized()]
        if not self._opt._global_step.is_initialized():
            names.append(self._opt._global_step._name)
        return np.array(names, dtype=object)


class _SyncTrainOp(Op):
    """Worker side of one synchronous step: push grads into the accumulators, wait for a token."""

    def __init__(self, sro, name):
        self.sro = sro
        super().__init__(lambda c: None, [g for g, _ in sro._gv], name)

    def _eval(self, ctx):
        sro = self.sro
        grads = [ctx.eval(g) for g, _ in sro._gv]
        for g, (_, v) in zip(grads, sro._gv):
            ok = v._client().acc_apply(sro._acc_name(v), int(sro.local_step), _as_np(g.float()))
            if not ok:
                sro.dropped += 1
        client = sro._gs_client()
        import time
        t0 = time.monotonic()
        while True:
            tok = client.q_dequeue(sro._token_queue(), 0.5)
            if tok is not None:
                sro.local_step = int(tok)
                return None
            sess = ctx.session
            if sess is not None and sess._stop_requested_externally():
                return None
            if time.monotonic() - t0 > sro.sync_timeout:
                raise SyncTimeoutError(
                    "SyncReplicasOptimizer: no aggregated step for %.0f s -- fewer than replicas_to_aggregate=%d "
                    "workers are pushing gradients (a worker may be lost).  With total_num_replicas > "
                    "replicas_to_aggregate the surplus workers are backups and the job survives such a loss."
                    % (sro.sync_timeout, sro._replicas_to_aggregate))


class _SyncReplicasHook(SessionRunHook):
    def __init__(self, sro, is_chief, num_tokens):
        self._sro = sro
        self._is_chief = is_chief
        self._num_tokens = num_tokens
        sro.strict = num_tokens == 0

    def after_create_session(self, session, coord):
        sro = self._sro
        if self._is_chief:
            sro._init_local_step()
            G.RunContext(session).eval(sro.get_init_tokens_op(self._num_tokens))
            sro.start_chief()
        else:
            sro._init_local_step()

    def end(self, session):
        if self._is_chief:
            self._sro.stop_chief()


class _AllReduceTrainOp(Op):
    """All-reduce mode for graph variables that live on the workers: every replica evaluates its gradients, they
    are summed over the process group and averaged, and every replica applies the wrapped optimizer's rule
    locally -- the same update on every rank, one global step per run."""

    def __init__(self, sro, name):
        self.sro = sro
        super().__init__(lambda c: None, [g for g, _ in sro._gv], name)

    def _eval(self, ctx):
        import torch.distributed as dist
        sro = self.sro
        opt = sro._opt
        grads = [ctx.eval(g) for g, _ in sro._gv]
        w = sro._world()
        if w > 1:
            # one flat fp32 buffer: a single collective per step
            flat = torch.cat([g.detach().float().reshape(-1) for g in grads])
            dist.all_reduce(flat, group=sro._pg)
            flat /= w
            out, off = [], 0
            for g in grads:
                out.append(flat[off:off + g.numel()].view(g.shape))
                off += g.numel()
            grads = out
        lr = opt._lr_value(ctx)
        opt._t += 1
        for g, (_, v) in zip(grads, sro._gv):
            if g is not None:
                opt._apply_local(v, g, lr)
        gs = sro._global_step
        with gs._lock:
            gs._local.add_(1)
        return None


class _AllReduceSyncHook(SessionRunHook):
    """All-reduce mode: once the session exists (the chief has restored its checkpoint or initialised), every
    rank takes the chief's parameters, buffers, optimizer state and global step -- TF's chief-init + token
    rendezvous collapsed into one broadcast."""

    def __init__(self, sro, is_chief):
        self._sro = sro
        self._is_chief = is_chief

    def after_create_session(self, session, coord):
        sro = self._sro
        if sro._world() == 1:
            return
        if sro._flat_opt is not None and sro.dp is not None:
            from .eager import broadcast_training_state
            broadcast_training_state(sro._flat_opt.flat, sro._flat_opt, sro.dp, sro._global_step, 0, sro._pg)
            return
        import torch.distributed as dist
        for _, v in sro._gv:
            t = v.read_value()
            dist.broadcast(t, 0, group=sro._pg)
        for s in _slot_tensors(sro._opt, [v for _, v in sro._gv]):
            dist.broadcast(s, 0, group=sro._pg)
        gs = sro._global_step
        t = gs.read_value()
        dist.broadcast(t, 0, group=sro._pg)


def _slot_tensors(opt, vars_):
    out = []
    for v in vars_:
        for k in opt.get_slot_names():
            s = opt.get_slot(v, k)
            if isinstance(s, torch.Tensor):
                out.append(s)
    return out
