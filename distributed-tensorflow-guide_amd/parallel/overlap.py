"""Weight gradients on a second HIP stream, overlapped with the rest of backward.

In a layer's backward the data gradient (dgrad) continues the chain to the layer below, while the
weight gradient (wgrad) is a leaf: it reads the layer's output gradient and saved input and writes
the flat gradient buffer, which nothing reads until the all-reduce / optimizer.  dtg's MFMA kernels
run at 25-45 % of the dense MFMA peak at these sizes (profiles/r02_gemm, r02_pmc), so running each
wgrad on a side stream next to the next layer's BN-backward and dgrad kernels fills the chip with two
independent kernels instead of one.

    with overlap.wgrad_scope(dy, x):       # inside an autograd backward
        gemm(dy, False, x, False, out=p.grad, beta=1.0)

* the side stream first waits for everything the main stream has queued (dy is ready);
* every tensor the side stream reads is kept referenced until the join below, so the caching allocator
  cannot hand its memory to a main-stream allocation before the side kernels are done.  (This avoids
  ``record_stream``, which grew the allocator's reserve from 31 to 191 GiB over 25 ResNet-50 b512 steps:
  every recorded block waits for an event before it is reused, so new blocks keep being allocated);
* the first scope of a backward pass queues an autograd end-of-backward callback that makes the main
  stream wait for the side stream, so any consumer after ``backward()`` (optimizer, tests, eager
  reads of ``.grad``) sees finished gradients;
* a gradient all-reduce launched during backward (parallel/ddp.py) first makes the main stream wait
  for the side stream (an event, no host sync), then is enqueued from the main stream as usual.

Several ranks over RCCL: the side stream is used too, and a bucket's collective is enqueued from it
(parallel/ddp.py).  What decides the speed is which HIP streams share a hardware queue: a HIP process
gets GPU_MAX_HW_QUEUES=4 queues by default, streams are bound to queues when torch creates its stream
pools, and two streams on one queue serialise (a cross-stream wait packet blocks the whole queue).  A
rocprofv3 kernel trace (Queue_Id per dispatch) of a one-rank RCCL group (``DTG_DDP_FORCE=1``, ResNet-50
b512; profiles/r03_streams) showed the side stream drawn from torch's pool onto the main stream's queue
once the process group had taken its own pool stream first.  Queues are per priority, so the side stream
is a HIGH-priority stream (its own queue, never the main stream's) and the process group's collective
stream is high-priority too (parallel/comm.py):

- main stream only: 13.86k img/s;  side stream, normal priority: 12.37k (main and side on one queue);
- side high-priority, process group normal: 13.97k;  both high-priority: 14.47k;
- both normal but GPU_MAX_HW_QUEUES=8: 14.50k;  no process group at all: 14.58k.

gloo (host-staged) keeps the wgrads on the main stream: there the side stream ran 9-40x slower
(profiles/r02_overlap), because the staging copies synchronise the host.

``DTG_WGRAD_STREAM=0`` runs every wgrad on the main stream (A/B runs).  ``=2`` forces the side stream
with several gloo ranks too.  Measured gain on one rank:
ResNet-50 +2.3 % (+4 % with the side-stream split targets of models/resnet_fused.py), BERT-base +1.1 %.
The record_stream version once ran a whole bench 5x slower (191 ms/step instead of 37 ms, same losses),
most likely because its allocator reserve kept growing (profiles/r02_overlap).
"""
import contextlib
import os

import torch

_ON = os.environ.get("DTG_WGRAD_STREAM", "1") != "0"
_MULTI = os.environ.get("DTG_WGRAD_STREAM") == "2"  # also with several ranks (rehearsals)
# torch stream priority of the side stream: high (its own hardware queue, see above); DTG_SIDE_PRIO overrides it
# (A/B runs together with bench.py's DTG_MAIN_PRIO, which runs the step itself on a stream of that priority)
_PRIO = int(os.environ.get("DTG_SIDE_PRIO", "-1"))
_side = {}      # device index -> side stream
_main = {}      # device index -> the main stream of the backward the side work belongs to
_pending = set()
_keep = {}      # device index -> tensors the side stream reads, released at the join
_cb_task = {}   # device index -> autograd graph task whose end-of-backward callback joins it


def _host_staged_multi_rank():
    """Several ranks on a backend that stages collectives through host memory (gloo)."""
    import torch.distributed as dist
    return (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
            and dist.get_backend() != "nccl")


def enabled():
    return _ON and (_MULTI or not _host_staged_multi_rank())


def set_enabled(on):
    global _ON
    _ON = bool(on)


def set_side_priority(prio):
    """Priority of the side streams created from now on (bench.py: BERT on one rank, see there)."""
    global _PRIO
    _PRIO = int(prio)


def side_stream(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = _side[idx] = torch.cuda.Stream(device=idx, priority=_PRIO)
    return s


def _join(idx):
    if idx in _pending:
        _main[idx].wait_stream(_side[idx])
        _pending.discard(idx)
        # every later main-stream use of these blocks is ordered after the side stream's work
        _keep.pop(idx, None)


@contextlib.contextmanager
def wgrad_scope(*tensors):
    """Run the enclosed kernel launches on the device's side stream (see module docstring)."""
    t0 = tensors[0] if tensors else None
    if t0 is None or not t0.is_cuda or not enabled():
        yield
        return
    idx = t0.device.index
    main = torch.cuda.current_stream(t0.device)
    side = side_stream(t0.device)
    side.wait_stream(main)
    if idx in _pending and _main[idx] != main:
        _join(idx)  # left over from a scope under another stream: settle it first
    if idx not in _pending:
        _pending.add(idx)
        _main[idx] = main
    # one end-of-backward join per backward pass (graph task): a scope entered outside backward, or a
    # backward that raised before its callback ran, must not stop later passes from queueing theirs
    task = torch._C._current_graph_task_id()
    if task >= 0 and _cb_task.get(idx) != task:
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _join(idx))
        _cb_task[idx] = task
    _keep.setdefault(idx, []).extend(t for t in tensors if t is not None)
    with torch.cuda.stream(side):
        yield


def pending_stream(t):
    """The side stream if it has queued work on t's device this backward pass, else None."""
    if not t.is_cuda:
        return None
    idx = t.device.index
    return _side[idx] if idx in _pending else None


def sync_current(device):
    """Make the current stream wait for the side stream's queued work on ``device`` (an event, no host
    sync) without ending the backward's pending set.  For gradients handed to autograd from inside a
    backward (parameters without a flat gradient buffer): AccumulateGrad may add them into an existing
    ``.grad`` on the current stream right away."""
    if device.type != "cuda":
        return
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx in _pending:
        torch.cuda.current_stream(device).wait_stream(_side[idx])


def join(device=None):
    """Make the main stream wait for all queued side-stream work (no-op when there is none)."""
    for idx in list(_pending):
        if device is None or torch.device(device).index in (None, idx):
            _join(idx)
