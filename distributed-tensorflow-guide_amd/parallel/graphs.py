"""Whole-step HIP-graph capture: forward + backward + gradient reduction + fused optimizer apply
recorded once into a hipGraph and replayed, so a training step costs one graph launch on the host.

This is dtg's answer to a tracing compiler (eager PyTorch-ROCm + hand-written
kernels): nothing is re-traced or re-compiled, the exact kernel sequence of an eager step is
recorded (hipStreamBeginCapture under ``torch.cuda.graph``) and replayed with zero Python, zero
dispatcher and zero per-kernel launch cost.  Every dtg op is capture-safe by construction
(csrc/bindings/ops.cc: outputs from the caching allocator, launches on the current stream, no
host synchronisation; optimizer hyper-parameters live in a device tensor, optim/fused.py).

Rules for a capturable ``step_fn``:
  * its inputs are static tensors (refill them in place between replays, e.g. ``x.copy_(batch)``);
  * it returns tensors (the loss); after a replay they hold that replay's values;
  * no host reads (``.item()``), no data-dependent Python control flow;
  * world size 1 (or a backend whose collectives are capture-safe): the bucketed all-reduce hooks of
    ``DataParallel`` fire from Python during backward; under capture they would be recorded once, so
    multi-rank steps stay eager (``capture_supported``).

The host-side optimizer step counter (``opt.step_count``) advances only during warmup/capture; the
DEVICE counter the kernels read (``opt.hyper[1]``) advances on every replay, which is what Adam's
bias correction uses.
"""
import torch


def capture_supported(world_size=1):
    """Graph capture needs a GPU; multi-rank steps keep their collectives eager."""
    return torch.cuda.is_available() and world_size == 1


class GraphedStep:
    """Capture ``step_fn`` on first call (after ``warmup`` eager runs on a side stream, which
    initialise lazily allocated workspaces and library handles outside the capture), then replay.

        step = GraphedStep(lambda: train_step(x, y))
        for _ in range(n):
            loss = step()          # one hipGraphLaunch
    """

    def __init__(self, step_fn, warmup=2, pool=None):
        self.fn = step_fn
        self.warmup = warmup
        self.pool = pool
        self.graph = None
        self.out = None

    @property
    def captured(self):
        return self.graph is not None

    def capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool):
            self.out = self.fn()
        self.graph = g
        return self

    def __call__(self):
        if self.graph is None:
            self.capture()
        self.graph.replay()
        return self.out

    def reset(self):
        """Drop the graph (e.g. after the model or optimizer state buffers were re-allocated)."""
        self.graph = None
        self.out = None
