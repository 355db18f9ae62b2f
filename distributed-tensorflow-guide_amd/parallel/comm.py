"""Process-group bootstrap: one process per GPU, RCCL ("nccl" backend on ROCm) over xGMI, or gloo
on CPU.  Ranks come from the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*)
or from a :class:`dtg.ClusterSpec` (job "worker", task_index = rank).

Failure detection (the reference's sync replicas wait on a chief that may be gone,
Synchronous-SGD/ssgd.py:65-69): RCCL communicators cannot shrink, so a lost rank is fail-stop.  What
matters is to stop quickly and say who is gone: every rank runs a :class:`Watchdog` thread that
heartbeats into the job's TCP store and watches its peers' heartbeats.  A peer silent for
``DTG_RANK_TIMEOUT`` seconds (default 60) -- crashed, killed, or its host gone -- makes every survivor
print which rank was lost and exit with status 75, instead of sitting in a collective for the
``DTG_COLLECTIVE_TIMEOUT`` (default 600 s) process-group timeout.  The job is then restarted and resumes
from its last ``save_flat`` checkpoint (examples/ResNet50/resnet50_train.py).
"""
import datetime
import os
import sys
import threading
import time

import torch
import torch.distributed as dist

LOST_RANK_EXIT = 75


def env_rank():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")), int(
        os.environ.get("WORLD_SIZE", "1"))


def init(backend=None, timeout_s=None, watchdog=True):
    """Initialise the default process group from the environment (no-op for world_size 1).

    ``watchdog=False`` skips the fail-stop rank :class:`Watchdog` -- for jobs that survive a lost rank on
    their own (the async parameter server, parallel/async_ps.py, also stops it when it is constructed).
    Returns (rank, local_rank, world, device)."""
    rank, local, world = env_rank()
    # DTG_BACKEND=gloo with DTG_GLOO_DEVICE=cuda rehearses the multi-rank GPU path on ONE card
    # (several ranks share cuda:0; gloo stages the collectives through host memory) -- RCCL
    # refuses two ranks on one device, so this is how the bucket/hook/grad-sink path is tested on a
    # one-GPU box.  Production runs leave both unset (RCCL, one GPU per rank).
    backend = os.environ.get("DTG_BACKEND") or backend
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    elif os.environ.get("DTG_GLOO_DEVICE") == "cuda" and torch.cuda.is_available():
        device = torch.device("cuda", local % torch.cuda.device_count())
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")
    # DTG_DDP_FORCE=1: a process group (and DataParallel's bucket hooks, parallel/ddp.py) even at world size
    # 1 -- a one-rank RCCL communicator exercises the collective / stream interplay on a one-GPU box
    force = os.environ.get("DTG_DDP_FORCE") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
            # collectives on a high-priority stream: its own hardware queue, apart from the main and the
            # (high-priority) wgrad side stream's (parallel/overlap.py; 12.3k -> 14.5k img/s one-rank RCCL)
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            kw["pg_options"] = opts
        if timeout_s is None:
            timeout_s = float(os.environ.get("DTG_COLLECTIVE_TIMEOUT", "600"))
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        if world > 1 and watchdog and os.environ.get("DTG_WATCHDOG", "1") == "1":
            Watchdog.start(rank, world)
    return rank, local, world, device


class Watchdog:
    """Heartbeat + peer-liveness thread (see the module docstring).  Uses its own TCP-store client, so it
    never contends with the process group's; ``on_lost(ranks)`` defaults to print + ``os._exit(75)``."""

    _inst = None

    def __init__(self, rank, world, interval=None, timeout=None, on_lost=None):
        self.rank, self.world = rank, world
        self.interval = interval if interval is not None else float(os.environ.get("DTG_HEARTBEAT_S", "5"))
        self.timeout = timeout if timeout is not None else float(os.environ.get("DTG_RANK_TIMEOUT", "60"))
        self.on_lost = on_lost or self._die
        self.lost = []
        self._stop = threading.Event()
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500"))
        self.store = dist.PrefixStore("dtg.hb", dist.TCPStore(host, port, world, False,
                                                              timeout=datetime.timedelta(seconds=60)))
        self.t = threading.Thread(target=self._run, name="dtg-watchdog", daemon=True)

    @classmethod
    def start(cls, rank, world, **kw):
        cls._inst = cls(rank, world, **kw)
        cls._inst.t.start()
        return cls._inst

    def _die(self, ranks):
        print("dtg: rank(s) %s lost -- no heartbeat for %.0f s.  Collectives with them cannot complete (RCCL "
              "communicators cannot shrink): stopping rank %d.  Restart the job to resume from the latest "
              "checkpoint." % (ranks, self.timeout, self.rank), file=sys.stderr, flush=True)
        os._exit(LOST_RANK_EXIT)

    def _run(self):
        seen = {}  # peer -> (last counter value, local time it last changed)
        n = 0
        unreachable_since = None
        while not self._stop.is_set():
            n += 1
            now = time.monotonic()
            try:
                self.store.set(str(self.rank), str(n))
                lost = []
                for r in range(self.world):
                    if r == self.rank or self.store.check(["done.%d" % r]):
                        continue  # finished peers are not lost
                    v = self.store.get(str(r)) if self.store.check([str(r)]) else b""
                    last = seen.get(r)
                    if last is None or last[0] != v:
                        seen[r] = (v, now)
                    elif now - last[1] > self.timeout:
                        lost.append(r)
                unreachable_since = None
            except Exception:
                # the store lives in rank 0's process: unreachable for a whole timeout means rank 0 is gone
                # (shorter outages, e.g. rank 0 exiting at the end of a run while we shut down, are no news)
                unreachable_since = unreachable_since or now
                lost = [0] if now - unreachable_since > self.timeout and self.rank != 0 else []
            if lost and not self._stop.is_set():
                self.lost = lost
                self.on_lost(lost)
                return
            self._stop.wait(self.interval)

    def stop(self):
        self._stop.set()
        try:
            self.store.set("done.%d" % self.rank, "1")
        except Exception:
            pass


def stop_watchdog():
    """Stop this rank's fail-stop watchdog, if one runs (it also marks the rank finished for the peers'
    watchdogs, so a job whose ranks all call this never fail-stops on a lost peer)."""
    if Watchdog._inst is not None:
        Watchdog._inst.stop()
        Watchdog._inst = None


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x: float, device):
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown():
    stop_watchdog()
    if dist.is_initialized():
        dist.destroy_process_group()
