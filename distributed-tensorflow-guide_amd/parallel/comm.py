"""Process-group bootstrap: one process per GPU, RCCL ("nccl" backend on ROCm) over xGMI, or gloo
on CPU.  Ranks come from the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*)
or from a :class:`dtg.ClusterSpec` (job "worker", task_index = rank).
"""
import datetime
import os

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")), int(
        os.environ.get("WORLD_SIZE", "1"))


def init(backend=None, timeout_s=600):
    """Initialise the default process group from the environment (no-op for world_size 1).

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
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, local, world, device


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
    if dist.is_initialized():
        dist.destroy_process_group()
