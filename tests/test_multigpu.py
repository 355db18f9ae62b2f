"""Multi-rank correctness of the distributed paths (tools/multigpu_checks.py: all-reduce vs host sum, DP
equivalence on a fused ResNet and on BERT, async PS update accounting), three ways:

* CPU, 2 gloo ranks (always);
* GPU, 2 gloo ranks sharing one card (host-staged collectives: the GPU kernels + hooks + buckets);
* GPU, one rank per device over RCCL -- switches itself on when the box has >= 2 GPUs (up to 8 ranks),
  skipped on a one-GPU box.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, env, timeout=600, names=()):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "multigpu_checks.py"), *names]
    e = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=e)
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert r.returncode == 0 and rows and rows[0]["ok"], (r.stdout + r.stderr)[-4000:]
    j = rows[0]
    assert j["world"] == n and set(j["checks"]) == (set(names) or {"allreduce", "dp_resnet", "dp_bert", "async_ps"})
    if "async_ps" in j["checks"]:
        assert j["checks"]["async_ps"]["updates"] == 5 * (n - 1)
        assert j["checks"]["async_ps"]["replay_max_rel_err"] < 1e-5  # PS state == replay in its logged order
    return j


def test_multirank_checks_cpu_gloo():
    j = _run(2, {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    assert j["backend"] == "gloo" and j["device"] == "cpu"


def test_async_ps_replay_three_ranks_cpu():
    """1 PS + 2 workers (one with overlapped pulls): the PS parameters equal the replay of both workers'
    pushes in the order the PS applied them."""
    j = _run(3, {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}, names=("async_ps",))
    assert sorted({w for w, _ in j["checks"]["async_ps"]["order_head"]}) == [1, 2]


@pytest.mark.gpu
def test_multirank_checks_one_card_gloo():
    j = _run(2, {"DTG_BACKEND": "gloo", "DTG_GLOO_DEVICE": "cuda"})
    assert j["device"].startswith("cuda")


def _gpus():
    import torch
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.mark.gpu
@pytest.mark.skipif(_gpus() < 2, reason="needs >= 2 GPUs (one RCCL rank per device)")
def test_multirank_checks_rccl():
    n = min(_gpus(), 8)
    j = _run(n, {})
    assert j["backend"] == "nccl"
