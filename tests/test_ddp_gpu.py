"""Two ranks sharing the one GPU (gloo collectives on CUDA tensors) drive the real sync-DP hot path:
fused ResNet bottleneck / fused BERT layer backward writing into flat gradient buffers, bucket
all-reduces launched from inside backward, DataParallel.finish().  The gradient must equal the
sum of the ranks' local gradients and replicas must stay bit-identical (tools/ddp_rehearsal.py).
The RCCL (one GPU per rank) variant of the same path is the round-end 8-GPU bench."""
import os
import subprocess
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("model,port", [("resnet", 29541), ("bert", 29542)])
def test_ddp_two_ranks_on_one_gpu(model, port):
    env = dict(os.environ, DTG_BACKEND="gloo", DTG_GLOO_DEVICE="cuda")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(ROOT, "tools", "ddp_rehearsal.py"), "--model", model]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ddp rehearsal ok" in r.stdout


@pytest.mark.parametrize("model,extra", [("resnet", ["--batch", "8", "--image", "128"]), ("bert", [])])
def test_ddp_emulated_collective_data_mode(model, extra):
    """One rank on an RCCL group (DTG_DDP_FORCE=1) with the emulated 8-rank collective in its pessimistic form
    (busy-polling, ring HBM traffic, data): every bucket comes back as 8 x itself, so the flat gradient must be
    8 x the plain one-rank gradient -- a bucket whose collective read a gradient before the side-stream weight
    gradient or main-stream BN-parameter gradient landed would break it (ResNet fused path at b8 / 128^2 reaches
    the fused dx + weight-gradient passes; BERT: the fused layers)."""
    from _cluster import free_ports
    port = free_ports(1)[0]
    env = dict(os.environ, DTG_DDP_FORCE="1", DTG_COMM_EMULATE="100,8,32,10,busy+traffic+data",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "tools", "ddp_rehearsal.py"), "--model", model, *extra]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ddp rehearsal ok" in r.stdout and "emulated_ranks=8 (data mode)" in r.stdout, r.stdout[-2000:]
