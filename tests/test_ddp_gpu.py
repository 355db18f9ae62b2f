"""Two ranks sharing the one GPU (gloo collectives on CUDA tensors) drive the real sync-DP hot path:
fused ResNet bottleneck / fused BERT layer backward writing into flat gradient buffers, bucket
all-reduces launched from inside backward, DataParallel.finish().  The gradient must equal the
sum of the ranks' local gradients and replicas must stay bit-identical (tools/ddp_rehearsal.py).
The RCCL (one GPU per rank) variant of the same path is the round-end 8-GPU bench."""
import os
import subprocess
import sys

import pytest

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
