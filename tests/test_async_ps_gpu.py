"""ResNet-50 async parameter server (BASELINE.json config 4) on the GPU: 1 PS + 2 workers sharing
one card, point-to-point over gloo with host staging (tools/async_ps_rehearsal.sh).  On a node the
same code runs over RCCL, one GPU per process; this covers the HIP model + fused PS apply +
push/pull protocol on real hardware (parallel/async_ps.py)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_async_ps_resnet50_one_card():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "async_ps_rehearsal.sh"), "2", "--steps", "6",
                        "--batch", "16"], capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    m = re.search(r"\[ps\] (\d+) updates .* per worker \{1: (\d+), 2: (\d+)\}", out)
    assert m, out[-3000:]
    assert (int(m.group(1)), int(m.group(2)), int(m.group(3))) == (12, 6, 6)


@pytest.mark.gpu
def test_bench_async_ps_mode_one_card():
    """bench.py --mode async_ps on one card (PS + 1 worker sharing cuda:0, gloo point-to-point staged
    through the host): the whole-node JSON line, every timed update accounted for."""
    import json
    env = dict(os.environ, DTG_BACKEND="gloo", DTG_GLOO_DEVICE="cuda")
    r = subprocess.run(["python", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mode", "async_ps", "--batch", "32",
                        "--steps", "4", "--warmup", "2"], capture_output=True, text=True, timeout=300, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(rows) == 1
    j = rows[0]
    assert j["n_gpus"] == 2 and j["dtype"] == "bf16" and j["per_worker"] == {"1": 6} and j["value"] > 0
