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
