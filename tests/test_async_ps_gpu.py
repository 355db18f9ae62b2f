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


@pytest.mark.gpu
def test_async_ps_token_waits_for_device_gradient():
    """The worker's request token leaves only when its gradient exists on the device: an event recorded behind
    an 80 ms device spin (comm_spin stands in for a slow backward; it caps a spin at 100 ms) holds the token back
    80 ms, while the host that submitted it returned at once (parallel/async_ps.py::_Announcer, _ready_event)."""
    import time

    import torch
    from dtg.ops import lib
    from dtg.parallel.async_ps import _Announcer, _ready_event

    sent = []

    class Ctl:
        def request(self, rank, kind):
            torch.cuda.current_stream()  # (touches nothing on the device)
            sent.append((rank, kind, time.perf_counter()))

    g = torch.zeros(1 << 20, device="cuda", dtype=torch.bfloat16)
    torch.cuda.synchronize()
    a = _Announcer(Ctl())
    t0 = time.perf_counter()
    lib().comm_spin(0.08, 1, 0)  # the "backward" producing g is still running ...
    g.add_(1.0)
    a.submit(3, 1, _ready_event([g]))
    t_submit = time.perf_counter() - t0
    a.close()
    assert t_submit < 0.05, t_submit
    assert sent and sent[0][:2] == (3, 1)
    assert sent[0][2] - t0 >= 0.075, sent[0][2] - t0
    assert g.float().mean().item() == 1.0


@pytest.mark.gpu
def test_async_ps_slow_worker_one_card():
    """1 PS + 3 workers on one card (gloo, device tensors staged through the host), worker 3's gradients
    delayed by a device spin before each push: the fast workers take proportionally more updates."""
    import json
    env = dict(os.environ, DTG_BACKEND="gloo", DTG_GLOO_DEVICE="cuda", DTG_APS_TEST_SLOW="3:0.1")
    r = subprocess.run(["python", os.path.join(ROOT, "tools", "async_ps_slow_worker.py"), "--workers", "3",
                        "--seconds", "6"], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    pw = {int(k): v for k, v in rows[-1]["per_worker"].items()}
    assert rows[-1]["lost"] == [] and pw[3] >= 1, pw
    assert min(pw[1], pw[2]) >= 3 * pw[3], pw
