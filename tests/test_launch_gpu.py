"""Launch failures surface as Python errors, and the emulated collective behaves as specified.

* DTG_LAUNCH_CHECK (csrc/include/dtg/common.h) after every kernel launch: an impossible launch (dynamic LDS
  above the 160 KB per-CU limit, an empty grid) raises RuntimeError instead of leaving an output unwritten.
* comm_spin (csrc/kernels/comm_emu.hip): holds its workgroups for the requested time, measured with events.
* DTG_COMM_EMULATE through DataParallel on a one-rank RCCL group (DTG_DDP_FORCE=1): bench.py reports the
  compute-only and exposed-communication split (subprocess, so the env knobs apply at import).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from dtg.ops._native import lib

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_impossible_launch_raises():
    L = lib()
    with pytest.raises(RuntimeError, match="kernel launch"):
        L.launch_probe(1, 512 * 1024)  # LDS over the per-workgroup limit
    with pytest.raises(RuntimeError, match="kernel launch"):
        L.launch_probe(0, 0)  # empty grid
    L.launch_probe(4, 1024)  # a valid launch still works afterwards (no sticky error left behind)
    torch.cuda.synchronize()


def test_comm_spin_duration():
    L = lib()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    L.comm_spin(1e-3, 32, 0)  # warm
    s.record()
    L.comm_spin(3e-3, 32, 0)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e)
    assert 2.8 <= ms <= 6.0, ms
    s.record()
    L.comm_spin(10.0, 32, 0)  # capped at 100 ms on the host
    e.record()
    torch.cuda.synchronize()
    assert s.elapsed_time(e) <= 150.0


def test_bench_emulated_collective_reports_exposed_comm():
    env = dict(os.environ, DTG_DDP_FORCE="1", DTG_COMM_EMULATE="100", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29561")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "64", "--steps", "3",
                        "--warmup", "2"], env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    p = line["allreduce_probe"]
    assert p["comm_emulate"]["busbw_GBps"] == 100.0 and p["comm_emulate"]["ranks"] == 8
    assert p["compute_only_ms_per_step"] > 0
    assert "exposed_comm_ms_per_step" in p
