"""Failure handling of the all-reduce data-parallel path ("sync all-reduce mode: fail-stop
with a clear error and resume from the checkpoint"), on gloo CPU ranks:

* a rank that stops heartbeating (SIGSTOP: alive sockets, no progress -- what a hung or vanished GPU rank
  looks like to its peers) is named by every survivor's watchdog, which exits with status 75 instead of
  waiting out the collective timeout;
* a training job whose rank is killed mid-run fails; restarted, it resumes from the chief's last
  checkpoint and finishes at the absolute last step (examples/ResNet50/resnet50_train.py);
* checkpoints written before the slot-layout marker (channels_last slots in physical order) restore
  converted.
"""
import os
import signal
import subprocess
import sys
import time

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    e = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DTG_FAULT"):
        e.pop(k, None)
    e.update(kw)
    return e


_STALL = r'''
import os, signal, sys, time
sys.path.insert(0, sys.argv[1])
import torch, torch.distributed as dist
import dtg
from dtg.parallel import comm
rank, _, world, _ = comm.init("gloo")
if rank == 1:
    print("rank 1 stopping", flush=True)
    os.kill(os.getpid(), signal.SIGSTOP)
time.sleep(0.5)
t = torch.ones(4)
dist.all_reduce(t)   # never completes: rank 1 is stopped
print("unreachable", flush=True)
'''


def test_watchdog_names_a_silent_rank(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    script = tmp_path / "stall.py"
    script.write_text(_STALL)
    procs = []
    for r in range(2):
        e = _env(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                 DTG_RANK_TIMEOUT="3", DTG_HEARTBEAT_S="0.5")
        procs.append(subprocess.Popen([sys.executable, str(script), ROOT], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    t0 = time.time()
    try:
        out, err = procs[0].communicate(timeout=60)
    finally:
        procs[1].kill()
        procs[1].wait()
    assert procs[0].returncode == 75, (out, err)
    assert "rank(s) [1] lost" in err, err
    assert time.time() - t0 < 45  # well before the 600 s collective timeout


def test_killed_rank_then_resume_from_checkpoint(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    ck = str(tmp_path / "ck")
    script = os.path.join(ROOT, "examples", "ResNet50", "resnet50_train.py")

    def launch(**env):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
               "127.0.0.1", "--master-port", str(free_ports(1)[0]), script, "--tiny", "--batch", "4", "--steps", "6",
               "--save_every", "2", "--ckpt_dir", ck]
        return subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_env(**env))

    r1 = launch(DTG_FAULT="kill_rank_at_step:1@4")
    assert r1.returncode != 0, r1.stdout + r1.stderr[-2000:]
    assert "killing rank 1 at step 4" in r1.stderr
    import dtg
    first = dtg.train.latest_checkpoint(ck)
    assert first.endswith("model.ckpt-2") or first.endswith("model.ckpt-3"), first
    r2 = launch()
    assert r2.returncode == 0, r2.stdout + r2.stderr[-3000:]
    assert "resumed from" in r2.stdout and "done at global step 6" in r2.stdout
    rd = dtg.train.NewCheckpointReader(dtg.train.latest_checkpoint(ck))
    assert int(rd.get_tensor("global_step")) == 6 and int(rd.get_tensor("optimizer/step")) >= 4


def test_restore_slot_layouts(tmp_path):
    """Marked logical, UNMARKED logical (every save_flat between f74dff1 and the marker) and -- opt-in only --
    legacy physical [K,R,S,C] slots all restore to the same momentum."""
    import dtg  # noqa: F401
    from dtg.models.layers import Conv2d
    from dtg.optim import FusedSGD
    from dtg.parallel import FlatParams
    from dtg.train import restore_flat, save_flat
    from dtg.train.saver import read_tensors, write_tensors

    def build():
        torch.manual_seed(0)
        m = torch.nn.Sequential(Conv2d(4, 8, 3))
        return m, FlatParams(m, compute_dtype=torch.float32)

    m, flat = build()
    opt = FusedSGD(flat, lr=0.1, momentum=0.9)
    mom = flat.groups["compute"].state_buffer("momentum")
    mom.copy_(torch.arange(mom.numel(), dtype=torch.float32))  # physical order = flat order
    p = save_flat(flat, str(tmp_path / "m"), global_step=1, optimizer=opt)
    vals = read_tensors(p)
    logical = torch.from_numpy(vals["0.weight/momentum"]).clone()
    # forge a legacy checkpoint: no marker, slot in physical [K,R,S,C] order
    vals.pop("dtg/slot_layout")
    w = m[0].weight
    write_tensors(str(tmp_path / "unmarked-1"), list(vals.items()))
    vals["0.weight/momentum"] = logical.permute(0, 2, 3, 1).contiguous().numpy()
    write_tensors(str(tmp_path / "legacy-1"), list(vals.items()))
    for pref, legacy in ((p, None), (str(tmp_path / "unmarked-1"), None), (str(tmp_path / "legacy-1"), True)):
        m2, flat2 = build()
        opt2 = FusedSGD(flat2, lr=0.1, momentum=0.9)
        assert restore_flat(flat2, pref, optimizer=opt2, legacy_slot_layout=legacy) == 1
        got = flat2.groups["compute"].state["momentum"]
        assert torch.equal(got[:w.numel()], mom[:w.numel()]), pref
    # the default no longer scrambles an unmarked checkpoint: read as legacy it WOULD differ
    m2, flat2 = build()
    opt2 = FusedSGD(flat2, lr=0.1, momentum=0.9)
    restore_flat(flat2, str(tmp_path / "unmarked-1"), optimizer=opt2, legacy_slot_layout=True)
    assert not torch.equal(flat2.groups["compute"].state["momentum"][:w.numel()], mom[:w.numel()])
    with pytest.raises(ValueError):
        restore_flat(flat2, p, optimizer=opt2, legacy_slot_layout=True)
