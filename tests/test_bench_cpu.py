"""bench.py's launch contract on the CPU (gloo): ``python bench.py --gpus N`` starts N ranks by itself and
reports the whole job, and a launcher whose world size disagrees with ``--gpus`` is a hard error."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--model", "mnist", "--batch", "4", "--steps", "2", "--warmup", "1"]


def _env(**kw):
    e = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "DTG_DDP_FORCE"):
        e.pop(k, None)
    e.update(kw)
    return e


def _json_line(out):
    rows = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    assert len(rows) == 1, out  # rank 0 only
    return rows[0]


def test_plain_gpus2_self_launches_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL, cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    j = _json_line(r.stdout)
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2", j
    assert j["config"]["global_batch"] == 8 and j["steps"] == 2 and j["warmup"] == 1
    assert j["value"] > 0 and j["ms_per_step"] > 0


def test_world_size_mismatch_is_an_error():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "4"] + SMALL
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]
    assert not any(x.startswith("{") for x in r.stdout.splitlines())


def test_async_ps_mode_reports_whole_node_rate():
    """bench.py --mode async_ps (BASELINE config 4): rank 0 is the PS, the other ranks are workers; the PS
    prints one JSON line of whole-node images/sec over the updates applied after every worker's warm-up."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--mode", "async_ps",
                        "--batch", "2", "--image", "32", "--steps", "3", "--warmup", "1"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    j = _json_line(r.stdout)
    assert j["n_gpus"] == 3 and j["config"]["parallelism"] == "ps1+w2" and j["value"] > 0
    assert j["per_worker"] == {"1": 4, "2": 4} and j["lost_workers"] == []
    assert 1 <= j["updates_timed"] <= 8


def test_async_ps_mode_downpour_window_with_local_optimizer():
    """bench.py --mode async_ps in its DOWNPOUR form (--window 3, local Adagrad inside the window, Adagrad on the
    PS; /root/reference/DOWNPOUR/DOWNPOUR.py:54-102): every worker pushes once per window and the JSON line names
    the rule."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mode", "async_ps",
                        "--batch", "2", "--image", "32", "--steps", "3", "--warmup", "3", "--window", "3",
                        "--local_opt", "adagrad", "--ps_opt", "adagrad", "--lr", "0.01"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    j = _json_line(r.stdout)
    c = j["config"]
    assert c["window"] == 3 and c["local_opt"] == "adagrad" and c["optimizer"].startswith("adagrad"), c
    assert j["per_worker"] == {"1": 2} and j["lost_workers"] == []


def test_driver_launch_form_eight_ranks_resnet():
    """The round-end scaling run's exact launch form (torch.distributed.run, 8 ranks on 127.0.0.1, bench.py
    --gpus 8) with the headline model, shrunk to 32x32 images and batch 2 per rank on gloo: one JSON line
    from rank 0 with the whole-job rate, dp8 and the global batch."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cluster import free_ports
    port = free_ports(1)[0]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "8", "--image", "32",
           "--batch", "2", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=_env())
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    j = _json_line(r.stdout)
    assert j["n_gpus"] == 8 and j["config"]["parallelism"] == "dp8" and j["config"]["global_batch"] == 16, j
    assert j["config"]["model"] == "ResNet-50" and j["scaling"] == "weak" and j["value"] > 0
    p = j["allreduce_probe"]  # the collective alone, after the timed steps: bytes of the whole gradient
    assert p["grad_bytes"] > 25_000_000 * 2 * 0.9 and p["full_busbw_GBps"] > 0 and p["bucket_ms"] > 0, p
    assert p["compute_only_ms_per_step"] > 0 and "exposed_comm_ms_per_step" in p, p
