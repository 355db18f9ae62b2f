"""Unit tests of the native runtime (csrc/ps, csrc/ckpt) and the cluster/placement/flags layer."""
import os
import threading
import time

import numpy as np
import pytest

import dtg
from dtg import _runtime as R


@pytest.fixture
def ps():
    s = R.PSServer("127.0.0.1", 0, 2)
    s.start()
    c = R.PSClient("127.0.0.1", s.port, 10.0)
    yield s, c
    c.close()
    s.stop()


def test_variable_store_ops(ps):
    s, c = ps
    assert c.ping()
    assert c.create("a", np.zeros(3, np.float32))
    assert not c.create("a", np.ones(3, np.float32))  # exists: not overwritten
    c.assign([("a", np.arange(3, dtype=np.float32))])
    np.testing.assert_array_equal(c.read(["a"])[0], [0, 1, 2])
    c.create("gs", np.array(5, np.int64))
    assert int(c.assign_add("gs", np.array(2, np.int64))) == 7
    assert c.is_init(["a", "nope"]) == [True, False]
    names = {n for n, _, _ in c.list()}
    assert names == {"a", "gs"}


def test_apply_sgd_adagrad_momentum_adam(ps):
    s, c = ps
    c.create("w", np.ones(4, np.float32))
    c.create("gs", np.array(0, np.int32))
    g = np.full(4, 0.5, np.float32)
    step, vals = c.apply(R.SGD, [0.1], False, "gs", [("w", g)], True)
    assert step == 1
    np.testing.assert_allclose(vals[0], 1 - 0.05)
    step, vals = c.apply(R.ADAGRAD, [0.1, 0.1], True, "gs", [("w", g)], True)
    acc = 0.1 + 0.25
    np.testing.assert_allclose(vals[0], 0.95 - 0.1 * 0.5 / np.sqrt(acc), rtol=1e-6)
    np.testing.assert_allclose(c.read(["w/Adagrad"])[0], acc, rtol=1e-6)  # TF slot naming
    c.create("m", np.zeros(2, np.float32))
    c.apply(R.MOMENTUM, [1.0, 0.9], False, "", [("m", np.ones(2, np.float32))])
    _, v = c.apply(R.MOMENTUM, [1.0, 0.9], False, "", [("m", np.ones(2, np.float32))], True)
    np.testing.assert_allclose(v[0], -(1 + 1.9))
    c.create("z", np.zeros(1, np.float32))
    _, v = c.apply(R.ADAM, [0.1, 0.9, 0.999, 1e-8, 1], False, "", [("z", np.ones(1, np.float32))], True)
    np.testing.assert_allclose(v[0], -0.1, rtol=1e-4)


def test_hogwild_concurrent_applies_count_every_step(ps):
    s, c = ps
    c.create("w", np.zeros(64, np.float32))
    c.create("gs", np.array(0, np.int64))

    def worker():
        cl = R.PSClient("127.0.0.1", s.port, 10.0)
        for _ in range(200):
            cl.apply(R.SGD, [1.0], False, "gs", [("w", -np.ones(64, np.float32))])
        cl.close()
    ts = [threading.Thread(target=worker) for _ in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert int(c.read(["gs"])[0]) == 800
    w = c.read(["w"])[0]
    assert (w <= 800).all() and (w > 0).all()  # lock-free: updates may be lost, never invented


def test_conditional_accumulator_drops_stale(ps):
    s, c = ps
    c.acc_create("acc", np.zeros(2, np.float32), 3)
    assert not c.acc_apply("acc", 2, np.ones(2, np.float32))  # local_step < global_step -> dropped
    assert c.acc_apply("acc", 3, np.full(2, 2, np.float32))
    assert c.acc_apply("acc", 4, np.full(2, 4, np.float32))
    assert c.acc_num("acc") == (2, 1)
    np.testing.assert_allclose(c.acc_take("acc", 2, 1.0), 3.0)  # mean
    assert c.acc_take("acc", 1, 0.05) is None  # blocks -> timeout


def test_token_queue_blocks_until_enqueue(ps):
    s, c = ps
    got = []

    def deq():
        cl = R.PSClient("127.0.0.1", s.port, 10.0)
        got.append(cl.q_dequeue("q", 5.0))
        cl.close()
    t = threading.Thread(target=deq)
    t.start()
    time.sleep(0.1)
    assert not got
    c.q_enqueue("q", [7, 8])
    t.join()
    assert got == [7] and c.q_size("q") == 1


def test_barrier_and_join(ps):
    s, c = ps
    res = []

    def b():
        cl = R.PSClient("127.0.0.1", s.port, 10.0)
        res.append(cl.barrier("b", 2, 5.0))
        cl.close()
    t = threading.Thread(target=b)
    t.start()
    assert c.barrier("b", 2, 5.0)
    t.join()
    assert res == [True]
    assert not s.join(0.05)
    c.worker_done(0)
    c.worker_done(0)  # idempotent
    assert not s.join(0.05)
    c.worker_done(1)
    assert s.join(1.0)


def test_tensor_bundle_roundtrip_and_format(tmp_path):
    prefix = str(tmp_path / "model.ckpt-7")
    arrays = [("global_step", np.array(7, np.int64)), ("g/Variable", np.array([1.5, -2], np.float32)),
              ("conv1/kernel", np.random.RandomState(0).randn(3, 3, 8, 16).astype(np.float32))]
    dtg.train.saver.write_tensors(prefix, arrays)
    back = dtg.train.saver.read_tensors(prefix)
    for n, a in arrays:
        np.testing.assert_array_equal(back[n], a)
        assert back[n].shape == a.shape
    idx = R.read_index(prefix)
    assert idx["global_step"][0] == 9 and idx["g/Variable"][0] == 1  # TF DataType enums
    # SSTable footer magic + data file size = sum of tensor bytes
    with open(prefix + ".index", "rb") as f:
        raw = f.read()
    assert raw[-8:] == (0xdb4775248b80fb57).to_bytes(8, "little")
    assert os.path.getsize(prefix + ".data-00000-of-00001") == sum(a.nbytes for _, a in arrays)
    # corruption is detected by the masked CRC32C
    with open(prefix + ".data-00000-of-00001", "r+b") as f:
        f.seek(8)
        f.write(b"\xff")
    with pytest.raises(Exception):
        R.read_bundle(prefix, True)


def test_crc32c_known_vector():
    assert R.crc32c(b"123456789") == 0xE3069283  # CRC-32C check value


def test_checkpoint_state_file(tmp_path):
    from dtg.train import saver as S
    d = str(tmp_path)
    S.update_checkpoint_state(d, os.path.join(d, "model.ckpt-3"), [os.path.join(d, "model.ckpt-1"),
                                                                    os.path.join(d, "model.ckpt-3")])
    txt = open(os.path.join(d, "checkpoint")).read()
    assert 'model_checkpoint_path: "model.ckpt-3"' in txt and 'all_model_checkpoint_paths: "model.ckpt-1"' in txt
    st = S.get_checkpoint_state(d)
    assert st.model_checkpoint_path.endswith("model.ckpt-3") and len(st.all_model_checkpoint_paths) == 2


def test_event_file(tmp_path):
    from dtg.train.summary import FileWriter, read_records
    w = FileWriter(str(tmp_path))
    w.add_scalar("global_step/sec", 12.5, 3)
    w.flush()
    recs = read_records(w.path)
    assert len(recs) == 2 and b"brain.Event:2" in recs[0] and b"global_step/sec" in recs[1]


def test_cluster_spec_and_flags():
    spec = dtg.ClusterSpec({"ps": ["localhost:2222"], "worker": ["localhost:2223", "localhost:2224"]})
    assert spec.num_tasks("worker") == 2 and spec.task_address("ps", 0) == "localhost:2222"
    assert spec.as_dict()["worker"][1] == "localhost:2224" and "ps" in spec
    f = dtg.flags.parse(["--job_name", "worker", "--task_index", "1", "--unknown_flag", "x"])
    assert f.job_name == "worker" and f.task_index == 1  # unknown flags ignored (parse_known_args)
    f = dtg.flags.parse([])
    assert f.job_name == "" and f.task_index == 0


def test_device_strings_and_replica_setter():
    from dtg.placement import DeviceSpec, resolve_device
    d = DeviceSpec.from_string("/job:worker/replica:0/task:1/cpu:0")
    assert (d.job, d.replica, d.task, d.device_type, d.device_index) == ("worker", 0, 1, "cpu", 0)
    assert DeviceSpec.from_string("/job:ps/task:0/device:GPU:1").device_type == "gpu"

    class V:
        _is_variable = True

    class O:
        _is_variable = False
    setter = dtg.replica_device_setter(ps_tasks=2, worker_device="/job:worker/task:3")
    got = [resolve_device([setter], V()).to_string() for _ in range(3)]
    assert got == ["/job:ps/task:0", "/job:ps/task:1", "/job:ps/task:0"]  # round robin
    assert resolve_device([setter], O()).to_string() == "/job:worker/task:3"
    assert resolve_device(["/job:worker", "/task:2/gpu:0"], O()).to_string() == "/job:worker/task:2/device:GPU:0"


def test_server_join_returns_when_workers_done():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    spec = {"ps": ["127.0.0.1:%d" % port], "worker": ["127.0.0.1:1", "127.0.0.1:2"]}
    srv = dtg.Server(spec, job_name="ps", task_index=0)
    assert srv.target == "dtg://127.0.0.1:%d" % port
    assert srv.server_def["job_name"] == "ps"
    c = R.PSClient("127.0.0.1", port, 5.0)
    c.worker_done(0)
    c.worker_done(1)
    assert srv.join(timeout=2.0)
    c.close()


def test_malformed_tensor_payloads_are_rejected(ps):
    """A tensor whose byte count disagrees with its shape, or a huge byte count that would wrap the
    reader's bounds check, gets an error status -- no over-read -- and the service stays up."""
    import socket
    import struct
    s, c = ps
    c.acc_create("acc_m", np.zeros(4, np.float32), 0)

    def request(op, body):
        k = socket.create_connection(("127.0.0.1", s.port), timeout=10)
        try:
            k.sendall(struct.pack("<IHHQ", 0x50475444, op, 0, len(body)) + body)
            hdr = b""
            while len(hdr) < 16:
                chunk = k.recv(16 - len(hdr))
                assert chunk, "server closed the connection"
                hdr += chunk
            _, status, _ = struct.unpack("<IiQ", hdr)
            return status
        finally:
            k.close()

    name = b"acc_m"
    head = struct.pack("<I", len(name)) + name + struct.pack("<q", 0)
    short = head + struct.pack("<BBq", 1, 1, 4) + struct.pack("<Q", 4) + b"\0" * 4   # 4 floats, 4 bytes
    assert request(9, short) != 0
    wrap = head + struct.pack("<BBq", 1, 1, 4) + struct.pack("<Q", (1 << 64) - 8)    # nb wraps off + nb
    assert request(9, wrap) != 0
    good = head + struct.pack("<BBq", 1, 1, 4) + struct.pack("<Q", 16) + np.ones(4, np.float32).tobytes()
    assert request(9, good) == 0
    assert c.acc_num("acc_m")[0] == 1
