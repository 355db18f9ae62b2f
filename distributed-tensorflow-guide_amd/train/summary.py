"""Minimal TF event-file writer: ``events.out.tfevents.<time>.<host>`` holding
TFRecord-framed ``Event`` protos (file_version record, then scalar summaries), readable by
TensorBoard.  Protobuf is hand-encoded; record CRCs are masked CRC32C from the native runtime.
"""
import os
import socket
import struct
import threading
import time


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _field_bytes(num, payload):
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def _field_double(num, v):
    return _varint((num << 3) | 1) + struct.pack("<d", v)


def _field_float(num, v):
    return _varint((num << 3) | 5) + struct.pack("<f", v)


def _field_int(num, v):
    return _varint((num << 3) | 0) + _varint(v & ((1 << 64) - 1))


def encode_event(wall_time, step=None, file_version=None, scalars=None):
    b = _field_double(1, wall_time)
    if step is not None:
        b += _field_int(2, int(step))
    if file_version is not None:
        b += _field_bytes(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, val in scalars:
            summ += _field_bytes(1, _field_bytes(1, tag.encode()) + _field_float(2, float(val)))
        b += _field_bytes(5, summ)
    return b


def _masked_crc(data):
    from .. import _runtime
    return _runtime.crc_mask(_runtime.crc32c(data))


def frame_record(data):
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", _masked_crc(hdr)) + data + struct.pack("<I", _masked_crc(data))


def read_records(path):
    out = []
    with open(path, "rb") as f:
        while True:
            hdr = f.read(12)
            if len(hdr) < 12:
                break
            (n,) = struct.unpack("<Q", hdr[:8])
            data = f.read(n)
            f.read(4)
            out.append(data)
    return out


class FileWriter:
    _cache = {}
    _lock = threading.Lock()

    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, "events.out.tfevents.%d.%s" % (int(time.time()), socket.gethostname()))
        self._f = open(self.path, "ab")
        self._f.write(frame_record(encode_event(time.time(), file_version="brain.Event:2")))
        self._f.flush()

    @classmethod
    def for_dir(cls, logdir):
        with cls._lock:
            w = cls._cache.get(os.path.abspath(logdir))
            if w is None:
                w = cls(logdir)
                cls._cache[os.path.abspath(logdir)] = w
            return w

    def add_scalar(self, tag, value, step):
        self._f.write(frame_record(encode_event(time.time(), step, scalars=[(tag, value)])))
        self._f.flush()

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()
