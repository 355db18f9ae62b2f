"""JSONL metrics: one JSON object per line, tagged with rank and wall time.

    log = MetricsLogger("logdir/metrics.jsonl", rank=rank)
    log.log(step=100, loss=2.31, images_per_sec=13950.0)

Appends (several processes may share one file: each record is a single ``write`` of one line,
which POSIX appends atomically for the sizes involved).  ``path=None`` keeps records in memory only
(``records``), which the tests and the examples' summaries read back.
"""
import json
import os
import time


class MetricsLogger:
    def __init__(self, path=None, rank=None, **static):
        self.path = path
        self.rank = rank
        self.static = static
        self.records = []
        if path:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)

    def log(self, **fields):
        rec = {"time": time.time()}
        if self.rank is not None:
            rec["rank"] = self.rank
        rec.update(self.static)
        rec.update(fields)
        self.records.append(rec)
        if self.path:
            line = json.dumps(rec, default=float) + "\n"
            with open(self.path, "a") as f:
                f.write(line)
        return rec

    @staticmethod
    def read(path):
        with open(path) as f:
            return [json.loads(line) for line in f if line.strip()]
