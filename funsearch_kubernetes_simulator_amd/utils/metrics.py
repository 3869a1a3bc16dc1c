"""Structured JSONL metrics log (generation, island, scores, evals/s, latencies).

The reference only prints; every record here is one JSON object
per line with a wall-clock timestamp, so runs can be plotted or diffed.
"""

from __future__ import annotations

import json
import os
import threading
import time
from typing import Optional


class MetricsLog:
    def __init__(self, path: Optional[str] = None):
        self.path = path
        self._lock = threading.Lock()
        if path:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)

    def write(self, **record) -> None:
        if not self.path:
            return
        record.setdefault("ts", round(time.time(), 3))
        line = json.dumps(record, default=float)
        with self._lock, open(self.path, "a") as fh:
            fh.write(line + "\n")

    @staticmethod
    def read(path: str):
        with open(path) as fh:
            return [json.loads(l) for l in fh if l.strip()]
