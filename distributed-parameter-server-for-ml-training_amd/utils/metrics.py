"""METRICS_JSON observability contract + phase timers.

Every process ends by printing exactly one ``METRICS_JSON: {...}`` line whose record type and
field names match the reference (reference: server.py:347-368 SERVER_FINAL_METRICS,
worker.py:419-436 WORKER_FINAL_METRICS; parsed by scripts/parse_cloudwatch_logs.py:100 with
the regex ``METRICS_JSON:\\s*(\\{.*\\})``). Additional fields (images_per_second, gpus,
phase_ms, staleness_histogram, rejected_pushes, bytes_pushed, bytes_fetched) are appended,
never renamed. Records are also appended to ``<log_dir>/rank<k>.jsonl`` when a log dir is set.
"""
from __future__ import annotations

import json
import os
import re
import time
from collections import defaultdict

METRICS_RE = re.compile(r"METRICS_JSON:\s*(\{.*\})")


def emit(record: dict, log_dir: str = "", rank: int | None = None, stream=None) -> str:
    line = "METRICS_JSON: " + json.dumps(record)
    print(line, file=stream, flush=True)
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
        name = f"rank{rank}.jsonl" if rank is not None else "metrics.jsonl"
        with open(os.path.join(log_dir, name), "a") as f:
            f.write(json.dumps(record) + "\n")
    return line


def parse_lines(lines) -> list[dict]:
    out = []
    for ln in lines:
        m = METRICS_RE.search(ln)
        if m:
            try:
                out.append(json.loads(m.group(1)))
            except json.JSONDecodeError:
                continue
    return out


class PhaseTimer:
    """Accumulates wall time per named phase; GPU phases are bracketed by HIP events when a
    device is in use (timed=True), so nothing forces a host sync inside the hot loop."""

    def __init__(self, device=None):
        self.device = device
        self.wall = defaultdict(float)
        self.count = defaultdict(int)
        self._events = defaultdict(list)

    def add(self, name, seconds):
        self.wall[name] += seconds
        self.count[name] += 1

    def span(self, name):
        return _Span(self, name)

    def gpu_begin(self, name):
        import torch

        if self.device is None or not torch.cuda.is_available():
            return None
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        return (name, e0)

    def gpu_end(self, token):
        import torch

        if token is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self._events[token[0]].append((token[1], e1))

    def flush(self):
        """Resolve pending GPU events (call outside the timed region)."""
        for name, pairs in self._events.items():
            for e0, e1 in pairs:
                e1.synchronize()
                self.add(name, e0.elapsed_time(e1) / 1e3)
        self._events.clear()

    def summary_ms(self) -> dict:
        self.flush()
        return {k: round(1e3 * v / max(1, self.count[k]), 4) for k, v in self.wall.items()}


class _Span:
    def __init__(self, t: PhaseTimer, name: str):
        self.t, self.name = t, name

    def __enter__(self):
        from . import trace

        trace.push(self.name)  # roctx range when PSX_ROCTX=1 (utils/trace.py)
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        from . import trace

        self.t.add(self.name, time.perf_counter() - self.t0)
        trace.pop()
        return False


def aggregate_worker_metrics(worker_metrics: list[dict]) -> dict | None:
    """Same aggregate schema as the reference parser (parse_cloudwatch_logs.py:125-177)."""
    if not worker_metrics:
        return None
    agg = {
        "num_workers": len(worker_metrics),
        "total_training_time_seconds": max(w["total_training_time_seconds"] for w in worker_metrics),
        "average_epoch_time_seconds": sum(w["average_epoch_time_seconds"] for w in worker_metrics)
        / len(worker_metrics),
        "final_test_accuracy_percent": sum(w["final_test_accuracy_percent"] for w in worker_metrics)
        / len(worker_metrics),
        "total_local_steps": sum(w["local_steps_completed"] for w in worker_metrics),
        "per_worker_metrics": worker_metrics,
    }
    max_epochs = max(len(w["epoch_times_seconds"]) for w in worker_metrics)
    by_epoch = []
    acc_by_epoch = []
    for e in range(max_epochs):
        ts = [w["epoch_times_seconds"][e] for w in worker_metrics if e < len(w["epoch_times_seconds"])]
        if ts:
            by_epoch.append({"epoch": e + 1, "max_time": max(ts), "avg_time": sum(ts) / len(ts), "min_time": min(ts)})
        accs = [w["all_accuracies_percent"][e] for w in worker_metrics if e < len(w["all_accuracies_percent"])]
        if accs:
            acc_by_epoch.append({"epoch": e + 1, "avg_accuracy": sum(accs) / len(accs), "max_accuracy": max(accs),
                                 "min_accuracy": min(accs)})
    agg["epoch_times_by_epoch"] = by_epoch
    agg["accuracy_by_epoch"] = acc_by_epoch
    return agg
