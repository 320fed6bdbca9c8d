"""Experiment result pipeline: METRICS_JSON logs -> aggregate JSON -> figures + summary table.

MI355X-native counterpart of the reference's CloudWatch parser and visualiser (reference:
scripts/parse_cloudwatch_logs.py:30-217 and scripts/visualize_results.py:28-296). The
reference pulls ``METRICS_JSON:`` lines out of CloudWatch log groups with the AWS CLI; here the
sources are local: captured stdout/stderr of a run (any file containing ``METRICS_JSON:``
lines) or the per-rank ``rank<k>.jsonl`` files a run writes with ``--log-dir``. The aggregate
schema is the reference's (experiment_name, timestamp, server_metrics,
worker_metrics_aggregated{...}, raw_worker_metrics) so existing result files load unchanged.

The visualiser also works when ``server_metrics`` is missing (null in every result file the
reference checked in): mode / worker count then come from the worker records or the file name
(``sync_4workers.json``), and it adds img/s panels and a bench-JSON scaling plot.
"""
from __future__ import annotations

import json
import os
import re
from collections import defaultdict
from datetime import datetime
from pathlib import Path

from .metrics import METRICS_RE, aggregate_worker_metrics


# ---------------------------------------------------------------------------- parsing
def _records_from_file(path: Path) -> list[dict]:
    out = []
    with open(path, errors="replace") as f:
        for ln in f:
            m = METRICS_RE.search(ln)
            if m:
                try:
                    out.append(json.loads(m.group(1)))
                except json.JSONDecodeError:
                    continue
                continue
            s = ln.strip()
            if path.suffix == ".jsonl" and s.startswith("{"):
                try:
                    out.append(json.loads(s))
                except json.JSONDecodeError:
                    continue
    return out


def collect_records(sources) -> list[dict]:
    recs = []
    for src in sources:
        p = Path(src)
        files = sorted(p.rglob("*")) if p.is_dir() else [p]
        for f in files:
            if f.is_file() and f.suffix in (".log", ".txt", ".jsonl", ".out", ".err", ""):
                recs.extend(_records_from_file(f))
    return recs


def parse_experiment(sources, experiment_name: str, verbose: bool = True) -> dict:
    """Reference parse_experiment (parse_cloudwatch_logs.py:179-217) over local files."""
    recs = collect_records(sources)
    servers = [r for r in recs if r.get("type") == "SERVER_FINAL_METRICS"]
    workers = [r for r in recs if r.get("type") == "WORKER_FINAL_METRICS"]
    # one record per worker id (a re-emitted record of the same worker replaces the older one)
    by_id = {}
    for w in workers:
        by_id[w.get("worker_id")] = w
    workers = [by_id[k] for k in sorted(by_id, key=lambda x: (x is None, x))]
    res = {
        "experiment_name": experiment_name,
        "timestamp": datetime.now().isoformat(),
        "server_metrics": servers[-1] if servers else None,
        "worker_metrics_aggregated": aggregate_worker_metrics(workers),
        "raw_worker_metrics": workers,
    }
    if verbose:
        sm, agg = res["server_metrics"], res["worker_metrics_aggregated"]
        print(f"\nParsing experiment: {experiment_name}\n{'=' * 60}")
        print(f"  {len(servers)} server record(s), {len(workers)} worker record(s)")
        if sm:
            print(f"  Mode: {sm['mode']}  Workers: {sm['total_workers']}  "
                  f"Training time: {sm['total_training_time_seconds']:.1f}s")
        if agg:
            print(f"  Avg epoch time: {agg['average_epoch_time_seconds']:.1f}s  "
                  f"Final accuracy: {agg['final_test_accuracy_percent']:.2f}%")
    return res


# ---------------------------------------------------------------------------- visualisation
_NAME_RE = re.compile(r"(sync|async)[_-]?(\d+)[_-]?workers?", re.I)


class ExperimentVisualizer:
    def __init__(self, output_dir="./plots"):
        self.output_dir = Path(output_dir)
        self.output_dir.mkdir(parents=True, exist_ok=True)
        self.experiments = []

    def load_experiment(self, filepath):
        with open(filepath) as f:
            data = json.load(f)
        exp = {"name": data.get("experiment_name", Path(filepath).stem), "filepath": str(filepath), "data": data}
        sm = data.get("server_metrics")
        agg = data.get("worker_metrics_aggregated")
        raw = data.get("raw_worker_metrics") or []
        if sm:
            exp["mode"] = sm.get("mode")
            exp["num_workers"] = sm.get("total_workers")
            exp["training_time"] = sm.get("total_training_time_seconds")
            if sm.get("images_per_second"):
                exp["images_per_second"] = sm["images_per_second"]
        m = _NAME_RE.search(exp["name"]) or _NAME_RE.search(Path(filepath).stem)
        if "mode" not in exp and m:
            exp["mode"] = m.group(1).lower()
        if "num_workers" not in exp:
            if m:
                exp["num_workers"] = int(m.group(2))
            elif raw and raw[0].get("total_workers"):
                exp["num_workers"] = raw[0]["total_workers"]
        if agg:
            exp.setdefault("training_time", agg.get("total_training_time_seconds"))
            exp["avg_epoch_time"] = agg.get("average_epoch_time_seconds")
            exp["final_accuracy"] = agg.get("final_test_accuracy_percent")
            exp["epoch_times"] = agg.get("epoch_times_by_epoch", [])
            exp["accuracy_by_epoch"] = agg.get("accuracy_by_epoch", [])
            ips = [w.get("images_per_second") for w in agg.get("per_worker_metrics", []) if w.get("images_per_second")]
            if ips and "images_per_second" not in exp:
                exp["images_per_second"] = sum(ips)
        self.experiments.append(exp)
        print(f"Loaded: {exp['name']} ({exp.get('mode', 'unknown')}, {exp.get('num_workers', '?')} workers)")
        return exp

    def load_experiments_from_directory(self, directory):
        for fp in sorted(Path(directory).glob("*.json")):
            try:
                self.load_experiment(fp)
            except Exception as e:  # keep going, like the reference
                print(f"Warning: Could not load {fp}: {e}")
        return self.experiments

    @staticmethod
    def _plt():
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        return plt

    def plot_sync_vs_async_comparison(self, worker_count=None):
        plt = self._plt()
        by_w = defaultdict(dict)
        for e in self.experiments:
            if e.get("mode") and e.get("num_workers"):
                by_w[e["num_workers"]][e["mode"]] = e
        written = []
        for nw, modes in sorted(by_w.items()):
            if worker_count and nw != worker_count:
                continue
            if "sync" not in modes or "async" not in modes:
                print(f"Warning: Missing sync or async data for {nw} workers, skipping...")
                continue
            s, a = modes["sync"], modes["async"]
            fig, ax = plt.subplots(2, 2, figsize=(14, 10))
            fig.suptitle(f"Sync vs Async Comparison ({nw} Workers)", fontsize=16, fontweight="bold")
            self._bars(ax[0, 0], [s.get("training_time"), a.get("training_time")], "Total Training Time", "s")
            self._bars(ax[0, 1], [s.get("avg_epoch_time"), a.get("avg_epoch_time")], "Average Epoch Time", "s")
            for e, lab in ((s, "Sync"), (a, "Async")):
                et = e.get("epoch_times") or []
                if et:
                    ax[1, 0].plot([x["epoch"] for x in et], [x["avg_time"] for x in et], marker="o", label=lab)
            ax[1, 0].set(title="Epoch Duration Over Time", xlabel="Epoch", ylabel="seconds")
            ax[1, 0].legend()
            self._bars(ax[1, 1], [s.get("final_accuracy"), a.get("final_accuracy")], "Final Test Accuracy", "%")
            out = self.output_dir / f"sync_vs_async_{nw}workers.png"
            fig.tight_layout()
            fig.savefig(out, dpi=150, bbox_inches="tight")
            plt.close(fig)
            written.append(out)
        return written

    @staticmethod
    def _bars(ax, vals, title, unit):
        vals = [v if v is not None else 0.0 for v in vals]
        bars = ax.bar(["Sync", "Async"], vals, color=["#3498db", "#e74c3c"], alpha=0.7, edgecolor="black")
        for b, v in zip(bars, vals):
            ax.text(b.get_x() + b.get_width() / 2, b.get_height(), f"{v:.1f}{unit}", ha="center", va="bottom")
        ax.set_title(title, fontweight="bold")
        ax.grid(axis="y", alpha=0.3)

    def plot_scaling_analysis(self):
        plt = self._plt()
        fig, ax = plt.subplots(2, 2, figsize=(14, 10))
        fig.suptitle("Scaling Analysis: Performance vs Worker Count", fontsize=16, fontweight="bold")
        any_data = False
        for mode, color in (("sync", "#3498db"), ("async", "#e74c3c")):
            es = sorted((e for e in self.experiments if e.get("mode") == mode and e.get("num_workers")),
                        key=lambda e: e["num_workers"])
            if not es:
                continue
            any_data = True
            w = [e["num_workers"] for e in es]
            for a, key, title in ((ax[0, 0], "training_time", "Total Training Time vs Workers"),
                                  (ax[0, 1], "avg_epoch_time", "Epoch Time vs Workers"),
                                  (ax[1, 0], "final_accuracy", "Final Accuracy vs Workers")):
                ys = [e.get(key) for e in es]
                pts = [(x, y) for x, y in zip(w, ys) if y is not None]
                if pts:
                    a.plot(*zip(*pts), marker="o", color=color, label=mode)
                a.set_title(title, fontweight="bold")
                a.set_xscale("log", base=2)
            base = next((e for e in es if e["num_workers"] == 1), None)
            if base and base.get("training_time"):
                sp = [(e["num_workers"], base["training_time"] / e["training_time"]) for e in es
                      if e.get("training_time")]
                ax[1, 1].plot(*zip(*sp), marker="o", color=color, label=f"{mode} speedup")
        ax[1, 1].plot([1, 32], [1, 32], "k--", alpha=0.4, label="linear")
        ax[1, 1].set(title="Speedup vs Workers (vs 1 worker)", xscale="log", yscale="log")
        for a in ax.flat:
            a.grid(alpha=0.3)
            if a.get_legend_handles_labels()[0]:
                a.legend()
        out = self.output_dir / "scaling_analysis.png"
        fig.tight_layout()
        fig.savefig(out, dpi=150, bbox_inches="tight")
        plt.close(fig)
        return out if any_data else None

    def plot_bench_scaling(self, records, name="bench_scaling.png"):
        """bench.py JSON lines (one per GPU count) -> img/s and efficiency vs GPUs."""
        plt = self._plt()
        recs = sorted(records, key=lambda r: r["n_gpus"])
        n = [r["n_gpus"] for r in recs]
        v = [r["value"] for r in recs]
        base = v[0] / n[0]
        fig, ax = plt.subplots(1, 2, figsize=(12, 4.5))
        ax[0].plot(n, v, marker="o", label="measured")
        ax[0].plot(n, [base * k for k in n], "k--", alpha=0.4, label="linear")
        ax[0].set(title="Throughput vs GPUs", xlabel="GPUs", ylabel="images/s", xscale="log")
        ax[0].legend()
        ax[1].plot(n, [100 * x / (base * k) for x, k in zip(v, n)], marker="o")
        ax[1].set(title="Weak-scaling efficiency", xlabel="GPUs", ylabel="% of linear", xscale="log", ylim=(0, 105))
        for a in ax:
            a.grid(alpha=0.3)
        out = self.output_dir / name
        fig.tight_layout()
        fig.savefig(out, dpi=150, bbox_inches="tight")
        plt.close(fig)
        return out

    def create_summary_table(self) -> str:
        hdr = f"{'Experiment':28s} {'Mode':6s} {'W':>3s} {'Time(s)':>9s} {'Epoch(s)':>9s} {'Acc(%)':>7s} {'img/s':>10s}"
        lines = [hdr, "-" * len(hdr)]
        for e in sorted(self.experiments, key=lambda e: (e.get("mode") or "", e.get("num_workers") or 0)):
            def f(k, fmt):
                v = e.get(k)
                return format(v, fmt) if isinstance(v, (int, float)) else "-"
            lines.append(f"{e['name'][:28]:28s} {str(e.get('mode', '-')):6s} {str(e.get('num_workers', '-')):>3s} "
                         f"{f('training_time', '9.1f'):>9s} {f('avg_epoch_time', '9.1f'):>9s} "
                         f"{f('final_accuracy', '7.2f'):>7s} {f('images_per_second', '10.1f'):>10s}")
        table = "\n".join(lines)
        print(table)
        (self.output_dir / "summary_table.txt").write_text(table + "\n")
        return table


def save_json(obj, path):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(obj, f, indent=2)
    return path
