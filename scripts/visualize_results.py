#!/usr/bin/env python3
"""Plots + summary table from experiment result JSONs (reference scripts/visualize_results.py).

  python scripts/visualize_results.py --results-dir experiment_results --output-dir plots
  python scripts/visualize_results.py --bench SCALE.jsonl --output-dir plots   # bench.py lines
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import psx  # noqa: E402,F401
from psx.utils.results import ExperimentVisualizer  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--results-dir", default=None)
    ap.add_argument("--results", nargs="*", default=[], help="individual result JSON files")
    ap.add_argument("--bench", default=None, help="file of bench.py JSON lines (one per GPU count)")
    ap.add_argument("--output-dir", default="./plots")
    ap.add_argument("--workers", type=int, default=None, help="only this worker count for sync-vs-async")
    a = ap.parse_args(argv)
    v = ExperimentVisualizer(a.output_dir)
    if a.results_dir:
        v.load_experiments_from_directory(a.results_dir)
    for r in a.results:
        v.load_experiment(r)
    if v.experiments:
        v.plot_sync_vs_async_comparison(a.workers)
        v.plot_scaling_analysis()
        v.create_summary_table()
    if a.bench:
        recs = []
        with open(a.bench) as f:
            for ln in f:
                ln = ln.strip()
                if ln.startswith("{"):
                    try:
                        r = json.loads(ln)
                    except json.JSONDecodeError:
                        continue
                    if "n_gpus" in r and "value" in r:
                        recs.append(r)
        if recs:
            print("bench scaling plot:", v.plot_bench_scaling(recs))
    print(f"Plots written to {a.output_dir}")


if __name__ == "__main__":
    main()
