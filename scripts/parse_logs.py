#!/usr/bin/env python3
"""Aggregate METRICS_JSON records of a run into the reference's experiment-result schema.

Counterpart of the reference's scripts/parse_cloudwatch_logs.py (which downloads CloudWatch
log groups): the inputs here are local — captured stdout of `psx_train.py` / `torchrun` runs
or the per-rank jsonl files written with --log-dir.

  python scripts/parse_logs.py --experiment-name sync_4workers run.log [more logs or dirs] \\
      [--output experiment_results/sync_4workers.json]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import psx  # noqa: E402,F401
from psx.utils.results import parse_experiment, save_json  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("sources", nargs="+", help="log files or directories (searched recursively)")
    ap.add_argument("--experiment-name", required=True)
    ap.add_argument("--output", default=None, help="default: experiment_results/<name>.json")
    a = ap.parse_args(argv)
    res = parse_experiment(a.sources, a.experiment_name)
    out = a.output or os.path.join("experiment_results", f"{a.experiment_name}.json")
    save_json(res, out)
    print(f"Results saved to: {out}")
    return 0 if (res["server_metrics"] or res["raw_worker_metrics"]) else 1


if __name__ == "__main__":
    raise SystemExit(main())
