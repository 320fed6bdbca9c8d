"""Async PS on one MI355X with W worker THREADS (real arrival order): images/s over accepted
pushes and the staleness distribution — the "async staleness" half of BASELINE.json's metric
(reference: src/parameter_server/server.py:171-186,290-304 — reject above the bound, weight
max(0.1, 1/(1+0.1 s)); its experiment JSONs publish no staleness data, server_metrics: null).

Each worker is a host thread with its own HIP stream, engine and step graph, pushing into the
native event loop as its steps complete (parallel/runner.py run_local_threads); round 5's version
interleaved a loopback's pushes round-robin, which gives every push staleness exactly W - 1.
One JSON line per W; with --out-dir also the run's METRICS_JSON log and its aggregate in the
reference's experiment_results schema (utils/results.py parse_experiment).

  python bench/async_staleness.py [--workers 4 7] [--steps 30] [--dtype fp32|bf16] [--out-dir DIR]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.parallel.runner import run_local_threads  # noqa: E402
from psx.utils import results as R  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, nargs="+", default=[4, 7])
    ap.add_argument("--steps", type=int, default=30, help="timed local steps per worker (after one capture step)")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--staleness-bound", type=int, default=5)
    ap.add_argument("--out-dir", default=None)
    a = ap.parse_args()
    for W in a.workers:
        cfg = PSConfig(model="resnet18", mode="async", workers=W, lr=0.1, batch_size=a.batch, epochs=1,
                       train_samples=50000, eval_every=0, verbose=0, dtype=a.dtype,
                       staleness_bound=a.staleness_bound).validate()
        t0 = time.time()
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            res = run_local_threads(cfg, a.steps, log=lambda *x, **k: None, emit=True)
        torch.cuda.synchronize()
        wall = time.time() - t0
        s, tm = res["server"], res["timed"]
        rec = {"bench": "async_staleness", "arrival": "worker threads", "workers": W, "dtype": a.dtype,
               "batch": a.batch, "timed_steps_per_worker": a.steps,
               "images_per_second_accepted": tm["images_per_second"],
               "images_per_second_all_pushes": tm["images_per_second_all_pushes"],
               "timed_pushes": tm["timed_pushes"], "timed_accepted_pushes": tm["timed_accepted_pushes"],
               "wall_s_incl_setup": round(wall, 2), "async_updates": s.get("async_updates"),
               "rejected": s.get("rejected_pushes"), "max_staleness": s.get("max_staleness_observed"),
               "mean_staleness_all": s.get("mean_staleness_all"),
               "staleness_histogram": s.get("staleness_histogram"), "staleness_bound": a.staleness_bound}
        print(json.dumps(rec), flush=True)
        if a.out_dir:
            os.makedirs(a.out_dir, exist_ok=True)
            name = f"async_{W}workers_threads_{a.dtype}"
            log = os.path.join(a.out_dir, name + ".log")
            with open(log, "w") as f:
                f.write(buf.getvalue())
            with contextlib.redirect_stdout(io.StringIO()):
                agg = R.parse_experiment([log], name, verbose=False)
            R.save_json(agg, os.path.join(a.out_dir, name + ".json"))


if __name__ == "__main__":
    main()
