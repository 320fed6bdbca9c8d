"""Async PS on one MI355X with W simulated workers (loopback): images/s and the staleness
histogram — the "async staleness" half of BASELINE.json's metric (reference:
src/parameter_server/server.py:171-186,290-304 — reject above the bound, weight max(0.1,
1/(1+0.1 s)); its experiment JSONs publish no staleness data, server_metrics: null).

The loopback interleaves the W workers' pushes round-robin, so every push after the first round
sees W-1 updates since its fetch. One JSON line per W.

  python bench/async_staleness.py [--workers 4 8] [--steps 60] [--dtype fp32|bf16]
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
from psx.parallel.runner import run_local  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, nargs="+", default=[4, 8])
    ap.add_argument("--steps", type=int, default=60, help="local steps per worker")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--staleness-bound", type=int, default=5)
    a = ap.parse_args()
    for W in a.workers:
        cfg = PSConfig(model="resnet18", mode="async", workers=W, lr=0.1, batch_size=a.batch, epochs=1,
                       train_samples=W * a.batch * a.steps, eval_every=0, verbose=0, dtype=a.dtype,
                       staleness_bound=a.staleness_bound, max_steps=a.steps).validate()
        t0 = time.time()
        with contextlib.redirect_stdout(io.StringIO()):
            res = run_local(cfg, log=lambda *x, **k: None)
        torch.cuda.synchronize()
        wall = time.time() - t0
        s = res["server"]
        print(json.dumps({"bench": "async_staleness", "workers": W, "dtype": a.dtype, "batch": a.batch,
                          "local_steps": a.steps, "images_per_second": s.get("images_per_second"),
                          "wall_s_incl_setup": round(wall, 2), "async_updates": s.get("async_updates"),
                          "rejected": s.get("rejected_pushes", s.get("rejected")),
                          "max_staleness": s.get("max_staleness_observed"),
                          "staleness_histogram": s.get("staleness_histogram"),
                          "staleness_bound": a.staleness_bound}), flush=True)


if __name__ == "__main__":
    main()
