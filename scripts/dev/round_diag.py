"""Diagnostic: drive the graph-captured sync round at world size 1 step by step, printing the
host time of every phase (used to debug parallel/graph_round.py; not part of the package).

usage: RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29599 python scripts/dev/round_diag.py [--steps N]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.parallel.compute import HipCompute  # noqa: E402
from psx.parallel.rccl import make_transport  # noqa: E402
from psx.parallel.runner import build_state, make_datasets, make_sync_channel  # noqa: E402
from psx.parallel.server import ParameterServer  # noqa: E402
from psx.parallel.worker import Worker  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--sync-every", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = PSConfig(model="resnet18", batch_size=128, train_samples=50000, lr=0.1, epochs=1, eval_every=0,
                   verbose=0).validate()
    model, layout, arena, counters = build_state(cfg)
    t = make_transport(dev)
    cfg.workers = 1
    srv = ParameterServer(cfg, layout, arena, counters, device=dev, total_workers=1, log=lambda *x, **k: None)
    srv.register_worker("w0", 0)
    train, _ = make_datasets(cfg, dev, 100)
    comp = HipCompute(model, layout, 128, dev, use_graph=True)
    chan = make_sync_channel(cfg, t, srv, 1, layout, dev)
    print("channel", type(chan).__name__, flush=True)
    wk = Worker(cfg, comp, chan, train, None, worker_name="w0", rank=0, log=lambda *x, **k: None, requested_id=0)
    wk.connect_to_server()
    wk.setup_data()
    batches = wk.sampler.epoch_indices(0)
    for i in range(a.steps):
        t0 = time.perf_counter()
        wk.fetch_parameters()
        t1 = time.perf_counter()
        wk.train_local_batch(batches[i])
        t2 = time.perf_counter()
        wk.push_gradients()
        t3 = time.perf_counter()
        if a.sync_every:
            torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"step {i} fetch {1e3*(t1-t0):.2f} train {1e3*(t2-t1):.2f} push {1e3*(t3-t2):.2f} "
              f"sync {1e3*(t4-t3):.2f} ms", flush=True)
    torch.cuda.synchronize()
    print("done", srv.core.global_step, flush=True)
    t.close()


if __name__ == "__main__":
    main()
