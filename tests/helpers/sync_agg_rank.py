"""One rank of the sync-aggregation check (tests/test_ps_cpu.py::test_sync_round_fp32_aggregation).

Every worker pushes a seeded random fp16 wire through SyncCollectiveChannel over gloo; rank 0's
arena after the round must equal  p0 - lr * mean_k float32(g_k)  computed in float64 numpy from
the same seeds — the reference's decompress-to-fp32 + average (server.py:145-169, 232-237)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import TinyResNet  # noqa: E402
from psx.parallel.server import ParameterServer  # noqa: E402
from psx.parallel.transport import DistTransport  # noqa: E402
from psx.parallel.worker import SyncCollectiveChannel  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402


def wire(seed, n):
    g = torch.Generator().manual_seed(1000 + seed)
    return (torch.randn(n, generator=g) * 3.0).to(torch.float16)


def main():
    topology = sys.argv[1]
    t = DistTransport(backend="gloo")
    rank, world = t.rank, t.world_size
    dedicated = topology == "dedicated"
    workers = list(range(1, world)) if dedicated else list(range(world))
    torch.manual_seed(0)
    m = TinyResNet(10)
    lay = ParamLayout.from_module(m)
    arena, counters = lay.pack(m)
    cfg = PSConfig(mode="sync", workers=len(workers), lr=0.05, verbose=0, model="resnet_tiny").validate()
    server = None
    if rank == 0:
        server = ParameterServer(cfg, lay, arena.clone(), counters, total_workers=len(workers), log=lambda *a: None)
        for i in range(len(workers)):
            server.register_worker(f"w{i}", i)
    chan = SyncCollectiveChannel(t, server, members=list(range(len(workers))), root_worker=not dedicated)
    n = lay.param_numel
    g = wire(rank, n) if rank in workers else torch.zeros(n, dtype=torch.float16)
    p0 = arena[:n].double().numpy().copy()
    chan.push(0, g, 0)
    if rank == 0:
        mean = np.zeros(n)
        for r in workers:
            mean += wire(r, n).float().double().numpy()
        mean /= len(workers)
        want = p0 - 0.05 * mean
        got = server.arena[:n].double().numpy()
        err = float(np.abs(got - want).max() / max(1e-30, np.abs(want).max()))
        # the fp16 RCCL-style alternative for contrast: a running fp16 sum
        acc16 = torch.zeros(n, dtype=torch.float16)
        for r in workers:
            acc16 += wire(r, n)
        err16 = float(np.abs((p0 - 0.05 * acc16.double().numpy() / len(workers)) - want).max() / np.abs(want).max())
        print("RESULT " + json.dumps({"err": err, "err_fp16_sum": err16, "gs": server.core.global_step}), flush=True)
    t.close()


if __name__ == "__main__":
    main()
