"""Async PS with W worker THREADS on one GPU (parallel/runner.py run_local_threads):
every push of every worker reaches the native event loop in real arrival order and is applied or
rejected by the staleness rule; the timed throughput counts accepted pushes only; the workers'
and the server's final records aggregate into the reference's experiment_results schema."""
import contextlib
import io

import pytest
import torch

pytestmark = pytest.mark.gpu

from psx.parallel.runner import run_local_threads  # noqa: E402
from psx.utils import results as R  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402


def test_threads_async(tmp_path):
    W, steps = 3, 4
    cfg = PSConfig(model="resnet18", mode="async", workers=W, lr=0.05, batch_size=32, epochs=1, train_samples=2048,
                   eval_every=0, verbose=0, staleness_bound=5).validate()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        res = run_local_threads(cfg, steps, log=lambda *a, **k: None, emit=True)
    s, tm = res["server"], res["timed"]
    total = W * (steps + 1)  # + each worker's capture step
    assert s["gradients_processed"] == total, s
    assert s["async_updates"] + s["rejected_pushes"] == total, s
    assert sum(s["staleness_histogram"]) == s["async_updates"], s  # the histogram counts accepted pushes
    assert tm["timed_pushes"] == W * steps and 0 <= tm["timed_accepted_pushes"] <= tm["timed_pushes"], tm
    assert tm["images_per_second"] == pytest.approx(tm["timed_accepted_pushes"] * 32 / tm["timed_seconds"], rel=2e-2)  # timed_seconds is rounded
    assert s["final_param_checksum"] == s["final_param_checksum"]  # finite / not NaN
    log = tmp_path / "run.log"
    log.write_text(buf.getvalue())
    agg = R.parse_experiment([str(log)], "async_threads", verbose=False)
    assert agg["server_metrics"]["mode"] == "async"
    assert agg["worker_metrics_aggregated"]["num_workers"] == W
    assert len(agg["raw_worker_metrics"]) == W
    torch.cuda.synchronize()
