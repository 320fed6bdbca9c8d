"""bench/scaling.py's efficiency math: the whole-node figure the driver computes and
the per-worker figure, with the dedicated topology's N - 1 workers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

import scaling  # noqa: E402


def _pt(n, value, topo, w):
    return {"n_gpus": n, "value": value, "ms_per_step": 1.0, "config": {"topology": topo, "workers": w}}


def test_whole_node_and_per_worker():
    per = 1000.0
    pts = {1: _pt(1, per, "colocated", 1), 2: _pt(2, per, "dedicated", 1), 4: _pt(4, 3 * per * 0.9, "dedicated", 3),
           8: _pt(8, 7 * per * 0.8, "dedicated", 7)}
    e, w = scaling.efficiency(pts), scaling.efficiency_per_worker(pts)
    assert e == {1: 1.0, 2: 0.5, 4: 0.675, 8: 0.7}  # capped at (N-1)/N by the dedicated server
    assert w == {1: 1.0, 2: 1.0, 4: 0.9, 8: 0.8}
    s = scaling.summarize(pts, list(pts.values()))
    assert s["per_point"]["8"]["topology"] == "dedicated" and s["per_point"]["8"]["workers"] == 7
    assert "worker eff" in scaling.table(s)


def test_workers_fallback_and_missing_base():
    assert scaling.workers({"n_gpus": 8, "config": {"topology": "dedicated"}}) == 7
    assert scaling.workers({"n_gpus": 4, "config": {"topology": "colocated"}}) == 4
    pts = {2: _pt(2, 10.0, "dedicated", 1)}
    assert scaling.efficiency(pts) == {2: None} and scaling.efficiency_per_worker(pts) == {2: None}
