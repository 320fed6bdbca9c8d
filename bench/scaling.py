"""Scaling curve of the headline benchmark: ``bench.py`` at N = 1, 2, 4, 8 GPUs of one node
(SURVEY.md §7.1 bench/scaling.py), for any mode / codec / topology bench.py takes.

Each point is its own job: N = 1 runs ``python bench.py``, N > 1 runs
``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ...``
(one rank per GPU over RCCL), exactly as the round-end driver does. The JSON line of every run is
kept, and two efficiencies are derived from those values (the reference quotes "~70-80 %" for its
4 -> 16 Fargate workers, README.md:473):

  whole node   value(N) / (N * value(1))            what the driver computes from the values
  per worker   value(N) / (W(N) * value(1) / W(1))  W = the point's data-parallel workers

They differ by topology: N = 1 co-locates the server with its one worker, N >= 2 dedicates rank 0
to the server (the reference's layout, BASELINE configs 2-4), so W(N) = N - 1 and the whole-node
figure is capped at (N - 1) / N (50 % at N = 2, 87.5 % at N = 8) even with free communication;
the per-worker figure is what communication and the server cost. Each point also carries its
topology, worker count and (dedicated sync, native server) rank 0's device time per round per
phase (``server_round_us``: gather incl. waiting for the workers, apply, broadcast).

    python bench/scaling.py                              # sync, N = 1 2 4 8 (capped by visible GPUs)
    python bench/scaling.py --gpus 1 2 --mode async -- --codec topk
    python bench/scaling.py --dry-run                    # print the commands only

Everything after ``--`` is passed to bench.py. Writes ``--out`` (JSON) with every point.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def command(n: int, steps: int, warmup: int, extra: list[str], port: int | None = None) -> list[str]:
    bench = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup)] + extra
    if n == 1:
        return [sys.executable] + bench
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port or free_port())] + bench


def parse_result(stdout: str) -> dict:
    """The last JSON object line bench.py printed (rank 0)."""
    for line in reversed(stdout.splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise ValueError("no bench.py JSON line in the output")


def workers(p: dict) -> int:
    """Data-parallel workers of a bench.py point (config.workers; N - 1 for the dedicated topology)."""
    cfg = p.get("config", {})
    if cfg.get("workers"):
        return int(cfg["workers"])
    n = int(p.get("n_gpus", 1))
    return n - 1 if cfg.get("topology") == "dedicated" and n > 1 else n


def efficiency(points: dict[int, dict]) -> dict[int, float | None]:
    """Whole-node weak-scaling efficiency per N against the N = 1 point (None without one)."""
    base = points.get(1, {}).get("value")
    return {n: (round(p["value"] / (n * base), 4) if base else None) for n, p in sorted(points.items())}


def efficiency_per_worker(points: dict[int, dict]) -> dict[int, float | None]:
    """value(N) / (W(N) * per-worker value(1)): the scaling of the workers actually training."""
    b = points.get(1)
    if not b or not b.get("value"):
        return {n: None for n in sorted(points)}
    per1 = b["value"] / workers(b)
    return {n: round(p["value"] / (workers(p) * per1), 4) for n, p in sorted(points.items())}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", choices=["sync", "async"], default="sync")
    ap.add_argument("--timeout", type=float, default=900.0, help="per point, seconds")
    ap.add_argument("--out", default="scaling.json")
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    extra = ["--mode", a.mode] + extra
    visible = None
    if not a.dry_run:
        import torch

        visible = torch.cuda.device_count()
    points, runs = {}, []
    for n in a.gpus:
        cmd = command(n, a.steps, a.warmup, extra)
        if a.dry_run:
            print(" ".join(cmd))
            continue
        if visible is not None and n > visible:
            print(f"[scaling] skip N={n}: {visible} GPU(s) visible", file=sys.stderr)
            continue
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           timeout=a.timeout)
        if r.returncode != 0:
            print(f"[scaling] N={n} failed (exit {r.returncode}):\n{r.stderr[-3000:]}", file=sys.stderr)
            runs.append({"n_gpus": n, "error": r.returncode})
            continue
        res = parse_result(r.stdout)
        points[n] = res
        runs.append(res)
        print(f"[scaling] N={n}: {res['value']:.1f} {res['unit']} ({res['ms_per_step']} ms/step)", flush=True)
    if a.dry_run:
        return None
    summary = summarize(points, runs, a.mode, extra)
    with open(a.out, "w") as f:
        json.dump(summary, f, indent=1)
    print(table(summary))
    return summary


def summarize(points: dict[int, dict], runs: list, mode: str = "sync", extra=()) -> dict:
    eff, effw = efficiency(points), efficiency_per_worker(points)
    per_point = {}
    for n, p in sorted(points.items()):
        cfg = p.get("config", {})
        per_point[str(n)] = {"topology": cfg.get("topology"), "workers": workers(p), "value": p["value"],
                             "ms_per_step": p.get("ms_per_step"), "whole_node_eff": eff[n],
                             "per_worker_eff": effw[n], "server_round_us": p.get("server_round_us")}
    return {"mode": mode, "bench_args": list(extra), "points": runs,
            "efficiency_vs_n1": {str(n): e for n, e in eff.items()},
            "per_worker_efficiency_vs_n1": {str(n): e for n, e in effw.items()}, "per_point": per_point}


def table(summary: dict) -> str:
    rows = [f"{'N':>3} {'topology':>10} {'W':>3} {'img/s':>12} {'ms/step':>9} {'node eff':>9} {'worker eff':>10}"]
    for n, q in summary["per_point"].items():
        fmt = lambda e: f"{e:.3f}" if e is not None else "-"  # noqa: E731
        rows.append(f"{n:>3} {str(q['topology']):>10} {q['workers']:>3} {q['value']:>12.1f} {q['ms_per_step']!s:>9} "
                    f"{fmt(q['whole_node_eff']):>9} {fmt(q['per_worker_eff']):>10}")
    return "\n".join(rows)


if __name__ == "__main__":
    main()
