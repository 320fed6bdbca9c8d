"""Scaling curve of the headline benchmark: ``bench.py`` at N = 1, 2, 4, 8 GPUs of one node
(SURVEY.md §7.1 bench/scaling.py), for any mode / codec / topology bench.py takes.

Each point is its own job: N = 1 runs ``python bench.py``, N > 1 runs
``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ...``
(one rank per GPU over RCCL), exactly as the round-end driver does. The JSON line of every run is
kept, and the weak-scaling efficiency value(N) / (N * value(1)) is derived here from those values
(the reference quotes "~70-80 %" for its 4 -> 16 Fargate workers, README.md:473).

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


def efficiency(points: dict[int, dict]) -> dict[int, float | None]:
    """Weak-scaling efficiency per N against the N = 1 point (None without one)."""
    base = points.get(1, {}).get("value")
    return {n: (round(p["value"] / (n * base), 4) if base else None) for n, p in sorted(points.items())}


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
    eff = efficiency(points)
    summary = {"mode": a.mode, "bench_args": extra, "points": runs,
               "efficiency_vs_n1": {str(n): e for n, e in eff.items()}}
    with open(a.out, "w") as f:
        json.dump(summary, f, indent=1)
    print(f"{'N':>3} {'img/s':>12} {'ms/step':>9} {'eff':>7}")
    for n, p in sorted(points.items()):
        e = eff[n]
        print(f"{n:>3} {p['value']:>12.1f} {p['ms_per_step']:>9} {e if e is not None else '-':>7}")
    return summary


if __name__ == "__main__":
    main()
