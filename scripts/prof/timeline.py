#!/usr/bin/env python3
"""Per-queue busy time and the step's kernel timeline from a rocprofv3 kernel trace (CSV):
which hardware queue (graph replay maps streams onto queues) carries how much kernel time per
step, how much of the step wall two queues overlap, and the idle gaps of the busiest queue.

  python scripts/prof/timeline.py run_kernel_trace.csv [--steps 8] [--marker augment] [--list]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--marker", default="augment")
    ap.add_argument("--list", action="store_true", help="print the last step's kernels in start order")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[3]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} markers")
    lo, hi = marks[-a.steps - 1], marks[-1]
    win = rows[lo:hi]
    t0, t1 = rows[lo][0], rows[hi][0]
    wall = (t1 - t0) / a.steps / 1e3
    busy = collections.defaultdict(float)
    for s, e, q, _ in win:
        busy[q] += (e - s) / 1e3
    print(f"{a.steps} steps: wall {wall:.1f} us/step")
    for q, b in sorted(busy.items(), key=lambda kv: -kv[1]):
        print(f"  queue {q}: kernel time {b / a.steps:.1f} us/step")
    # union busy time (any queue) and overlap
    ev = sorted([(s, 1) for s, e, _, _ in win] + [(e, -1) for s, e, _, _ in win])
    depth, last, any_busy, multi = 0, t0, 0, 0
    for t, d in ev:
        if depth >= 1:
            any_busy += t - last
        if depth >= 2:
            multi += t - last
        depth += d
        last = t
    print(f"  any kernel running: {any_busy / a.steps / 1e3:.1f} us/step; >= 2 concurrent: {multi / a.steps / 1e3:.1f}")
    if a.list:
        ls, le = marks[-2], marks[-1]
        base = rows[ls][0]
        for s, e, q, n in rows[ls:le]:
            n = re.sub(r"\(.*", "", n.replace("void ", ""))[:70]
            print(f"  q{q} {(s - base) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n}")


if __name__ == "__main__":
    main()
