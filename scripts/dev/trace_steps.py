"""Per-step view of a rocprofv3 kernel trace: step = interval between successive launches of a
marker kernel (default: the augment kernel that starts every training step).

usage: python scripts/dev/trace_steps.py <kernel_trace.csv> [--marker augment] [--steps 5]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="augment")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--detail", action="store_true")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70],
                         r.get("Queue_Id", "?")))
    rows.sort()
    marks = [s for s, _, n, _ in rows if a.marker in n]
    spans = list(zip(marks[:-1], marks[1:]))[-a.steps:]
    for s0, s1 in spans:
        ks = [r for r in rows if s0 <= r[0] < s1]
        busy, ce, gaps, prev = 0, s0, [], "<step start>"
        for s, e, n, q in ks:
            if s > ce:
                gaps.append((s - ce, prev, n))
            busy += max(0, e - max(s, ce))
            if e > ce:
                ce, prev = e, n
        print(f"step {(s1 - s0) / 1e3:8.1f} us  busy {busy / 1e3:8.1f} us  kernels {len(ks)}")
        gaps.sort(reverse=True)
        for g, p, n in gaps[: (12 if a.detail else 5)]:
            print(f"     gap {g / 1e3:7.1f} us  after {p[:45]:45s} before {n[:45]}")


if __name__ == "__main__":
    main()
