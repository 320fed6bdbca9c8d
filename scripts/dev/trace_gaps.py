"""Summarize a rocprofv3 kernel trace: GPU busy vs wall, idle gaps, per-queue split.

usage: python scripts/dev/trace_gaps.py <kernel_trace.csv> [--last-ms 50]
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last-ms", type=float, default=40.0, help="analyze only the final window (steady state)")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60],
                         r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    end = max(e for _, e, _, _ in rows)
    lo = end - int(a.last_ms * 1e6)
    rows = [r for r in rows if r[0] >= lo]
    t0 = rows[0][0]
    busy = 0
    cur_s, cur_e = rows[0][0], rows[0][1]
    gaps = []
    for s, e, n, q in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = end - t0
    print(f"window {wall / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / wall:.1f}%), kernels {len(rows)}")
    gaps.sort(reverse=True)
    tot = collections.Counter()
    for g, n in gaps:
        tot[n] += g
    print("largest idle gaps (us) before kernel:")
    for g, n in gaps[:15]:
        print(f"  {g / 1e3:8.1f}  {n}")
    q = collections.Counter()
    for s, e, n, qq in rows:
        q[qq] += e - s
    print("per-queue kernel time (ms):", {k: round(v / 1e6, 2) for k, v in q.items()})


if __name__ == "__main__":
    main()
