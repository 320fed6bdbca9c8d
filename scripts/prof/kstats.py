"""Per-kernel summary from a rocprofv3 kernel trace, restricted to the last N steps
(steps delimited by a marker kernel), grouped by kernel template.

usage: python scripts/prof/kstats.py run_kernel_trace.csv|run_results.db [--steps 20] [--marker augment]
       [--grid REGEX]  (kernels matching REGEX split per launch grid, CSV input: one line per layer shape)
(rocprofv3 writes a rocpd SQLite database by default, a CSV with --output-format csv)
"""
import argparse
import collections
import csv
import re


def short(n):
    if " grid=(" in n:
        return n[:100]
    n = re.sub(r"\(.*$", "", n) if not n.startswith("void ") else re.sub(r"\((?![^<]*>).*$", "", n[5:])
    return n[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="augment")
    ap.add_argument("--grid", default=None)
    a = ap.parse_args()
    rows = []
    if a.csv.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(a.csv)
        rows = [(int(s), int(e), n) for s, e, n in con.execute("select start, end, name from kernels")]
    else:
        with open(a.csv) as f:
            for r in csv.DictReader(f):
                n = r["Kernel_Name"]
                if a.grid and re.search(a.grid, n):
                    n = f"{short(n)} grid=({r.get('Grid_Size_X')},{r.get('Grid_Size_Y')},{r.get('Grid_Size_Z')})"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    rows.sort()
    marks = [s for s, _, n in rows if a.marker in n]
    lo, hi = marks[-a.steps - 1], marks[-1]
    sel = [r for r in rows if lo <= r[0] < hi]
    tot = collections.defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        k = short(n)
        tot[k][0] += 1
        tot[k][1] += e - s
    busy = sum(v[1] for v in tot.values())
    wall = hi - lo
    print(f"{a.steps} steps: wall {wall / a.steps / 1e3:.1f} us/step, kernel time {busy / a.steps / 1e3:.1f} us/step")
    print(f"{'kernel':100s} {'calls/step':>10s} {'us/step':>9s} {'%':>6s}")
    for k, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:100s} {c / a.steps:10.1f} {t / a.steps / 1e3:9.1f} {100 * t / busy:6.1f}")


if __name__ == "__main__":
    main()
