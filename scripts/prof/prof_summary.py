#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (``rocprofv3 --kernel-trace -d DIR -o run``).

Per kernel symbol: calls per step, time per step, share, and the dispatch resources rocprofv3
records (grid / workgroup size, LDS bytes, VGPR / AGPR / SGPR, scratch) — the columns that show
the LDS tiling of each kernel. Only dispatches inside the timed window are counted when
``--skip-first`` drops the warmup dispatches (by the first ``N`` occurrences of a marker kernel)."""
import argparse
import collections
import sqlite3
import sys


def load(db):
    c = sqlite3.connect(db)
    cur = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, lds_size, scratch_size, vgpr_count, "
                    "accum_vgpr_count, sgpr_count, start from kernels order by start")
    return cur.fetchall()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=1, help="divide totals by this many steps")
    ap.add_argument("--csv", default="", help="write the table as CSV too")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args(argv)
    rows = load(a.db)
    agg = collections.OrderedDict()
    for name, dur, gx, gy, gz, wx, lds, scr, vg, ag, sg, _ in rows:
        k = name
        e = agg.setdefault(k, dict(calls=0, ns=0, grids=set(), wx=wx, lds=lds, scr=scr, vg=vg, ag=ag, sg=sg))
        e["calls"] += 1
        e["ns"] += dur
        e["grids"].add(gx // max(1, wx) * gy * gz)
    total = sum(e["ns"] for e in agg.values())
    items = sorted(agg.items(), key=lambda kv: -kv[1]["ns"])
    hdr = ("us/step", "%", "calls/step", "WGs", "WG", "LDS_B", "VGPR", "AGPR", "SGPR", "scratch", "kernel")
    print(f"total kernel time {total / 1e3 / a.steps:.1f} us/step over {len(rows)} dispatches ({a.steps} steps)")
    print("{:>9} {:>5} {:>6} {:>10} {:>4} {:>7} {:>5} {:>5} {:>5} {:>7}  {}".format(*hdr))
    out = []
    for name, e in items[: a.top]:
        g = sorted(e["grids"])
        gs = str(g[0]) if len(g) == 1 else f"{g[0]}-{g[-1]}"
        r = (f"{e['ns'] / 1e3 / a.steps:.1f}", f"{100 * e['ns'] / total:.1f}", f"{e['calls'] / a.steps:.1f}", gs,
             str(e["wx"]), str(e["lds"]), str(e["vg"]), str(e["ag"]), str(e["sg"]), str(e["scr"]), name[:110])
        out.append(r)
        print("{:>9} {:>5} {:>6} {:>10} {:>4} {:>7} {:>5} {:>5} {:>5} {:>7}  {}".format(*r))
    if a.csv:
        import csv

        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(hdr)
            w.writerows(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
