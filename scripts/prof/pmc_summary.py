#!/usr/bin/env python3
"""Summarise rocprofv3 counter collection (``--pmc ... --output-format csv``) per kernel.

Per kernel symbol: dispatches, summed counters, and the ratios that say where a kernel's issue
slots go — VALU instructions per MFMA, LDS instructions per MFMA, LDS bank conflicts per LDS
instruction, and MFMA busy share (SQ_VALU_MFMA_BUSY_CYCLES over SQ_BUSY_CYCLES x SIMDs per SE
block as rocprofv3 sums them; reported raw as well). Writes a CSV with --csv.

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the busy
counter is summed over every SIMD (MI355X_MICROARCH.md: it counts MFMA cycles, 32 per f32
16x16x4 or bf16 32x32x16, 16 per bf16 16x16x32 — ``busy_per_mfma`` checks that), and the GRBM
counter over the 8 XCDs. Cross-check: the fp32 3x3 forward at 64 % here runs at 100 TF/s =
64 % of the 157 TF fp32 peak in bench/conv_layers_f32.py."""
import argparse
import collections
import csv
import glob
import os
import sys


def find_csv(path):
    if os.path.isfile(path):
        return path
    c = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))
    if not c:
        sys.exit(f"no counter_collection.csv under {path}")
    return c[0]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path", nargs="+", help="one directory / CSV per counter pass: merged per kernel")
    ap.add_argument("--csv", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args(argv)
    # per pass: counters summed per kernel, divided by that pass's dispatch count; passes merge
    # per kernel name (each pass is its own run of the same program)
    per = collections.OrderedDict()
    disp = {}
    for path in a.path:
        sums = collections.OrderedDict()
        ids = collections.defaultdict(set)
        for r in csv.DictReader(open(find_csv(path))):
            k = r.get("Kernel_Name") or r.get("kernel_name")
            name = r.get("Counter_Name") or r.get("counter_name")
            val = float(r.get("Counter_Value") or r.get("counter_value") or 0)
            sums.setdefault(k, collections.Counter())[name] += val
            ids[k].add(r.get("Dispatch_Id") or r.get("dispatch_id"))
        for k, d in sums.items():
            n = max(1, len(ids[k]))
            disp[k] = max(disp.get(k, 0), len(ids[k]))
            tgt = per.setdefault(k, collections.Counter())
            for c, v in d.items():
                tgt[c] = v / n
    names = sorted({n for d in per.values() for n in d})
    out = []
    for k, d in per.items():
        mf = d.get("SQ_INSTS_MFMA", 0.0)
        lds = d.get("SQ_INSTS_LDS", 0.0)
        e = {"kernel": k[:100], "dispatches": disp[k]}
        for n in names:
            e[n] = d.get(n, 0.0)
        e["valu_per_mfma"] = round(d.get("SQ_INSTS_VALU", 0.0) / mf, 2) if mf else None
        e["lds_per_mfma"] = round(lds / mf, 2) if mf else None
        e["bank_conflict_per_lds"] = round(d.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds, 3) if lds else None
        busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        e["busy_per_mfma"] = round(busy / mf, 1) if mf else None
        if d.get("GRBM_GUI_ACTIVE"):
            e["mfma_util"] = round(busy / (d["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
        hit, miss = d.get("TCC_HIT_sum", 0.0), d.get("TCC_MISS_sum", 0.0)
        if hit + miss:
            e["l2_hit"] = round(hit / (hit + miss), 3)
        out.append(e)
    out.sort(key=lambda e: -(e.get("SQ_INSTS_MFMA", 0.0) or e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)) * e["dispatches"])
    cols = ["kernel", "dispatches", "mfma_util", "busy_per_mfma", "valu_per_mfma", "lds_per_mfma",
            "bank_conflict_per_lds", "l2_hit"]
    print(" | ".join(cols))
    for e in out[: a.top]:
        print(" | ".join(str(e.get(c)) for c in cols))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=cols[:2] + names + cols[2:])
            w.writeheader()
            for e in out:
                w.writerow({c: e.get(c) for c in cols[:2] + names + cols[2:]})
    return 0


if __name__ == "__main__":
    sys.exit(main())
