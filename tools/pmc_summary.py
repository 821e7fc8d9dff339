#!/usr/bin/env python3
"""Join a rocprofv3 --pmc counter_collection.csv with its kernel_trace.csv: per kernel, mean duration,
HBM read bytes (FETCH_SIZE x 2: on gfx950 FETCH_SIZE tallies 128-B requests as 64 B,
MI355X_MICROARCH.md) -> achieved read TB/s, and MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES (summed
over SIMDs; 32 per 32x32x16 bf16 MFMA) / (kernel cycles at 2.4 GHz x 1024 SIMDs) when collected, and
the SQ_WAIT_* / SQ_ACTIVE_* counters as shares of SQ_WAVE_CYCLES (where a wave's time goes)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    trace = {}
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            trace[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
    ctr = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            d = row["Dispatch_Id"]
            names[d] = row["Kernel_Name"].split("(")[0][:70]
            ctr[d][row["Counter_Name"]] += float(row["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(float))
    for d, cs in ctr.items():
        k = names[d]
        a = agg[k]
        a["n"] += 1
        a["us"] += trace.get(d, 0.0)
        for c, v in cs.items():
            a[c] += v
    extra = sorted({c for a in agg.values() for c in a if c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE")})
    print("%-70s %6s %9s %9s %8s %8s %8s %s" % ("kernel", "calls", "mean_us", "read_MB", "TB/s", "mfma%", "ldsconf%",
                                                 " ".join("%%%s" % c[3:] for c in extra)))
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["us"])[:30]:
        n = a["n"]
        us = a["us"] / n
        rd = 2 * a.get("FETCH_SIZE", 0.0) * 1024 / n  # FETCH_SIZE is in KiB
        tbps = rd / (us * 1e-6) / 1e12 if us else 0.0
        mf = ""
        if "SQ_VALU_MFMA_BUSY_CYCLES" in a and us:
            mf = "%.1f" % (100.0 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / n / (us * 2.4e3 * 1024))
        lc = ""  # LDS bank-conflict cycles as a share of all LDS-array cycles
        if a.get("SQ_LDS_IDX_ACTIVE"):
            lc = "%.1f" % (100.0 * a.get("SQ_LDS_BANK_CONFLICT", 0.0) / a["SQ_LDS_IDX_ACTIVE"])
        wc = a.get("SQ_WAVE_CYCLES", 0.0)
        shares = " ".join("%5.1f" % (100.0 * a[c] / wc) if wc else "-" for c in extra)
        print("%-70s %6d %9.1f %9.1f %8.2f %8s %8s %s" % (k, n, us, rd / 1e6, tbps, mf, lc, shares))
    shown = {"n", "us", "FETCH_SIZE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT"}
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["us"])[:30]:
        rest = {c: v / a["n"] for c, v in a.items() if c not in shown and not c.startswith(("SQ_WAIT", "SQ_ACTIVE"))}
        if rest:  # other counters: mean per dispatch
            print("  %-68s %s" % (k, " ".join("%s=%.4g" % kv for kv in sorted(rest.items()))))


if __name__ == "__main__":
    main(sys.argv[1])
