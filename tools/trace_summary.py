#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv: per-kernel total/mean time, grouped by short name."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
tot = defaultdict(float)
cnt = defaultdict(int)
for f in files:
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "?")
            short = name.split("(")[0][:90]
            dt = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            tot[short] += dt
            cnt[short] += 1
total = sum(tot.values())
print("kernel time total %.1f ms over %d dispatches" % (total / 1e3, sum(cnt.values())))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:40]:
    print("%8.1f ms %5.1f%% %7d  %8.1f us  %s" % (v / 1e3, 100 * v / total, cnt[k], v / cnt[k], k))
