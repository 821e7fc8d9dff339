#!/usr/bin/env python3
"""Where a decode step's wall time goes: kernel time vs the idle gaps between consecutive kernels.

Reads a rocprofv3 kernel_trace.csv (one GPU queue), keeps the dispatches between the first and last
kernel whose name contains --marker (default: the sampler, one per decode step), and reports per step:
kernel-busy time, idle gap time (start of kernel i+1 - end of kernel i, clipped at 0), dispatch count,
plus the median per-kernel duration and the median gap AFTER each kernel name.

    python tools/trace_gaps.py <rocprof output dir> [--marker sample_kernel] [--skip 2]
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--marker", default="sample_kernel")
    ap.add_argument("--skip", type=int, default=4, help="steps to skip at the start (warm-up / capture)")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?").split("(")[0][:70]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    steps = []
    per_kernel = defaultdict(list)
    gap_after = defaultdict(list)
    for s, e in zip(marks[a.skip:], marks[a.skip + 1:]):
        seg = rows[s + 1:e + 1]  # one step: after a sample kernel up to and including the next one
        if not seg:
            continue
        busy = sum(r[1] - r[0] for r in seg)
        gaps = [max(0, seg[i + 1][0] - seg[i][1]) for i in range(len(seg) - 1)]
        span = seg[-1][1] - seg[0][0]
        steps.append((span, busy, sum(gaps), len(seg)))
        for i, r in enumerate(seg):
            per_kernel[r[2]].append(r[1] - r[0])
            if i + 1 < len(seg):
                gap_after[r[2]].append(gaps[i])
    if not steps:
        print("no steps found")
        return
    med = lambda xs: statistics.median(xs)  # noqa: E731
    print("steps %d: span %.1f us, kernel-busy %.1f us, gaps %.1f us, %d dispatches per step (medians)"
          % (len(steps), med([s[0] for s in steps]) / 1e3, med([s[1] for s in steps]) / 1e3,
             med([s[2] for s in steps]) / 1e3, med([s[3] for s in steps])))
    nsteps = len(steps)
    print("%-72s %6s %9s %9s %9s" % ("kernel", "n/step", "med us", "sum us", "gap after"))
    for k, v in sorted(per_kernel.items(), key=lambda kv: -sum(kv[1])):
        print("%-72s %6.1f %9.2f %9.1f %9.2f" % (k, len(v) / nsteps, med(v) / 1e3, sum(v) / nsteps / 1e3,
                                                med(gap_after[k]) / 1e3 if gap_after[k] else 0.0))


if __name__ == "__main__":
    main()
