#!/usr/bin/env python3
"""In-situ rate of the prefill GEMMs from a rocprofv3 kernel trace of a Llama-3-8B prefill run
(tools/bench_prefill.py under ``rocprofv3 --kernel-trace --output-format csv``).

Each gemm_kernel dispatch is classified by its place in the layer (the dispatch before a prefill
attention is the QKV projection, the one after it the o projection, the SwiGLU-epilogue variant is
gate_up, the one after gate_up is down) and its tile count (grid / 512 threads = tiles_m x tiles_n, with
tiles_n known per role), so its FLOPs are 2 x M x N x K with M = --rows (the packed rows of a full
prefill batch) when tiles_m = ceil(M / 256).  Prints one JSON line per role: dispatches, mean us,
PFLOP/s (the same count the microbench tools/bench_gemm.py uses).

    python tools/gemm_insitu.py <rocprof output dir> --rows 16000
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--rows", type=int, required=True)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tm = -(-a.rows // 256)
    stats = defaultdict(list)
    prev = ""
    for i, r in enumerate(rows):
        name = r.get("Kernel_Name", "")
        if "gemm_kernel" not in name or "stream" in name:
            prev = name
            continue
        nxt = rows[i + 1].get("Kernel_Name", "") if i + 1 < len(rows) else ""
        if "gemm_kernel<false, 1" in name:
            role = "gate_up"
        elif "attn_prefill" in prev:
            role = "o"
        elif "gemm_kernel<false, 1" in prev:
            role = "down"
        elif "attn_prefill" in nxt or "rope" in nxt:
            role = "qkv"
        else:
            role = None
        prev = name
        if role is None:
            continue
        grid = int(r.get("Grid_Size", 0) or r.get("Grid_Size_X", 0) or 0)
        tiles = grid // 512 if grid else 0
        N, K = SHAPES[role]
        if tiles != tm * (-(-N // 256)):
            continue  # a partial batch (not the --rows shape)
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        stats[role].append(dt)
    for role, ts in stats.items():
        N, K = SHAPES[role]
        us = sum(ts) / len(ts) * 1e6
        print(json.dumps({"role": role, "M": a.rows, "N": N, "K": K, "dispatches": len(ts), "mean_us": round(us, 1),
                          "PFLOPs": round(2 * a.rows * N * K / (us * 1e-6) / 1e15, 3), "source": "in-situ prefill"}))


if __name__ == "__main__":
    main()
