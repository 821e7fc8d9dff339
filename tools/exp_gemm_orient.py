#!/usr/bin/env python3
"""Prefill GEMM throughput (hipBLASLt via F.linear, Llama-3-8B projections) as a function of the packed
token count M: finds the M granularity at which hipBLASLt's heuristics pick its fast kernels."""
import json
import sys
import time

import torch
import torch.nn.functional as F


def bench(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    dev = "cuda:0"
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    Ms = [int(m) for m in sys.argv[1].split(",")] if len(sys.argv) > 1 else \
        [4096, 6144, 8192, 12288, 14336, 15360, 15872, 16000, 16128, 16384, 16640, 17408]
    ws = {n: torch.randn(N, K, device=dev, dtype=torch.bfloat16) for n, (N, K) in shapes.items()}
    for M in Ms:
        row = {"M": M}
        tot_fl, tot_t = 0.0, 0.0
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            t = bench(lambda: F.linear(x, ws[name]))
            fl = 2.0 * M * N * K
            row[name] = round(fl / t / 1e12)
            tot_fl += fl
            tot_t += t
        row["layer_TF"] = round(tot_fl / tot_t / 1e12)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
