#!/usr/bin/env python3
"""Prefill GEMMs (Llama-3-8B, M ~ 16k packed tokens): hipBLASLt default heuristic vs PyTorch
TunableOp's searched solution, TFLOP/s per shape.  Decides whether tuned GEMM selection is worth
wiring into the engine."""
import json
import os
import sys
import time


def bench(fn, reps=10):
    import torch
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", "/tmp/tunableop_results.csv")
    import torch
    import torch.nn.functional as F
    dev = "cuda:0"
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 15872
    res = {}
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        torch.cuda.tunable.enable(False)
        t0 = bench(lambda: F.linear(x, w))
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        F.linear(x, w)  # tunes this shape
        torch.cuda.synchronize()
        t1 = bench(lambda: F.linear(x, w))
        torch.cuda.tunable.enable(False)
        fl = 2.0 * M * N * K
        res[name] = {"default_TFLOPs": round(fl / t0 / 1e12, 1), "tuned_TFLOPs": round(fl / t1 / 1e12, 1)}
        print(json.dumps({"M": M, "op": name, **res[name]}), flush=True)


if __name__ == "__main__":
    main()
