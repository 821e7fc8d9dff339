#!/usr/bin/env python3
"""bf16 prefill GEMM: gemm.hip (8 waves) vs gemm4w.hip (4 waves, 4- and 5-step rings) vs hipBLASLt on the
Llama-3-8B projections, interleaved rounds in one process after a sustained warm-up (random operands)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llm_map_reduce_summarizer_amd.ops import hip
    dev = torch.device("cuda:0")
    M = int(os.environ.get("M", "16384"))
    for role, (N, K, sw) in {"qkv": (6144, 4096, False), "o": (4096, 4096, False),
                             "gate_up": (28672, 4096, True), "down": (4096, 14336, False)}.items():
        g = torch.Generator(device="cpu").manual_seed(1)
        x = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
        w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16).to(dev)
        out = torch.empty(M, N // 2 if sw else N, dtype=torch.bfloat16, device=dev)
        ref = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        fns = {"8w": lambda: hip.gemm(x, w, out=out, swiglu=sw, kernel="8w"),
               "4w": lambda: hip.gemm(x, w, out=out, swiglu=sw, kernel="4w"),
               "4w5": lambda: hip.gemm(x, w, out=out, swiglu=sw, kernel="4w5"),
               "4wL": lambda: hip.gemm(x, w, out=out, swiglu=sw, kernel="4wL"),
               "4w5L": lambda: hip.gemm(x, w, out=out, swiglu=sw, kernel="4w5L"),
               "blas": lambda: torch.matmul(x, w.t(), out=ref)}
        # agreement of the two own kernels (same math, different summation order)
        a = hip.gemm(x, w, swiglu=sw, kernel="8w").float()
        b = hip.gemm(x, w, swiglu=sw, kernel="4w").float()
        c = hip.gemm(x, w, swiglu=sw, kernel="4w5").float()
        rel = float((a - b).norm() / a.norm()), float((a - c).norm() / a.norm())
        t_end = time.time() + 1.5
        while time.time() < t_end:
            for f in fns.values():
                f()
            torch.cuda.synchronize()
        res = {k: [] for k in fns}
        for _ in range(5):
            for k, f in fns.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    f()
                e1.record()
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) * 1000 / 5)
        fl = 2.0 * M * N * K
        row = {"role": role, "M": M, "N": N, "K": K, "rel_diff_4w_4w5": [round(r, 5) for r in rel]}
        for k, v in res.items():
            us = statistics.median(v)
            row[k + "_us"] = round(us, 1)
            row[k + "_tflops"] = round(fl / us / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
