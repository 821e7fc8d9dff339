#!/usr/bin/env python3
"""Prefill GEMM throughput: our MFMA kernel (csrc/kernels/gemm.hip) vs hipBLASLt (torch F.linear, the
previous prefill path), interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24),
random operands of the model's init scale.  One JSON line per (shape, variant): median / min us, TF/s.

    python tools/bench_gemm.py [--model llama3-8b] [--ms 4096,16384] [--variants ours,blas] [--fp8]
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402
from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight  # noqa: E402

SHAPES = {
    "llama3-8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)},
    "llama3-70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)},
    "llama3-70b-tp8": {"qkv": (1280, 8192), "o": (8192, 1024), "gate_up": (7168, 8192), "down": (8192, 3584)},
}


def timeit(fn, iters):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ms", default="4096,8192,16384,24576,49152")
    ap.add_argument("--roles", default="qkv,o,gate_up,down")
    ap.add_argument("--variants", default="g4,g8,blas", help="gN = our kernel, group_m N; blas = hipBLASLt")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda:0"
    torch.manual_seed(0)
    for role in a.roles.split(","):
        N, K = SHAPES[a.model][role]
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        wq = Fp8Weight.quantize(w) if a.fp8 else None
        for M in [int(m) for m in a.ms.split(",")]:
            x = (torch.randn(M, K, device=dev)).to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            xq, xs = hip.quant_fp8_rows(x) if a.fp8 else (None, None)
            fns = {}
            for v in a.variants.split(","):
                if v == "blas":
                    if a.fp8:
                        fns[v] = lambda: torch._scaled_mm(xq, wq.q.t(), scale_a=xs.view(-1, 1),
                                                          scale_b=wq.scale.view(1, -1), out_dtype=torch.bfloat16)
                    else:
                        fns[v] = lambda: torch.nn.functional.linear(x, w)
                else:
                    gm = int(v[1:])
                    if a.fp8:
                        fns[v] = (lambda gm=gm: hip.gemm_fp8(xq, xs, wq, out=out, group_m=gm))
                    else:
                        fns[v] = (lambda gm=gm: hip.gemm(x, w, out=out, group_m=gm))
            times = {v: [] for v in fns}
            for f in fns.values():
                f()
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for v, f in fns.items():
                    times[v].append(timeit(f, a.iters))
            flop = 2.0 * M * N * K
            for v, ts in times.items():
                ts.sort()
                med = ts[len(ts) // 2]
                print(json.dumps({"model": a.model, "role": role, "M": M, "N": N, "K": K, "fp8": a.fp8, "variant": v,
                                  "us_med": round(med, 1), "us_min": round(ts[0], 1),
                                  "tflops_med": round(flop / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
