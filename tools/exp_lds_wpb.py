#!/usr/bin/env python3
"""Sweep the LDS decode GEMM over waves-per-block (tile rows = 16 * wpb) and split-K, per projection
and batch size; rotating weight copies (cold HBM).  Output: one JSON line per config + best per (op, M)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402


def b2b(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / n


dev = "cuda:0"
best = {}
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336), "gate_up": (28672, 4096)}
if os.environ.get("SHAPES") == "70b":
    shapes = {"qkv": (1280, 8192), "o": (8192, 1024), "down": (8192, 3584), "gate_up": (7168, 8192)}
for name, (N, K) in shapes.items():
    ncopy = max(2, int(1.2e9 // (N * K * 2)))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
    it = [0]

    def nxt():
        it[0] += 1
        return ws[it[0] % ncopy]

    nb = N * K * 2
    for M in (int(m) for m in os.environ.get("MS", "1,8,16,39,64").split(",")):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        for wpb in (4, 5, 6, 7, 8):
            if N % (16 * wpb):
                continue
            for S in (1, 2, 4, 7, 8, 14, 16):
                if (K // 128) % S:
                    continue
                if name == "gate_up" and S > 2:
                    continue
                o = torch.empty(S, M, N, dtype=torch.float32, device=dev)
                t = b2b(lambda: hip._skinny_lds(x, nxt(), o, hip.EPI_F32_PARTIAL, S, N, 2, wpb))
                r = {"op": name, "M": M, "wpb": wpb, "S": S, "grid": N // (16 * wpb) * S, "us": round(t, 1),
                     "TBps": round(nb / t / 1e6, 2)}
                print(json.dumps(r), flush=True)
                k = (name, M)
                if k not in best or t < best[k]["us"]:
                    best[k] = r
                if os.environ.get("STREAM", "1") == "1":
                    t = b2b(lambda: hip._stream_gemm(x, nxt(), o, hip.EPI_F32_PARTIAL, S, N, wpb))
                    r = {"op": name, "M": M, "kind": "stream", "wpb": wpb, "S": S, "grid": N // (16 * wpb) * S,
                         "us": round(t, 1), "TBps": round(nb / t / 1e6, 2)}
                    print(json.dumps(r), flush=True)
                    k = (name + "_stream", M)
                    if k not in best or t < best[k]["us"]:
                        best[k] = r
            if name == "gate_up":
                o = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
                t = b2b(lambda: hip._stream_gemm(x, nxt(), o, hip.EPI_SWIGLU, 1, N // 2, wpb))
                r = {"op": name, "M": M, "kind": "stream", "wpb": wpb, "S": 1, "swiglu": True, "us": round(t, 1),
                     "TBps": round(nb / t / 1e6, 2)}
                print(json.dumps(r), flush=True)
                k = (name + "_stream_swiglu", M)
                if k not in best or t < best[k]["us"]:
                    best[k] = r
                t = b2b(lambda: hip._skinny_lds(x, nxt(), o, hip.EPI_SWIGLU, 1, N // 2, 2, wpb))
                r = {"op": name, "M": M, "wpb": wpb, "S": 1, "swiglu": True, "us": round(t, 1),
                     "TBps": round(nb / t / 1e6, 2)}
                print(json.dumps(r), flush=True)
                k = (name + "_swiglu", M)
                if k not in best or t < best[k]["us"]:
                    best[k] = r
        t = b2b(lambda: torch.nn.functional.linear(x, nxt()))
        print(json.dumps({"op": name, "M": M, "kind": "hipblaslt", "us": round(t, 1), "TBps": round(nb / t / 1e6, 2)}))
    del ws
    torch.cuda.empty_cache()
print("BEST")
for k, r in best.items():
    print(json.dumps(r))
