#!/usr/bin/env python3
"""bf16 LDS-DMA stream GEMM (decode) configuration sweep at Llama-3-8B shapes: every (waves per workgroup,
split-K) whose grid is 192..512 workgroups, split-K fp32 slabs epilogue, back-to-back launches over weight
copies beyond the 256 MiB Infinity Cache.  The plan in ops/hip.py (stream_config) prefers the fewest
splits among configurations that fill the chip; this tool checks that choice.  JSON line per case.

    python tools/sweep_stream_cfg.py [--ms 1,10,39] [--ops o,down,qkv]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402


def timeit(fn, iters=40, warm=4):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,10,39")
    ap.add_argument("--ops", default="o,down,qkv")
    a = ap.parse_args()
    dev = "cuda:0"
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336), "gate_up": (28672, 4096),
              "o70": (8192, 8192), "down70h": (8192, 14336)}  # 70B o; the fp8 70B down's row bytes in bf16
    for name in a.ops.split(","):
        N, K = shapes[name]
        ncopy = max(2, int(1.2e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        it = [0]

        def nxt():
            it[0] += 1
            return ws[it[0] % ncopy]
        plan = hip.stream_config(N, K)
        for M in (int(m) for m in a.ms.split(",")):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            for wpb in (4, 5, 6, 7, 8):
                if N % (16 * wpb):
                    continue
                for S in range(1, 17):
                    if (K // 128) % S:
                        continue
                    grid = N // (16 * wpb) * S
                    if grid < 192 or grid > 512:
                        continue
                    o = torch.empty(S, M, N, dtype=torch.float32, device=dev)
                    us = min(timeit(lambda: hip._stream_gemm(x, nxt(), o, hip.EPI_F32_PARTIAL, S, N, wpb)) for _ in range(2))
                    print(json.dumps({"op": name, "M": M, "wpb": wpb, "S": S, "grid": grid, "plan": [wpb, S] == list(plan),
                                      "us": round(us, 1), "TBps": round(N * K * 2 / us / 1e6, 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
