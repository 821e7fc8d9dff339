#!/usr/bin/env python3
"""fp8 (W8A16) decode GEMM configuration sweep at Llama-3-70B TP=1 shapes: every register-streaming
(skinny_fp8: nt, splits) and LDS-DMA stream (stream_fp8: wpb, splits) configuration, back-to-back
launches over weight copies beyond the 256 MiB Infinity Cache.  JSON line per (op, M, kernel, config).

    python tools/sweep_fp8_decode.py [--ms 1,4,8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402
from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight  # noqa: E402


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
    ap.add_argument("--ms", default="1")
    ap.add_argument("--ops", default="qkv,o,gate_up,down")
    ap.add_argument("--tp", type=int, default=1, help="one rank's shard of a TP=tp engine")
    a = ap.parse_args()
    dev = "cuda:0"
    t = a.tp
    shapes = {"qkv": (10240 // t, 8192), "o": (8192, 8192 // t), "gate_up": (57344 // t, 8192),
              "down": (8192, 28672 // t)}
    for name in a.ops.split(","):
        N, K = shapes[name]
        ncopy = max(2, int(1.2e9 // (N * K)))
        ws = [Fp8Weight.quantize(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        sw = name == "gate_up"
        it = [0]

        def nxt():
            it[0] += 1
            return ws[it[0] % ncopy]
        for M in (int(m) for m in a.ms.split(",")):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            cands = []
            for nt in ((1,) if sw else (1, 2)):
                if N % (16 * nt):
                    continue
                for S in ((1,) if sw else (1, 2, 4, 8)):
                    if (K // 256) % S:
                        continue
                    if sw:
                        o = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
                        cands.append(("skinny", (nt, S), lambda o=o, nt=nt: hip._skinny_fp8(x, nxt(), o, hip.EPI_SWIGLU, nt, 1, N // 2)))
                    else:
                        o = torch.empty(S, M, N, dtype=torch.float32, device=dev)
                        cands.append(("skinny", (nt, S), lambda o=o, nt=nt, S=S: hip._skinny_fp8(x, nxt(), o, hip.EPI_F32_PARTIAL, nt, S, N)))
            for wpb in (4, 5, 6, 7, 8):
                if N % (16 * wpb):
                    continue
                for S in ((1,) if sw else (1, 2, 4, 8)):
                    if (K // 256) % S:
                        continue
                    grid = N // (16 * wpb) * S
                    if grid < 128 or grid > 1024:
                        continue
                    if sw:
                        o = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
                        cands.append(("stream", (wpb, S), lambda o=o, wpb=wpb: hip._stream_fp8(x, nxt(), o, hip.EPI_SWIGLU, 1, N // 2, wpb)))
                    else:
                        o = torch.empty(S, M, N, dtype=torch.float32, device=dev)
                        cands.append(("stream", (wpb, S), lambda o=o, wpb=wpb, S=S: hip._stream_fp8(x, nxt(), o, hip.EPI_F32_PARTIAL, S, N, wpb)))
            for kind, cfg, f in cands:
                us = min(timeit(f) for _ in range(2))
                print(json.dumps({"op": name, "tp": t, "M": M, "kind": kind, "cfg": cfg, "us": round(us, 1),
                                  "TBps": round(N * K / us / 1e6, 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
