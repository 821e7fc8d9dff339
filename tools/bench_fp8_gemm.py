#!/usr/bin/env python3
"""fp8 (W8A16) decode GEMMs at Llama-3-70B shapes (TP=1 and TP=8 shards): LDS-DMA stream kernel (256-wide
k slots) vs the register-streaming skinny_fp8 kernel, back-to-back launches over weights beyond the
256 MiB Infinity Cache.  One JSON line per (shape, M)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402
from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight  # noqa: E402


def timeit(fn, iters=50, warm=5):
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
    dev = "cuda:0"
    shapes = [("qkv", 10240, 8192), ("o", 8192, 8192), ("gate_up", 57344, 8192), ("down", 8192, 28672),
              ("qkv_tp8", 1280, 8192), ("o_tp8", 8192, 1024), ("gate_up_tp8", 7168, 8192), ("down_tp8", 8192, 3584)]
    for name, N, K in shapes:
        ncopy = max(2, int(1.5e9 // (N * K)))
        ws = [Fp8Weight.quantize(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        sw = name.startswith("gate_up")
        for M in (1, 16, 40):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            it = [0]

            def nxt():
                it[0] += 1
                return ws[it[0] % ncopy]
            osw = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
            t_sk = timeit(lambda: hip._skinny_fp8(x, nxt(), osw, hip.EPI_SWIGLU, 1, 1, N // 2) if sw else
                          hip.fp8_linear_parts(x, nxt(), *(_skinny_cfg(hip, name, M, N, K))))
            cfg = hip.stream_config(N, K // 2, swiglu=sw)  # the stream kernel's config, whatever the plan says
            t_st = None
            if cfg is not None:
                t_st = timeit(lambda: hip.fp8_linear_swiglu(x, nxt()) if sw else
                              hip.fp8_linear_parts(x, nxt(), cfg[1], stream_wpb=cfg[0]))
            print(json.dumps({"op": name, "M": M, "N": N, "K": K, "skinny_us": round(t_sk, 1),
                              "skinny_TBps": round(N * K / t_sk / 1e6, 2), "stream_cfg": cfg,
                              "stream_us": t_st and round(t_st, 1),
                              "stream_TBps": t_st and round(N * K / t_st / 1e6, 2)}), flush=True)
        del ws


def _skinny_cfg(hip, name, M, N, K):
    p = hip.plan(name.split("_tp")[0], M, N, K, stream=False)
    nt = p[1] if p[0] == "skinny" else 1
    s = p[2] if p[0] == "skinny" else (p[1] if p[0] == "lds" else 1)
    if N % (16 * nt):
        nt = 1
    return s, nt


if __name__ == "__main__":
    main()
