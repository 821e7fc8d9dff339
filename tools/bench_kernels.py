#!/usr/bin/env python3
"""Kernel micro-benchmarks on one GPU (events, interleaved A/B in one process).

Decode GEMMs (Llama-3-8B shapes): our MFMA weight-streaming kernels vs
torch.nn.functional.linear (hipBLASLt), reported as achieved weight-stream
bandwidth; decode attention as KV bandwidth; prefill attention as TFLOP/s.
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402


def timeit(fn, iters=50, warm=5):
    """Back-to-back launches (as in a decode graph): mean per call."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e-3 / iters


def main():
    dev = "cuda:0"
    torch.manual_seed(0)
    res = {"gemm": [], "attn_decode": [], "attn_prefill": []}
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    # a few big weights so every call streams from HBM (working set >> 256 MiB L3)
    for name, (N, K) in (shapes.items() if os.environ.get("GEMM", "1") == "1" else []):
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(4)]
        for M in (1, 8, 16, 32, 48, 64):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            it = [0]

            def ours():
                w = ws[it[0] % 4]; it[0] += 1
                if name == "gate_up":
                    hip.linear_swiglu(x, w)
                elif name in ("o", "down"):
                    hip.linear_parts(x, w)
                else:
                    hip.linear(x, w)

            def blas():
                w = ws[it[0] % 4]; it[0] += 1
                torch.nn.functional.linear(x, w)

            t1, t2 = timeit(ours), timeit(blas)
            gb = N * K * 2 / 1e9
            res["gemm"].append({"op": name, "M": M, "ours_us": round(t1 * 1e6, 1), "hipblaslt_us": round(t2 * 1e6, 1),
                                "ours_TBps": round(gb / t1 / 1e3, 2), "hipblaslt_TBps": round(gb / t2 / 1e3, 2)})
            print(json.dumps(res["gemm"][-1]), flush=True)
        del ws
    # decode attention: B seqs x ctx, Llama-3-8B kv layout
    hq, hkv, d, page = 32, 8, 128, 64
    for B, ctx in (((1, 8192), (8, 4096), (39, 4400), (64, 2048)) if os.environ.get("DECODE", "1") == "1" else ()):
        npg = -(-ctx // page)
        kc = torch.randn(B * npg + 1, hkv, page, d, device=dev, dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = (torch.arange(B * npg, dtype=torch.int32, device=dev).view(B, npg) + 1)
        pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=dev)
        q = torch.randn(B, (hq + 2 * hkv) * d, device=dev, dtype=torch.bfloat16)
        for splits in sorted({hip.decode_splits(B, hkv, ctx), 4, 8, 16, 32}):
            ws = hip.DecodeWorkspace(B, hq, d, splits, dev, hkv)
            t = timeit(lambda: hip.attn_decode(q, kc, vc, bt, pos, hq, hkv, d, page, 1 / math.sqrt(d), workspace=ws))
            gb = B * ctx * hkv * d * 2 * 2 / 1e9
            res["attn_decode"].append({"B": B, "ctx": ctx, "S": splits, "us": round(t * 1e6, 1),
                                       "TBps": round(gb / t / 1e3, 2)})
            print(json.dumps(res["attn_decode"][-1]), flush=True)
    # prefill attention
    for nseq, L in ((1, 4096), (8, 4096), (4, 8192), (1, 32768)):
        T = nseq * L
        qkv = torch.randn(T, (hq + 2 * hkv) * d, device=dev, dtype=torch.bfloat16)
        cu = torch.arange(0, T + 1, L, dtype=torch.int32, device=dev)
        items = hip.prefill_items([L] * nseq, hq // hkv).to(dev)
        t = timeit(lambda: hip.attn_prefill(qkv, cu, hq, hkv, d, 1 / math.sqrt(d), items=items, seqlens=[L] * nseq),
                   iters=20)
        fl = nseq * 4 * L * L / 2 * d * hq
        res["attn_prefill"].append({"nseq": nseq, "L": L, "ms": round(t * 1e3, 3), "TFLOPs": round(fl / t / 1e12, 1)})
        print(json.dumps(res["attn_prefill"][-1]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bench_kernels.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
