#!/usr/bin/env python3
"""Micro-benchmarks of the TP-shard decode blocks of Llama-3-8B on one GPU (events, back-to-back
launches): decode attention from QKV split-K slabs at hkv = 8 / TP (attention split count sweep),
and the gate_up + SwiGLU GEMM at N = 2 * 14336 / TP (split-K SwiGLU vs the register-streaming /
LDS-x / hipBLASLt alternatives).  One JSON line per measurement."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip, reference  # noqa: E402


def timeit(fn, iters=100, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def main():
    dev = "cuda:0"
    tps = [int(t) for t in os.environ.get("TPS", "8,4,1").split(",")]
    do_gemm = os.environ.get("GEMM", "1") == "1"
    do_attn = os.environ.get("ATTN", "1") == "1"
    ctx = int(os.environ.get("CTX", "4000"))
    for tp in tps:
        hq, hkv, d, page = 32 // tp, 8 // tp, 128, 64
        for B in ((1, 10, 39) if do_attn else ()):
            npg = -(-ctx // page) + 1
            n_pages = B * npg + 1
            kc = torch.randn(n_pages, hkv, page, d, device=dev, dtype=torch.bfloat16)
            vc = torch.randn_like(kc)
            bt = (1 + torch.arange(B * npg, dtype=torch.int32, device=dev)).view(B, npg)
            pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=dev)
            cs = reference.rope_cos_sin(ctx + 64, d, 500000.0, dev)
            for SP in ((2, 4) if tp == 1 else (4, 16)):
                parts = torch.randn(SP, B, (hq + 2 * hkv) * d, device=dev) * 0.5
                for S in (8, 16, 32, 64):
                    for fused in (False, True):
                        if S > npg:
                            continue
                        ws = hip.DecodeWorkspace(B, hq, d, S, dev, hkv, fused_combine=fused)
                        us = timeit(lambda: hip.attn_decode_rope(parts, cs, kc, vc, bt, pos, hq, hkv, d, page,
                                                                 1 / math.sqrt(d), workspace=ws))
                        kv = B * ctx * hkv * d * 2 * 2
                        print(json.dumps({"op": "attn_decode_rope", "tp": tp, "B": B, "ctx": ctx, "qkv_slabs": SP,
                                          "splits": S, "fused_combine": fused, "us": round(us, 2),
                                          "kv_TBps": round(kv / us / 1e6, 2),
                                          "default_splits": hip.decode_splits(B, hkv, ctx + 64)}), flush=True)
        if not do_gemm:
            continue
        N, K = 2 * 14336 // tp, 4096
        ws_ = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(8)]
        for M in (1, 10, 39):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            out = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
            it = [0]

            def nxt():
                it[0] += 1
                return ws_[it[0] % len(ws_)]

            cands = {"skinny": lambda: hip.linear_swiglu(x, nxt(), out, kernel="skinny"),
                     "lds": lambda: hip.linear_swiglu(x, nxt(), out, kernel="lds"),
                     "blas+swiglu": lambda: hip.swiglu(torch.nn.functional.linear(x, nxt()))}
            for wpb in (4, 7, 8):
                for S in (2, 4, 8, 16):
                    if N % (16 * wpb) == 0 and 32 % S == 0 and (N // (16 * wpb)) * S <= 512:
                        cands["split_w%d_s%d" % (wpb, S)] = (
                            lambda wpb=wpb, S=S: hip.stream_swiglu_split(x, nxt(), out, wpb, S))
            for name, fn in cands.items():
                try:
                    us = timeit(fn)
                except Exception as e:  # noqa: BLE001 -- a shape a kernel does not take
                    print(json.dumps({"op": "gate_up", "kernel": name, "error": str(e)[:80]}))
                    continue
                print(json.dumps({"op": "gate_up", "tp": tp, "M": M, "N": N, "kernel": name, "us": round(us, 2),
                                  "TBps": round(N * K * 2 / us / 1e6, 2), "plan": list(hip.plan("gate_up", M, N, K))}),
                      flush=True)


if __name__ == "__main__":
    main()
