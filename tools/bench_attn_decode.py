#!/usr/bin/env python3
"""Decode attention micro-benchmark: achieved KV bandwidth of the MFMA paged decode kernel per
(batch, splits, fused merge, nontemporal policy), rotating over LAYERS distinct KV caches so every call
streams from HBM (a decode step reads each layer's cache once; a repeated single cache would sit in the
256 MiB Infinity Cache).  Interleaved rounds in one process; JSON lines.

    python tools/bench_attn_decode.py [--batches 1,10,39] [--ctx 4000] [--splits auto,4,8,16]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,10,39")
    ap.add_argument("--ctx", type=int, default=4000)
    ap.add_argument("--splits", default="auto")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--hkv", type=int, default=8, help="kv heads (q heads = 4 x): 8 = TP=1, 2 / 1 = TP=4 / 8 shard")
    a = ap.parse_args()
    dev = "cuda:0"
    hkv, d, page = a.hkv, 128, 64
    hq = 4 * hkv
    for B in (int(b) for b in a.batches.split(",")):
        ctx = a.ctx
        npg = -(-ctx // page)
        caches = []
        for _ in range(a.layers):
            kc = torch.randn(B * npg + 1, hkv, page, d, device=dev, dtype=torch.bfloat16)
            caches.append((kc, torch.randn_like(kc)))
        bt = (torch.arange(B * npg, dtype=torch.int32, device=dev).view(B, npg) + 1)
        pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=dev)
        q = torch.randn(B, hq * d, device=dev, dtype=torch.bfloat16)
        auto_s, auto_f = hip.decode_attn_plan(B, hkv, ctx)
        variants = []
        for sp in a.splits.split(","):
            s = auto_s if sp == "auto" else int(sp)
            for fused in ([auto_f] if sp == "auto" else [False, True]):
                if fused and s > 32:
                    continue
                variants.append((sp, s, fused, hip.DecodeWorkspace(B, hq, d, s, dev, hkv, fused_combine=fused)))
        gb = B * ctx * hkv * d * 2 * 2 / 1e9
        res = {v[:3]: [] for v in variants}
        for _ in range(a.rounds):
            for sp, s, fused, ws in variants:
                for i in range(a.layers):  # warm
                    hip.attn_decode(q, caches[i][0], caches[i][1], bt, pos, hq, hkv, d, page, 1 / math.sqrt(d),
                                    workspace=ws)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(a.iters):
                    kc, vc = caches[i % a.layers]
                    hip.attn_decode(q, kc, vc, bt, pos, hq, hkv, d, page, 1 / math.sqrt(d), workspace=ws)
                e1.record()
                e1.synchronize()
                res[(sp, s, fused)].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        for (sp, s, fused), ts in res.items():
            ts.sort()
            us = ts[len(ts) // 2]
            print(json.dumps({"B": B, "hkv": hkv, "ctx": ctx, "splits": s, "plan": sp, "fused": fused, "us": round(us, 2),
                              "TBps": round(gb / us * 1e6 / 1e3, 2)}), flush=True)
        del caches


if __name__ == "__main__":
    main()
