#!/usr/bin/env python3
"""Prefill flash-attention throughput (causal, GQA 32:8, d=128, random data), contiguous packed rows and
the paged (chunked-prefill) variant; imports the package from the CURRENT directory, so the same script
A/B-tests two trees on one box (cd <tree> && python <this script>).  JSON line per case: ms, TFLOP/s.

    python tools/bench_attn_prefill.py [--cases 1x4096,8x4096,39x4000,1x32768]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from llm_map_reduce_summarizer_amd import ops  # noqa: E402
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="1x4096,8x4096,39x4000,1x32768")
    ap.add_argument("--tag", default=os.path.basename(os.getcwd()))
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--prefix", type=int, default=0, help="paged case: cached tokens before each slice")
    a = ap.parse_args()
    dev, hq, hkv, d = "cuda:0", a.hq, a.hkv, 128
    torch.manual_seed(0)
    for case in a.cases.split(","):
        nseq, L = (int(v) for v in case.split("x"))
        T = nseq * L
        qkv = torch.randn(T, (hq + 2 * hkv) * d, device=dev, dtype=torch.bfloat16)
        cu = torch.arange(0, T + 1, L, dtype=torch.int32, device=dev)
        # trees before the GQA-packed kernel take 256-row blocks of one head
        items = (hip.prefill_items([L] * nseq, hq // hkv) if hasattr(hip, "prefill_block_m")
                 else hip.prefill_items([L] * nseq)).to(dev)
        fl = nseq * 4 * L * L / 2 * d * hq
        ms = timeit(lambda: hip.attn_prefill(qkv, cu, hq, hkv, d, 1 / math.sqrt(d), items=items, seqlens=[L] * nseq))
        print(json.dumps({"tree": a.tag, "kind": "contiguous", "hq": hq, "hkv": hkv, "nseq": nseq, "L": L, "ms": round(ms, 3),
                          "TFLOPs": round(fl / ms / 1e9, 1)}), flush=True)
        # paged: the same keys from a page cache (``--prefix`` cached tokens before each slice), pages shuffled
        P = a.prefix
        npg = -(-(P + L) // 64)
        kc = torch.randn(nseq * npg + 1, hkv, 64, d, device=dev, dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = (torch.randperm(nseq * npg, device=dev).to(torch.int32) + 1).view(nseq, npg)
        pp = ops.PagedPrefill(bt, torch.arange(nseq, dtype=torch.int32, device=dev),
                              torch.full((nseq,), P, dtype=torch.int32, device=dev), list(range(nseq)), [P] * nseq,
                              kc, vc)
        ms = timeit(lambda: hip.attn_prefill(qkv, cu, hq, hkv, d, 1 / math.sqrt(d), items=items, seqlens=[L] * nseq,
                                             paged=pp))
        flp = nseq * 4 * (P * L + L * L / 2) * d * hq
        print(json.dumps({"tree": a.tag, "kind": "paged", "hq": hq, "hkv": hkv, "nseq": nseq, "L": L, "prefix": P,
                          "ms": round(ms, 3), "TFLOPs": round(flp / ms / 1e9, 1)}), flush=True)
        del qkv, kc, vc


if __name__ == "__main__":
    main()
