#!/usr/bin/env python3
"""Back-to-back (graph-like) per-kernel cost of streaming X MB: probe vs decode GEMMs.
Rotates over enough weight copies that nothing stays in the 256 MiB Infinity Cache."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import _lib, hip  # noqa: E402

lib = _lib.kernels_lib()
lib.mrsum_stream_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p]


def b2b(fn, n=60):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e-3 / n


dev = "cuda:0"
sink = torch.zeros(65536, dtype=torch.int32, device=dev)
out = []
for name, (N, K) in {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336), "gate_up": (28672, 4096)}.items():
    ncopy = max(2, int(1.2e9 // (N * K * 2)))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
    nb = N * K * 2
    it = [0]

    def nxt():
        it[0] += 1
        return ws[it[0] % ncopy]

    for blocks in (4096,):
        for unroll in (8,):
            t = b2b(lambda: lib.mrsum_stream_probe(nxt().data_ptr(), nb, sink.data_ptr(), blocks, unroll,
                                                   torch.cuda.current_stream().cuda_stream))
            out.append({"op": name, "kind": "probe", "blocks": blocks, "unroll": unroll, "us": round(t * 1e6, 1),
                        "TBps": round(nb / t / 1e12, 2)})
    for M in (int(m) for m in os.environ.get("MS", "1,4,16,48").split(",")):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        for nt in (1, 2):
            for splits in (1, 2, 4, 8):
                if (K // 128) % splits:
                    continue
                o = torch.empty(splits, M, N, dtype=torch.float32, device=dev)
                t = b2b(lambda: hip._skinny(x, nxt(), o, hip.EPI_F32_PARTIAL, nt, splits, N))
                out.append({"op": name, "kind": "skinny", "M": M, "nt": nt, "S": splits, "us": round(t * 1e6, 1),
                            "TBps": round(nb / t / 1e12, 2)})
        for splits in (1, 2, 4, 8, 16):
            if (K // 128) % splits:
                continue
            o = torch.empty(splits, M, N, dtype=torch.float32, device=dev)
            for depth in (1, 2):
                t = b2b(lambda: hip._skinny_lds(x, nxt(), o, hip.EPI_F32_PARTIAL, splits, N, depth))
                out.append({"op": name, "kind": "lds", "M": M, "depth": depth, "S": splits,
                            "us": round(t * 1e6, 1), "TBps": round(nb / t / 1e12, 2)})
        if name == "gate_up":
            o = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
            for depth in (1, 2):
                t = b2b(lambda: hip._skinny_lds(x, nxt(), o, hip.EPI_SWIGLU, 1, N // 2, depth))
                out.append({"op": name, "kind": "lds_swiglu", "M": M, "depth": depth, "us": round(t * 1e6, 1),
                            "TBps": round(nb / t / 1e12, 2)})
            t = b2b(lambda: hip._skinny(x, nxt(), o, hip.EPI_SWIGLU, 1, 1, N // 2))
            out.append({"op": name, "kind": "skinny_swiglu", "M": M, "us": round(t * 1e6, 1),
                        "TBps": round(nb / t / 1e12, 2)})
        t = b2b(lambda: torch.nn.functional.linear(x, nxt()))
        out.append({"op": name, "kind": "hipblaslt", "M": M, "us": round(t * 1e6, 1), "TBps": round(nb / t / 1e12, 2)})
    del ws
    torch.cuda.empty_cache()
for r in out:
    print(json.dumps(r))
