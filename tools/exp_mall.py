#!/usr/bin/env python3
"""Does the 256 MiB Infinity Cache (MALL) hold decode weights between kernels?

1. warm vs cold streaming: the same buffer read back-to-back (warm) vs rotating copies (cold).
2. side-stream prefetch: main stream runs a chain of tiny dependent kernels (the attention /
   norm phase of a B=1 decode layer) then the o-projection GEMM; a side stream concurrently
   streams the GEMM's weights with a few workgroups.  Reports per-iteration time with/without.
"""
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
dev = "cuda:0"
sink = torch.zeros(65536, dtype=torch.int32, device=dev)


def probe(t, blocks=4096, stream=None):
    s = (stream or torch.cuda.current_stream()).cuda_stream
    lib.mrsum_stream_probe(t.data_ptr(), t.numel() * t.element_size(), sink.data_ptr(), blocks, 8, s)


def timed(fn, n=40):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n):
        fn(i)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / n


out = []
for mb in (16, 32, 64, 117, 160, 200, 300):
    n = mb * (1 << 20) // 2
    ncopy = max(2, int(2e9 // (n * 2)))
    ws = [torch.randn(n, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
    cold = timed(lambda i: probe(ws[i % ncopy]))
    warm = timed(lambda i: probe(ws[0]))
    out.append({"test": "stream", "MB": mb, "cold_us": round(cold, 1), "warm_us": round(warm, 1),
                "cold_TBps": round(n * 2 / cold / 1e6, 2), "warm_TBps": round(n * 2 / warm / 1e6, 2)})
    del ws
    torch.cuda.empty_cache()

# skinny GEMMs warm vs cold at M=1
for name, (N, K, S) in {"o": (4096, 4096, 2), "gate_up": (28672, 4096, 1), "down": (4096, 14336, 2)}.items():
    ncopy = max(2, int(2e9 // (N * K * 2)))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
    x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
    o = torch.empty(S, 1, N, dtype=torch.float32, device=dev)
    nt = 2 if name != "gate_up" else 1
    cold = timed(lambda i: hip._skinny(x, ws[i % ncopy], o, hip.EPI_F32_PARTIAL, nt, S, N))
    warm = timed(lambda i: hip._skinny(x, ws[0], o, hip.EPI_F32_PARTIAL, nt, S, N))
    out.append({"test": "skinny_m1", "op": name, "cold_us": round(cold, 1), "warm_us": round(warm, 1)})

    # side-stream prefetch while a chain of 6 tiny dependent kernels runs on the main stream
    side = torch.cuda.Stream()
    h = torch.randn(1, 4096, device=dev, dtype=torch.bfloat16)
    lnw = torch.ones(4096, device=dev, dtype=torch.bfloat16)

    def step(i, pf_blocks):
        w = ws[i % ncopy]
        main = torch.cuda.current_stream()
        if pf_blocks:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                probe(w, pf_blocks, side)
        for _ in range(6):
            hip.rmsnorm(h, lnw, 1e-5, out=h)
        hip._skinny(x, w, o, hip.EPI_F32_PARTIAL, nt, S, N)
        if pf_blocks:
            main.wait_stream(side)

    base = timed(lambda i: step(i, 0))
    for pfb in (32, 64, 128, 256):
        t = timed(lambda i: step(i, pfb))
        out.append({"test": "prefetch", "op": name, "pf_blocks": pfb, "base_us": round(base, 1), "us": round(t, 1)})
    tiny = timed(lambda i: [hip.rmsnorm(h, lnw, 1e-5, out=h) for _ in range(6)])
    out.append({"test": "tiny_chain", "us": round(tiny, 1)})
    del ws
    torch.cuda.empty_cache()
for r in out:
    print(json.dumps(r))
