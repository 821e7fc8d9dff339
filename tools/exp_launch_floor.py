#!/usr/bin/env python3
"""Per-launch fixed cost and streaming rate of a dependent kernel chain inside a captured hipGraph (the
decode step's execution model): n back-to-back launches of the HBM streaming probe (csrc/kernels/probe.hip),
each reading its own slice of a 4 GiB buffer (so slices >= 4 MiB are cold: n x slice >> the 256 MiB
Infinity Cache), replayed as one graph.  Fits t(bytes) = t0 + bytes / bw over the slices >= 16 MiB and
prints one JSON line per size plus the fit -- the two constants a decode step's time decomposes into
(docs/decode_latency.md: launches per step x t0 + bytes per step / bw).
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import _lib  # noqa: E402

lib = _lib.kernels_lib()
lib.mrsum_stream_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p]
dev = "cuda:0"
TOTAL = 4 << 30
buf = torch.empty(TOTAL // 2, dtype=torch.bfloat16, device=dev)
buf.normal_()
sink = torch.zeros(65536, dtype=torch.int32, device=dev)
base = buf.data_ptr()


def chain_us(size: int, n: int, blocks: int, reps: int = 20) -> float:
    stream = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        with torch.cuda.graph(g, stream=stream):
            s = torch.cuda.current_stream().cuda_stream
            for i in range(n):
                lib.mrsum_stream_probe(base + (i * size) % (TOTAL - size + 1), size, sink.data_ptr(), blocks, 8, s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * n)


rows = []
for mb in (0.0625, 0.25, 1, 4, 16, 32, 64, 128, 256):
    size = int(mb * (1 << 20))
    n = max(8, min(64, TOTAL // size))
    blocks = max(1, min(4096, size // (256 * 16 * 8)))
    us = chain_us(size, n, blocks)
    rows.append({"MiB": mb, "launches": n, "blocks": blocks, "us_per_launch": round(us, 2),
                 "TBps": round(size / us / 1e6, 2)})
    print(json.dumps(rows[-1]), flush=True)
pts = [(r["MiB"] * (1 << 20), r["us_per_launch"]) for r in rows if r["MiB"] >= 16]
mx = sum(p[0] for p in pts) / len(pts)
my = sum(p[1] for p in pts) / len(pts)
slope = sum((x - mx) * (y - my) for x, y in pts) / sum((x - mx) ** 2 for x, _ in pts)
t0 = my - slope * mx
print(json.dumps({"fit": "t = t0 + bytes / bw over slices >= 16 MiB", "t0_us": round(t0, 2),
                  "bw_TBps": round(1e-6 / slope, 2) if slope > 0 else None,
                  "smallest_launch_us": rows[0]["us_per_launch"]}), flush=True)
