#!/usr/bin/env python3
"""Do parallel branches of a captured hipGraph run concurrently on this chip?  A decode step is one dependent
chain of latency-bound launches (a TP shard's layer: six kernels of 2-30 MB, each paying the graph boundary,
its first-byte latency and its drain); two INDEPENDENT chains (e.g. two micro-batches) on two branches of
one graph could fill each other's gaps -- if the runtime dispatches the branches to separate hardware queues.

For chains of n launches of the HBM streaming probe (csrc/kernels/probe.hip) at a few sizes / grid widths:
  serial  -- 2n launches on one stream;
  branch2 -- n launches on each of two branches forked from and joined into the capture stream.
One JSON line per size: microseconds per replay for both and their ratio (0.5 = the branches fully overlap,
1.0 = serialised).  Slices rotate over a 4 GiB buffer (cold beyond the 256 MiB Infinity Cache).
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


def launch(i, size, blocks):
    s = torch.cuda.current_stream().cuda_stream
    lib.mrsum_stream_probe(base + (i * size) % (TOTAL - size + 1), size, sink.data_ptr(), blocks, 8, s)


def timed(g, reps=20):
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def graph(size, blocks, n, branches):
    s0 = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(branches)]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s0):
        with torch.cuda.graph(g, stream=s0):
            if branches == 1:
                for i in range(2 * n):
                    launch(i, size, blocks)
            else:
                ev = torch.cuda.Event()
                ev.record(s0)
                for b, st in enumerate(side):
                    st.wait_event(ev)
                    with torch.cuda.stream(st):
                        for i in range(2 * n // branches):
                            launch(b * n + i, size, blocks)
                for st in side:
                    s0.wait_stream(st)
    return g


for mb, blocks in ((0.25, 16), (2, 64), (8, 128), (32, 256), (32, 1024)):
    size = int(mb * (1 << 20))
    n = 32
    t1 = timed(graph(size, blocks, n, 1))
    t2 = timed(graph(size, blocks, n, 2))
    t4 = timed(graph(size, blocks, n, 4))
    print(json.dumps({"MiB": mb, "blocks": blocks, "launches": 2 * n, "serial_us": round(t1, 1),
                      "branch2_us": round(t2, 1), "branch4_us": round(t4, 1), "ratio2": round(t2 / t1, 3),
                      "ratio4": round(t4 / t1, 3)}), flush=True)
