#!/usr/bin/env python3
"""Does the decode GEMM's weight-tile read order cost HBM bandwidth?  Graph-captured chains of the
row-pattern probe (csrc/kernels/probe.hip stream_probe_rows_kernel) over cold weight-shaped buffers: one
workgroup per block of R rows, the block read C bytes per row per slot (C = 256: the stream GEMM's
128-wide bf16 k block) up to C = row_bytes (the block as one contiguous range), against the plain
grid-stride probe of the same bytes."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import _lib  # noqa: E402

lib = _lib.kernels_lib()
vp, ci = ctypes.c_void_p, ctypes.c_int
lib.mrsum_stream_probe.argtypes = [vp, ctypes.c_size_t, vp, ci, ci, vp]
lib.mrsum_stream_probe_rows.argtypes = [vp, ci, ci, ci, ci, ci, vp, vp]
dev = "cuda:0"
sink = torch.zeros(65536, dtype=torch.int32, device=dev)


def chain_us(launch, n=16, reps=10):
    st = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            s = torch.cuda.current_stream().cuda_stream
            for i in range(n):
                rc = launch(i, s)
                assert rc == 0, rc
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * n)


for name, rows, row_bytes in (("gate_up", 28672, 8192), ("down", 4096, 28672), ("lm_head", 128256 // 8 * 8, 8192)):
    nbytes = rows * row_bytes
    ncopy = max(2, int(2.2e9 // nbytes))
    ws = [torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev).normal_() for _ in range(ncopy)]
    res = []
    us = chain_us(lambda i, s: lib.mrsum_stream_probe(ws[i % ncopy].data_ptr(), nbytes, sink.data_ptr(), 4096, 8, s))
    res.append({"shape": name, "MB": round(nbytes / 1e6, 1), "kind": "grid_stride", "us": round(us, 2),
                "TBps": round(nbytes / us / 1e6, 2)})
    for R, thr in ((112, 512), (64, 512), (16, 256)):
        if rows % R:
            continue
        for C in (256, 512, 1024, 2048, row_bytes):
            if row_bytes % C:
                continue
            us = chain_us(lambda i, s: lib.mrsum_stream_probe_rows(ws[i % ncopy].data_ptr(), rows, row_bytes, R, C, thr,
                                                                   sink.data_ptr(), s))
            res.append({"shape": name, "MB": round(nbytes / 1e6, 1), "kind": "rows", "R": R, "C": C, "threads": thr,
                        "grid": rows // R, "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 2)})
    for r in res:
        print(json.dumps(r), flush=True)
    del ws
    torch.cuda.empty_cache()
