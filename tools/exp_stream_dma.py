#!/usr/bin/env python3
"""How much of the decode stream GEMM's time is the LDS-DMA weight stream itself?  Back-to-back launches
over weight copies beyond the 256 MiB Infinity Cache (graph-like), per shape:

  * ``gemm``   -- the production stream GEMM at its plan (ops/hip.py), M = 1 and 40 rows
  * ``dma``    -- tools/diag_stream_dma.hip: the same workgroups, tile and DMA pieces, no compute (MODE 0: the
                  GEMM's loop with its barrier; 1: no barrier; 2: refill before the wait, one slot deeper)
  * ``probe``  -- the grid-stride register-load probe (probe.hip), the calibration of docs/decode_latency.md

    python tools/exp_stream_dma.py --build     # here (hipcc): _native/diag/libmrsum_stream_dma_diag.so
    python tools/exp_stream_dma.py             # GPU: one JSON line per case
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "llm_map_reduce_summarizer_amd", "_native", "diag", "libmrsum_stream_dma_diag.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           os.path.join(ROOT, "tools", "diag_stream_dma.hip"), "-o", LIB])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    if a.build:
        return build()
    import torch
    from llm_map_reduce_summarizer_amd.ops import _lib, hip

    dev = "cuda:0"
    diag = ctypes.CDLL(LIB)
    diag.diag_dma_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib = _lib.kernels_lib()
    lib.mrsum_stream_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p]
    sink = torch.zeros(1 << 20, dtype=torch.int32, device=dev)

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

    shapes = {"gate_up": (28672, 4096), "down": (4096, 14336), "qkv": (6144, 4096)}
    for rep in range(a.reps):
        for name, (N, K) in shapes.items():
            nb = N * K * 2
            ncopy = max(2, int(1.2e9 // nb))
            ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
            it = [0]

            def nxt():
                it[0] += 1
                return ws[it[0] % ncopy]

            def emit(**kw):
                t = kw.pop("t")
                print(json.dumps(dict(rep=rep, op=name, **kw, us=round(t * 1e6, 2), TBps=round(nb / t / 1e12, 3))),
                      flush=True)

            stream = torch.cuda.current_stream().cuda_stream
            emit(kind="probe", t=b2b(lambda: lib.mrsum_stream_probe(nxt().data_ptr(), nb, sink.data_ptr(), 4096, 8,
                                                                    stream)))
            plan = hip.plan(name, 1, N, K)
            _, wpb, S = plan
            for M in (1, 40):
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                if name == "gate_up":
                    o = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                    fn = lambda: hip._stream_gemm(x, nxt(), o, hip.EPI_SWIGLU, 1, N // 2, wpb)  # noqa: E731
                else:
                    o = torch.empty(S, M, N, device=dev, dtype=torch.float32)
                    fn = lambda: hip._stream_gemm(x, nxt(), o, hip.EPI_F32_PARTIAL, S, N, wpb)  # noqa: E731
                emit(kind="gemm", M=M, wpb=wpb, S=S, t=b2b(fn))
            for dwpb, depths in ((7, (3, 4, 5)), (4, (4, 6, 8))):
                if N % (16 * dwpb):
                    continue
                splits = S if dwpb == wpb else max(1, (256 * 16 * dwpb) // N)
                if K % (128 * splits):
                    continue
                for d in depths:
                    for mode in (0, 1, 2):
                        def run():
                            rc = diag.diag_dma_probe(nxt().data_ptr(), N, K, splits, dwpb, d, mode, sink.data_ptr(),
                                                     stream)
                            assert rc == 0, rc
                        emit(kind="dma", wpb=dwpb, S=splits, depth=d, mode=mode, t=b2b(run))
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
