#!/usr/bin/env python3
"""Post-attention decode layer, Llama-3-8B shapes: the persistent one-launch kernel (decode_layer.hip)
vs the four stream-GEMM launches it replaces (o + residual, gate_up + SwiGLU, down + residual, next QKV;
deferred RMSNorm in both), each captured as a hipGraph over LAYERS distinct weight sets (weights stream
from HBM as in a real step), interleaved rounds in one process.  JSON line per (M, path): us per layer.

    python tools/bench_decode_layer.py [--ms 1,5,10,16] [--layers 6]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from llm_map_reduce_summarizer_amd import ops  # noqa: E402
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,5,10,16")
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = "cuda:0"
    torch.manual_seed(0)
    L = a.layers
    W = [{"wo": torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16) * 0.02,
          "wgu": torch.randn(28672, 4096, device=dev, dtype=torch.bfloat16) * 0.02,
          "wd": torch.randn(4096, 14336, device=dev, dtype=torch.bfloat16) * 0.02,
          "wqkv": torch.randn(6144, 4096, device=dev, dtype=torch.bfloat16) * 0.02} for _ in range(L)]
    eps = 1e-5
    for M in (int(m) for m in a.ms.split(",")):
        att = torch.randn(M, 4096, device=dev, dtype=torch.bfloat16)
        res = torch.randn(M, 4096, device=dev, dtype=torch.bfloat16)

        def persistent():
            for w in W:
                hip.decode_layer(att, w["wo"], w["wgu"], w["wd"], w["wqkv"], res, eps)

        def launches():
            p = hip.plan("qkv", M, 6144, 4096)
            for w in W:
                nr = ops.proj_add_rmsnorm(att, w["wo"], res, None, eps, "o")
                act = ops.gate_up_swiglu(nr, w["wgu"])
                nr2 = ops.proj_add_rmsnorm(act, w["wd"], res, None, eps, "down")
                hip.linear_parts(nr2.h, w["wqkv"], p[2], nt=p[1], kernel="stream", norm=nr2.norm)

        graphs = {}
        for name, fn in (("persistent", persistent), ("launches", launches)):
            fn()  # scratch / tickets before capture
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            graphs[name] = g
        times = {k: [] for k in graphs}
        for _ in range(a.rounds):
            for name, g in graphs.items():
                g.replay()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    g.replay()
                e.record()
                e.synchronize()
                times[name].append(s.elapsed_time(e) * 1e3 / (a.reps * L))
        for name, ts in times.items():
            ts.sort()
            print(json.dumps({"M": M, "path": name, "us_per_layer": round(ts[len(ts) // 2], 2),
                              "us_min": round(ts[0], 2)}), flush=True)
        assert hip.decode_layer_error() == 0


if __name__ == "__main__":
    main()
