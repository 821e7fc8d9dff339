#!/usr/bin/env python3
"""Decode LM head ([M, 4096] x [128256, 4096]^T bf16) on the stream GEMM at every workgroup width that
divides the vocabulary (wpb 4 / 6 / 8 -> 2004 / 1336 / 1002 column tiles), back-to-back over two weight
copies beyond the Infinity Cache.  JSON line per (M, wpb) with us and TB/s; the plan's choice is marked."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llm_map_reduce_summarizer_amd.ops import hip
    dev = "cuda:0"
    N, K = 128256, 4096
    ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(2)]
    plan = hip.stream_config(N, K, splits=1)
    for M in (1, 10, 39):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        for wpb in (4, 6, 8):
            if N % (16 * wpb):
                continue
            best = 1e9
            for _ in range(3):
                for i in range(4):
                    hip._stream_gemm(x, ws[i % 2], out, hip.EPI_BF16, 1, N, wpb)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for i in range(20):
                    hip._stream_gemm(x, ws[i % 2], out, hip.EPI_BF16, 1, N, wpb)
                e.record()
                e.synchronize()
                best = min(best, s.elapsed_time(e) * 1e3 / 20)
            print(json.dumps({"M": M, "wpb": wpb, "tiles": N // (16 * wpb), "plan": plan is not None and plan[0] == wpb,
                              "us": round(best, 1), "TBps": round(N * K * 2 / best / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
