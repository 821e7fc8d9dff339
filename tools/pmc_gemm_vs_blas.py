#!/usr/bin/env python3
"""Prefill GEMM launches for rocprofv3 --pmc passes: gemm.hip (8 waves) and gemm4w.hip against hipBLASLt
(torch.matmul) on the Llama-3-8B o (4096 x 4096) and gate_up (28672 x 4096) projections at M = 16384, bf16,
uniform random operands."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llm_map_reduce_summarizer_amd.ops import hip
    dev = "cuda:0"
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.rand(16384, 4096, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    for N in (4096, 28672):
        w = ((torch.rand(N, 4096, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16).to(dev)
        for _ in range(3):
            hip.gemm(x, w, kernel="8w")
            hip.gemm(x, w, kernel="4w")
            torch.matmul(x, w.t())
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
