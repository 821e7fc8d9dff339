#!/usr/bin/env python3
"""hipBLASLt's kernel choice (Tensile kernel names encode macro tile, MFMA shape, wave layout, depth U,
LDS buffering) for the four Llama-3-8B prefill projections at M = 16384, to run under
``rocprofv3 --kernel-trace --stats``; also times each against gemm.hip."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llm_map_reduce_summarizer_amd.ops import hip
    dev = torch.device("cuda:0")
    M = 16384
    for role, (N, K) in {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
                         "down": (4096, 14336)}.items():
        g = torch.Generator(device="cpu").manual_seed(1)
        x = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16).to(dev)
        for _ in range(5):
            torch.matmul(x, w.t())
            hip.gemm(x, w)
        torch.cuda.synchronize()
        print(role, "done", flush=True)


if __name__ == "__main__":
    main()
