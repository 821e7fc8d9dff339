#!/usr/bin/env python3
"""A few prefill GEMM launches for rocprofv3 --pmc passes (tools/gpu_r3_pmc_gemm.sh): Llama-3-8B o
(4096 x 4096) and gate_up + SwiGLU (28672 x 4096) at M = 16384 in bf16, each on the 16x16 and the 32x32
MFMA tiles, and the 70B fp8 gate_up + SwiGLU at M = 8192 on both tile shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llm_map_reduce_summarizer_amd.ops import hip
    from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight
    dev = "cuda:0"
    bf = dict(dtype=torch.bfloat16, device=dev)
    x = torch.randn(16384, 4096, **bf)
    wo = torch.randn(4096, 4096, **bf) * 0.02
    wgu = torch.randn(28672, 4096, **bf) * 0.02
    for gm in (4, 4 | 256):
        for _ in range(2):
            hip.gemm(x, wo, group_m=gm)
            hip.gemm(x, wgu, swiglu=True, group_m=gm)
    w8 = Fp8Weight.quantize(torch.randn(57344, 8192, **bf) * 0.02)
    xq, xs = hip.quant_fp8_rows(torch.randn(8192, 8192, **bf))
    for gm in (4, 4 | 256):
        for _ in range(2):
            hip.gemm_fp8(xq, xs, w8, swiglu=True, group_m=gm)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
