#!/usr/bin/env python3
"""fp8 stream GEMM (70B down, M=1, wpb 8, split 4) next to the bf16 stream GEMM on a same-byte shape
(8192 x 14336 bf16) for rocprofv3 --pmc passes: 20 launches each over weight copies beyond the MALL."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402
from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight  # noqa: E402

dev = "cuda:0"
N, K8, K16 = 8192, 28672, 14336
w8 = [Fp8Weight.quantize(torch.randn(N, K8, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(5)]
w16 = [torch.randn(N, K16, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(5)]
x8 = torch.randn(1, K8, device=dev, dtype=torch.bfloat16)
x16 = torch.randn(1, K16, device=dev, dtype=torch.bfloat16)
o = torch.empty(4, 1, N, dtype=torch.float32, device=dev)
for i in range(20):
    hip._stream_fp8(x8, w8[i % 5], o, hip.EPI_F32_PARTIAL, 4, N, 8)
for i in range(20):
    hip._stream_gemm(x16, w16[i % 5], o, hip.EPI_F32_PARTIAL, 4, N, 8)
torch.cuda.synchronize()
print("ok")
