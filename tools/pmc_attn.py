#!/usr/bin/env python3
"""Prefill attention only (for rocprofv3 --pmc passes): 8 x 4096 (Llama-3-8B heads) and 1 x 32768 (70B heads),
3 launches each, random data."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402

dev, d = "cuda:0", 128
for nseq, L, hq, hkv in ((8, 4096, 32, 8), (1, 32768, 64, 8)):
    T = nseq * L
    qkv = torch.randn(T, (hq + 2 * hkv) * d, device=dev, dtype=torch.bfloat16)
    cu = torch.arange(0, T + 1, L, dtype=torch.int32, device=dev)
    items = hip.prefill_items([L] * nseq, hq // hkv).to(dev)
    for _ in range(3):
        hip.attn_prefill(qkv, cu, hq, hkv, d, 1 / math.sqrt(d), items=items, seqlens=[L] * nseq)
    torch.cuda.synchronize()
print("ok")
