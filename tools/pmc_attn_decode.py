#!/usr/bin/env python3
"""Decode attention only (for rocprofv3 --pmc passes): B=1 at 13.5k (8 kv heads, 32 separate splits, the
headline's final reduce) and B=39 at 4.4k (4 splits, the map), 8 distinct caches each so every launch streams
from HBM; a few launches per case.  Kernel names separate the cases by their grid (summary by dispatch)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402

dev, d, page, hkv = "cuda:0", 128, 64, 8
hq = 4 * hkv
for B, ctx, S in ((1, 13500, 32), (39, 4400, 4)):
    npg = -(-ctx // page)
    caches = [(torch.randn(B * npg + 1, hkv, page, d, device=dev, dtype=torch.bfloat16),
               torch.randn(B * npg + 1, hkv, page, d, device=dev, dtype=torch.bfloat16)) for _ in range(8)]
    bt = torch.arange(B * npg, dtype=torch.int32, device=dev).view(B, npg) + 1
    pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=dev)
    q = torch.randn(B, hq * d, device=dev, dtype=torch.bfloat16)
    ws = hip.DecodeWorkspace(B, hq, d, S, dev, hkv)
    for i in range(16):
        kc, vc = caches[i % 8]
        hip.attn_decode(q, kc, vc, bt, pos, hq, hkv, d, page, 1 / math.sqrt(d), workspace=ws)
    torch.cuda.synchronize()
    del caches
print("ok")
