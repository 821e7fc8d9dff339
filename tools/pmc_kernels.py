#!/usr/bin/env python3
"""A lean, graph-free set of kernel launches for rocprofv3 --pmc passes (tools/gpu_pmc.sh): the
Llama-3-8B decode GEMMs at M=1 and M=39 (our LDS-DMA stream kernel, fused epilogues), paged decode
attention at B=1/39 x 4k context, the prefill flash attention on 4 x 4k tokens and the prefill GEMMs
(bf16 at M = 16384, fp8 at a 70B shape).  Few dispatches,
so the per-dispatch counter serialisation stays cheap."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from llm_map_reduce_summarizer_amd import ops
    from llm_map_reduce_summarizer_amd.ops import hip, reference
    dev = "cuda:0"
    bf = dict(dtype=torch.bfloat16, device=dev)
    hid, ffn, hd = 4096, 14336, 128
    W = {"qkv": torch.randn(6144, hid, **bf) * 0.02, "o": torch.randn(hid, hid, **bf) * 0.02,
         "gate_up": torch.randn(2 * ffn, hid, **bf) * 0.02, "down": torch.randn(hid, ffn, **bf) * 0.02}
    for M in (1, 39):
        x = torch.randn(M, hid, **bf)
        xf = torch.randn(M, ffn, **bf)
        for _ in range(3):
            for role in ("qkv", "o", "down"):
                w = W[role]
                a = xf if role == "down" else x
                p = hip.plan(role, M, w.shape[0], w.shape[1])
                ops._plan_parts(hip, p, a, w, None)
            ops.gate_up_swiglu(x, W["gate_up"])
    # decode attention, 4k context
    page, n_pages = 64, 64 * 40 + 1
    kc = torch.randn(n_pages, 8, page, hd, **bf)
    vc = torch.randn(n_pages, 8, page, hd, **bf)
    for B in (1, 39):
        bt = (1 + torch.arange(B * 64, dtype=torch.int32, device=dev).view(B, 64) % (n_pages - 1))
        pos = torch.full((B,), 4095, dtype=torch.int32, device=dev)
        q = torch.randn(B, 48 * hd, **bf)
        S, fused = hip.decode_attn_plan(B, 8, 64 * page)  # the engine's plan for this batch / context
        ws = hip.DecodeWorkspace(B, 32, hd, S, dev, 8, fused_combine=fused)
        for _ in range(3):
            hip.attn_decode(q, kc, vc, bt, pos, 32, 8, hd, page, 1 / math.sqrt(hd), workspace=ws)
    # prefill attention: 4 sequences x 4096 tokens
    lens = [4096] * 4
    qkv = torch.randn(sum(lens), 48 * hd, **bf)
    cu = torch.tensor([0, 4096, 8192, 12288, 16384], dtype=torch.int32, device=dev)
    items = hip.prefill_items(lens, 4).to(dev)
    for _ in range(3):
        hip.attn_prefill(qkv, cu, 32, 8, hd, 1 / math.sqrt(hd), seqlens=lens, items=items)
    # prefill GEMMs (gemm.hip, 256 x 256 tiles): bf16 qkv / gate_up + SwiGLU at M = 16384, fp8 gate_up at
    # a Llama-3-70B shape (M = 8192)
    xp = torch.randn(16384, hid, **bf)
    for _ in range(2):
        hip.gemm(xp, W["qkv"])
        ops.linear_swiglu(xp, W["gate_up"])
    w8 = reference.Fp8Weight.quantize(torch.randn(2 * 28672, 8192, **bf) * 0.02)
    x8 = torch.randn(8192, 8192, **bf)
    for _ in range(2):
        hip.fp8_linear(x8, w8, swiglu=True)
    torch.cuda.synchronize()
    print("pmc kernels done", flush=True)


if __name__ == "__main__":
    main()
