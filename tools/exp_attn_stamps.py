#!/usr/bin/env python3
"""Where a decode-attention workgroup's time goes: csrc/kernels/attn_decode.hip built with -DMRSUM_ATTN_STAMPS
(s_memtime deltas per phase, every wave: prologue, tile compute, barrier after compute, next tile's LDS write +
load issue, barrier after the write, epilogue incl. partial stores and the fused merge) into
_native/diag/libmrsum_attn_stamps.so, run on the decode shapes of the headline's phases, averaged per phase over
every wave of every workgroup with tiles.

    python tools/exp_attn_stamps.py --build        # here (hipcc)
    python tools/exp_attn_stamps.py                # on the GPU box

One JSON line per case: kernel wall us (events, the stamped build), mean shader cycles per phase, and cycles per
tile of the three loop phases.
"""
import argparse
import ctypes
import json
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KDIR = os.path.join(ROOT, "llm_map_reduce_summarizer_amd", "csrc", "kernels")
LIB = os.path.join(ROOT, "llm_map_reduce_summarizer_amd", "_native", "diag", "libmrsum_attn_stamps.so")
PHASES = ("prologue", "compute", "barrier_after_compute", "write_issue", "barrier_after_write", "epilogue")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-ffp-contract=fast", "-munsafe-fp-atomics", "-DMRSUM_ATTN_STAMPS", "-I", KDIR,
                           os.path.join(KDIR, "attn_decode.hip"), "-o", LIB])
    print("built", LIB)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--iters", type=int, default=16)
    a = ap.parse_args()
    if a.build:
        return build()
    import torch
    lib = ctypes.CDLL(LIB)
    vp, ci = ctypes.c_void_p, ctypes.c_int
    lib.mrsum_attn_set_stamps.argtypes = [vp]
    lib.mrsum_attn_decode_mfma.argtypes = [vp, ci, vp, vp, vp, ci, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci, ci,
                                           ctypes.c_float, vp, ci, vp]
    dev = "cuda:0"
    d, page = 128, 64
    # (name, B, hq, hkv, ctx, splits, fused): the headline's map (B=39), level-1 (B=10) and final (B=1) shapes
    # with their plans, and a Llama-3-8B TP=8 shard at B=1.  (A 512-thread specialised-wave variant -- 4 scoring
    # + 4 staging waves, two LDS tile buffers -- was stamped here too and removed: profiles/r6_attn_stamps.jsonl.)
    cases = [("map_b39", 39, 32, 8, 4400, 4, False), ("l1_b10", 10, 32, 8, 4800, 3, True),
             ("l1_b10_sep6", 10, 32, 8, 4800, 6, False), ("final_b1", 1, 32, 8, 13000, 32, False),
             ("tp8_b1", 1, 4, 1, 4000, 63, False)]
    for name, B, hq, hkv, ctx, S, fused in cases:
        npg = -(-ctx // page)
        layers = 8
        caches = [(torch.randn(B * npg + 1, hkv, page, d, device=dev, dtype=torch.bfloat16),
                   torch.randn(B * npg + 1, hkv, page, d, device=dev, dtype=torch.bfloat16)) for _ in range(layers)]
        bt = (torch.arange(B * npg, dtype=torch.int32, device=dev).view(B, npg) + 1)
        pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=dev)
        q = torch.randn(B, hq * d, device=dev, dtype=torch.bfloat16)
        out = torch.empty(B, hq * d, device=dev, dtype=torch.bfloat16)
        po = torch.empty(B * hq * S * d, device=dev)
        pm = torch.empty(B * hq * S * 2, device=dev)
        cnt = torch.zeros(B * hkv, dtype=torch.int32, device=dev) if fused else None
        nwg = S * hkv * B
        stamps = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device=dev)

        def call(i):
            kc, vc = caches[i % layers]
            rc = lib.mrsum_attn_decode_mfma(q.data_ptr(), q.stride(0), kc.data_ptr(), vc.data_ptr(), bt.data_ptr(),
                                            bt.stride(0), pos.data_ptr(), po.data_ptr(), pm.data_ptr(), out.data_ptr(),
                                            out.stride(0), B, hq, hkv, d, page, S, 1 / math.sqrt(d),
                                            cnt.data_ptr() if cnt is not None else None, 0,
                                            torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc

        lib.mrsum_attn_set_stamps(None)
        for i in range(layers):
            call(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.iters):
            call(i)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        lib.mrsum_attn_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
        call(3)
        torch.cuda.synchronize()
        lib.mrsum_attn_set_stamps(None)
        st = stamps.view(nwg * 4, 8).double().cpu()
        st = st[st[:, 7] > 0]  # waves of workgroups with tiles
        mean = st.mean(0)
        tiles = float(mean[7])
        rec = {"case": name, "B": B, "hq": hq, "hkv": hkv, "ctx": ctx, "splits": S, "fused": fused, "wall_us": round(us, 2),
               "tiles_per_wg": round(tiles, 2), "total_cycles": round(float(mean[6]))}
        rec.update({p: round(float(mean[i])) for i, p in enumerate(PHASES)})
        rec["per_tile"] = {p: round(float(mean[i]) / max(tiles, 1)) for i, p in enumerate(PHASES) if 1 <= i <= 4}
        rec["max_total_cycles"] = round(float(st[:, 6].max()))
        print(json.dumps(rec), flush=True)
        del caches


if __name__ == "__main__":
    main()
