#!/usr/bin/env python3
"""Prefill GEMM experiment: 32x32 MFMA tiles (v_mfma_f32_32x32x16_bf16 / v_mfma_scale_f32_32x32x64_f8f6f4,
group_m bit 8 of mrsum_gemm) vs the 16x16 tiles.  First a numerics check of the 32x32 variant against fp32
(bf16 / fp8, plain / SwiGLU, ragged M, N % 32 == 16, strided output for the register epilogue), then an
interleaved timing A/B in one process.  One JSON line per check / (shape, variant).

    python tools/exp_gemm_m32.py [--ms 4096,16384] [--fp8-model llama3-70b]
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402
from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight  # noqa: E402

M32 = 256
VARIANTS = [("m16g4", 4), ("m32g4", 4 | M32)]
SHAPES = {
    "llama3-8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)},
    "llama3-70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)},
}


def swiglu_ref(y):
    n = y.shape[1]
    y = y.view(y.shape[0], n // 16, 2, 8)
    return (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(y.shape[0], n // 2)


def check(dev):
    torch.manual_seed(1)
    ok = True
    for (M, N, K) in [(300, 272, 256), (777, 1040, 512), (4100, 6160, 1024)]:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        for swiglu in (False, True):
            if swiglu and N % 32:
                continue
            ref = x.float() @ w.float().t()
            ref = swiglu_ref(ref) if swiglu else ref
            for strided in (False, True):
                n_out = N // 2 if swiglu else N
                if strided:
                    buf = torch.zeros(M, n_out + 4, dtype=torch.bfloat16, device=dev)
                    out = buf[:, 4:]
                else:
                    out = torch.empty(M, n_out, dtype=torch.bfloat16, device=dev)
                for gm in [g for _, g in VARIANTS]:
                    out.fill_(float("nan"))
                    hip.gemm(x, w, out=out, swiglu=swiglu, group_m=gm)
                    err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                    good = err < 1e-2
                    ok &= good
                    print(json.dumps({"check": "bf16", "M": M, "N": N, "K": K, "swiglu": swiglu, "strided": strided,
                                      "group_m": gm, "rel_err": round(err, 5), "ok": good}), flush=True)
        wq = Fp8Weight.quantize(w)
        xq, xs = hip.quant_fp8_rows(x)
        deq = (xq.float() * xs.view(-1, 1)) @ (wq.q.float() * wq.scale.view(-1, 1)).t()
        for swiglu in (False, True):
            if swiglu and N % 32:
                continue
            ref = swiglu_ref(deq) if swiglu else deq
            for gm in (4, 4 | M32):
                out = hip.gemm_fp8(xq, xs, wq, swiglu=swiglu, group_m=gm)
                err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                good = err < 1e-2
                ok &= good
                print(json.dumps({"check": "fp8", "M": M, "N": N, "K": K, "swiglu": swiglu, "group_m": gm,
                                  "rel_err": round(err, 5), "ok": good}), flush=True)
    return ok


def timeit(fn, iters):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1000.0 / iters


def ab(dev, model, ms, fp8, rounds=5, iters=10, roles=None):
    for role, (N, K) in SHAPES[model].items():
        if roles and role not in roles:
            continue
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        wq = Fp8Weight.quantize(w) if fp8 else None
        swiglu = role == "gate_up"
        for M in ms:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=dev)
            xq, xs = hip.quant_fp8_rows(x) if fp8 else (None, None)
            fns = {}
            for name, gm in VARIANTS:
                if fp8:
                    fns[name] = (lambda gm=gm: hip.gemm_fp8(xq, xs, wq, out=out, swiglu=swiglu, group_m=gm))
                else:
                    fns[name] = (lambda gm=gm: hip.gemm(x, w, out=out, swiglu=swiglu, group_m=gm))
            for f in fns.values():
                f()
            torch.cuda.synchronize()
            times = {v: [] for v in fns}
            for _ in range(rounds):
                for v, f in fns.items():
                    times[v].append(timeit(f, iters))
            flop = 2.0 * M * N * K
            for v, ts in times.items():
                ts.sort()
                med = ts[len(ts) // 2]
                print(json.dumps({"model": model, "role": role, "M": M, "N": N, "K": K, "fp8": fp8, "variant": v,
                                  "us_med": round(med, 1), "us_min": round(ts[0], 1),
                                  "tflops_med": round(flop / med / 1e6, 1)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="4096,16384")
    ap.add_argument("--fp8-model", default="llama3-70b")
    ap.add_argument("--fp8-ms", default="8192")
    ap.add_argument("--fp8-roles", default="", help="comma list (default: all four)")
    ap.add_argument("--skip-check", action="store_true")
    ap.add_argument("--skip-bf16", action="store_true")
    ap.add_argument("--bf16-roles", default="", help="comma list (default: all four)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="m16g4=4,m32g4=260", help="name=group_m list (bit 8: 32x32 tiles)")
    a = ap.parse_args()
    VARIANTS[:] = [(v.split("=")[0], int(v.split("=")[1])) for v in a.variants.split(",")]
    dev = "cuda:0"
    if not a.skip_check and not check(dev):
        print(json.dumps({"check": "FAILED"}), flush=True)
        sys.exit(1)
    if not a.skip_bf16:
        ab(dev, "llama3-8b", [int(m) for m in a.ms.split(",")], False, a.rounds,
           roles=[r for r in a.bf16_roles.split(",") if r])
    if a.fp8_model:
        ab(dev, a.fp8_model, [int(m) for m in a.fp8_ms.split(",")], True, a.rounds,
           roles=[r for r in a.fp8_roles.split(",") if r])


if __name__ == "__main__":
    main()
