#!/usr/bin/env python3
"""In-situ plan experiments as whole decode steps (one engine; the plan of one op swapped between runs,
graphs / workspaces rebuilt; alternating rounds), for TP=1 or one rank's TP=K shard (the TP kernel
sequence over a group of one rank, engine/model.py LocalReduce).

Variants (comma separated, ``plan`` = unchanged):
  attnfusedS / attnsepS        decode attention with S splits, fused / separate merge (the batch's bucket)
  role:stream:WPB:S            stream GEMM for role (qkv | o | down | gate_up) with (wpb, S)
  role:skinny:NT:S             register-streaming kernel
  gate_up:stream_split:WPB:S   split-K gate_up with the SwiGLU in the last arriver
  deferM                       the TP=1 deferred RMSNorm up to M rows (ops.DEFER_NORM_MAX_M)
  waves:W                      register-streaming kernels with W (4 | 8) waves per workgroup at every grid
  fp8stream:N:K:WPB:S          the fp8 weight of shape N x K on the LDS-DMA stream kernel with (wpb, S) (SwiGLU: S > 1
                               = the split-K SwiGLU epilogue)
  fp8skinny:N:K                the fp8 weight of shape N x K on the register-streaming kernel
  w8max:N                      8-wave register-streaming workgroups for one row up to N workgroups
  fp8resid:N:K:WPB:S           the fp8 deferred-norm producer (stream_fp8, residual epilogue) of one shape
  buckets:B1+B2+...            decode graph buckets up to the largest given (the rest unchanged)
  resid:ROLE=KIND              the deferred-norm / TP-push producer of ROLE (o | down) forced to KIND
                               (skinny | stream): ops.RESID_FORCE
  env:NAME=VALUE[+NAME=VALUE]  environment overrides read at call time (e.g. env:MRSUM_TP_PUSH=0)
  A&B&...                      several of the above at once (e.g. buckets:1+2+4+8+10+16&attnfused3)

    python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --variants plan,attnfused32,gate_up:stream_split:4:4
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--ctx", type=int, default=4000)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp-shard", type=int, default=1)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--variants", default="plan")
    a = ap.parse_args()
    import torch
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    from llm_map_reduce_summarizer_amd.ops import hip
    base_attn, base_plan = hip.decode_attn_plan, hip.plan
    cfg = get_model_config(a.model)
    k = a.tp_shard
    if k > 1:
        cfg = get_model_config(a.model, n_heads=cfg.n_heads // k, n_kv_heads=cfg.n_kv_heads // k,
                               ffn=cfg.ffn // k, vocab_size=cfg.vocab_size // k)
    eng = LLMEngine(cfg, device="cuda:0", max_model_len=a.ctx + a.new + 64, max_num_seqs=max(8, a.batch),
                    kv_fraction=0.5, sync_every=32, weight_dtype=a.dtype)
    eng.model.emulate_tp_reduce = k > 1
    bucket = eng._bucket(a.batch)
    V = cfg.vocab_size
    prompt = [[1] + [(i * 7919 + j * 31) % (V - 20) + 10 for j in range(a.ctx)] for i in range(a.batch)]

    from llm_map_reduce_summarizer_amd import ops
    base_defer = ops.DEFER_NORM_MAX_M
    base_fp8r = hip.fp8_resid_cfg
    base_scf8 = hip.stream_config_fp8
    base_w8max = hip.SKINNY_WAVES8_MAX_WGS

    env_set = []
    import llm_map_reduce_summarizer_amd.engine.engine as engine_mod
    base_buckets = engine_mod.BUCKETS

    def install(v):
        reset()
        for part in v.split("&"):  # a variant may combine specs: buckets:1+2+4+8+10+16&attnfused3
            apply(part)

    def reset():
        hip.decode_attn_plan, hip.plan = base_attn, base_plan
        ops.DEFER_NORM_MAX_M = base_defer
        hip.fp8_resid_cfg = base_fp8r
        hip.stream_config_fp8 = base_scf8
        hip.SKINNY_WAVES_FORCE = None
        hip.SKINNY_WAVES8_MAX_WGS = base_w8max
        for name, old in env_set:
            if old is None:
                os.environ.pop(name, None)
            else:
                os.environ[name] = old
        env_set.clear()
        ops.RESID_FORCE.clear()
        import llm_map_reduce_summarizer_amd.engine.engine as engine_mod
        engine_mod.BUCKETS = base_buckets

    def apply(v):
        import llm_map_reduce_summarizer_amd.engine.engine as engine_mod
        if v == "plan":
            return
        if v.startswith("buckets:"):  # buckets:1+2+4+8+10+16 -- the decode graph buckets below 24
            low = tuple(int(t) for t in v[len("buckets:"):].split("+"))
            engine_mod.BUCKETS = low + tuple(b for b in base_buckets if b > max(low))
            return
        if v.startswith("resid:"):
            role, kind = v[len("resid:"):].split("=")
            ops.RESID_FORCE[role] = kind
            return
        if v.startswith("env:"):
            for kv in v[4:].split("+"):
                name, val = kv.split("=", 1)
                env_set.append((name, os.environ.get(name)))
                os.environ[name] = val
            return
        if v.startswith("fp8stream:"):  # fp8stream:N:K:wpb:S -- one fp8 shape on the stream kernel
            N0, K0, wpb, S = (int(t) for t in v.split(":")[1:])

            def scf8(N, K, swiglu=False, splits=None, M=1):
                if (N, K) == (N0, K0):
                    return (wpb, splits or S)
                return base_scf8(N, K, swiglu=swiglu, splits=splits, M=M)
            hip.stream_config_fp8 = scf8
            return
        if v.startswith("fp8skinny:"):  # fp8skinny:N:K -- that fp8 shape on the register-streaming kernel
            N0, K0 = (int(t) for t in v.split(":")[1:])
            hip.stream_config_fp8 = (lambda N, K, swiglu=False, splits=None, M=1:
                                     None if (N, K) == (N0, K0) else base_scf8(N, K, swiglu=swiglu, splits=splits, M=M))
            return
        if v.startswith("fp8resid:"):  # fp8resid:N:K:wpb:S -- the fp8 deferred-norm producer of one shape
            N0, K0, wpb, S = (int(t) for t in v.split(":")[1:])
            hip.fp8_resid_cfg = lambda M, N, K: (wpb, S) if (N, K) == (N0, K0) else base_fp8r(M, N, K)
            return
        if v.startswith("w8max:"):
            hip.SKINNY_WAVES8_MAX_WGS = int(v[len("w8max:"):])
            return
        if v.startswith("waves:"):
            hip.SKINNY_WAVES_FORCE = int(v[len("waves:"):])
            return
        if v.startswith("defer"):  # deferFOO: the deferred RMSNorm up to FOO rows
            ops.DEFER_NORM_MAX_M = int(v[5:])
            return
        if v.startswith("attn"):
            fused = v.startswith("attnfused")
            S = int(v[len("attnfused"):] if fused else v[len("attnsep"):])
            hip.decode_attn_plan = lambda B, hkv, ctx, **kw: (S, fused) if B == eng._bucket(a.batch) else base_attn(B, hkv, ctx, **kw)
            return
        role, kind, p1, p2 = v.split(":")
        p = (kind, int(p1), int(p2))

        def plan(r, M, N, K, splits=None, stream=True):
            if r == role and M <= bucket and splits is None:
                return p
            return base_plan(r, M, N, K, splits=splits, stream=stream)
        hip.plan = plan

    variants = a.variants.split(",")
    for r in range(a.rounds):
        for v in variants:
            install(v)
            eng._workspaces.clear()
            eng._graphs.clear()
            eng.generate(prompt, [SamplingParams(8, 0.3, i) for i in range(a.batch)], ignore_eos=True)
            s0 = dict(eng.stats)
            torch.cuda.synchronize()
            eng.generate(prompt, [SamplingParams(a.new, 0.3, i) for i in range(a.batch)], ignore_eos=True)
            st = eng.stats
            ms = 1000 * (st["decode_s"] - s0["decode_s"]) / max(1, st["decode_steps"] - s0["decode_steps"])
            print(json.dumps({"round": r, "tp_shard": k, "batch": a.batch, "variant": v, "ctx": a.ctx,
                              "decode_ms_per_step": round(ms, 4)}), flush=True)
    hip.decode_attn_plan, hip.plan = base_attn, base_plan


if __name__ == "__main__":
    main()
