#!/usr/bin/env python3
"""Experiment: stream-GEMM (wpb, splits) choices measured in situ as whole Llama-3-8B decode steps: one
engine, ``ops.hip.stream_config`` overridden for one weight shape per variant (graphs rebuilt), alternating
rounds.  A variant is ``name=N:K:wpb:S`` (``plan`` = no override).  JSON line per run.

    python tools/exp_stream_plan_insitu.py --batch 1 --variants plan,down88=4096:14336:8:8
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
    ap.add_argument("--variants", default="plan")
    a = ap.parse_args()
    import torch
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    from llm_map_reduce_summarizer_amd.ops import hip
    base = hip.stream_config
    variants = {}
    for v in a.variants.split(","):
        if v == "plan":
            variants[v] = None
        else:
            name, spec = v.split("=")
            N, K, wpb, S = (int(x) for x in spec.split(":"))
            variants[name] = (N, K, wpb, S)
    cfg = get_model_config("llama3-8b")
    eng = LLMEngine(cfg, device="cuda:0", max_model_len=a.ctx + a.new + 64, max_num_seqs=max(8, a.batch),
                    kv_fraction=0.5, sync_every=32)
    V = cfg.vocab_size
    prompt = [[1] + [(i * 7919 + j * 31) % (V - 20) + 10 for j in range(a.ctx)] for i in range(a.batch)]

    def override(o):
        def f(N, K, swiglu=False, splits=None, max_splits=16):
            if o is not None and (N, K) == (o[0], o[1]) and (splits is None or splits == o[3]):
                return (o[2], o[3])
            return base(N, K, swiglu=swiglu, splits=splits, max_splits=max_splits)
        return f
    for r in range(a.rounds):
        for name, o in variants.items():
            hip.stream_config = override(o)
            eng._workspaces.clear()
            eng._graphs.clear()
            eng.generate(prompt, [SamplingParams(8, 0.3, i) for i in range(a.batch)], ignore_eos=True)
            s0 = dict(eng.stats)
            torch.cuda.synchronize()
            eng.generate(prompt, [SamplingParams(a.new, 0.3, i) for i in range(a.batch)], ignore_eos=True)
            st = eng.stats
            ms = 1000 * (st["decode_s"] - s0["decode_s"]) / max(1, st["decode_steps"] - s0["decode_steps"])
            print(json.dumps({"round": r, "batch": a.batch, "variant": name, "override": o, "ctx": a.ctx,
                              "decode_ms_per_step": round(ms, 4)}), flush=True)
    hip.stream_config = base


if __name__ == "__main__":
    main()
