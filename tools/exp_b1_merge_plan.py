#!/usr/bin/env python3
"""Experiment: decode attention split plans measured in situ as whole decode steps of Llama-3-8B (one
engine, the plan of the --batch bucket swapped between runs, graphs / workspaces rebuilt; alternating
rounds): by default B = 1 in the <= 12k context class (the final reduce runs at ~10k), the current plan
(32 splits, separate merge) against fused merges at 8 / 16 splits and 64 / 16 separate splits; e.g.
``--batch 39 --ctx 4000 --variants plan,sep1,sep2,fused2`` for the map step.  JSON line per run."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=10000)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--variants", default="plan,fused16,fused8,sep64,sep16",
                    help="plan | fusedS | sepS (S splits, fused / separate merge)")
    a = ap.parse_args()
    import torch
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    from llm_map_reduce_summarizer_amd.ops import hip
    base = hip.decode_attn_plan
    variants = {}
    for v in a.variants.split(","):
        variants[v] = None if v == "plan" else ((int(v[5:]), True) if v.startswith("fused") else (int(v[3:]), False))
    cfg = get_model_config(a.model)
    eng = LLMEngine(cfg, device="cuda:0", max_model_len=a.ctx + a.new + 64, max_num_seqs=max(8, a.batch),
                    kv_fraction=0.5, sync_every=32, weight_dtype=a.dtype)
    V = cfg.vocab_size
    prompt = [[1] + [(i * 7919 + j * 31) % (V - 20) + 10 for j in range(a.ctx)] for i in range(a.batch)]
    for r in range(a.rounds):
        for name, v in variants.items():
            hip.decode_attn_plan = base if v is None else (lambda B, hkv, ctx, v=v: v if B == eng._bucket(a.batch) else base(B, hkv, ctx))
            eng._workspaces.clear()
            for attr in ("_graphs",):
                if hasattr(eng, attr):
                    getattr(eng, attr).clear()
            eng.generate(prompt, [SamplingParams(8, 0.3, i) for i in range(a.batch)], ignore_eos=True)
            s0 = dict(eng.stats)
            torch.cuda.synchronize()
            eng.generate(prompt, [SamplingParams(a.new, 0.3, i) for i in range(a.batch)], ignore_eos=True)
            st = eng.stats
            ms = 1000 * (st["decode_s"] - s0["decode_s"]) / max(1, st["decode_steps"] - s0["decode_steps"])
            print(json.dumps({"round": r, "model": a.model, "batch": a.batch, "variant": name,
                              "splits_fused": base(eng._bucket(a.batch), cfg.n_kv_heads, a.ctx + a.new) if v is None else v,
                              "ctx": a.ctx, "decode_ms_per_step": round(ms, 4)}), flush=True)
    hip.decode_attn_plan = base


if __name__ == "__main__":
    main()
