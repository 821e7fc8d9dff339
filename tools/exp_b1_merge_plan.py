#!/usr/bin/env python3
"""Experiment: B = 1 decode attention split plan in the <= 12k context class (the final reduce runs at
~10k): the current plan (32 splits, separate merge kernel) against fused last-arriver merges at 8 / 16
splits and 64 separate splits, measured in situ as whole decode steps of Llama-3-8B (one engine, the
plan swapped between rounds, graphs / workspaces rebuilt; alternating rounds).  JSON line per run."""
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
    a = ap.parse_args()
    import torch
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    from llm_map_reduce_summarizer_amd.ops import hip
    base = hip.decode_attn_plan
    variants = {"plan": None, "fused16": (16, True), "fused8": (8, True), "sep64": (64, False), "sep16": (16, False)}
    cfg = get_model_config("llama3-8b")
    eng = LLMEngine(cfg, device="cuda:0", max_model_len=a.ctx + a.new + 64, max_num_seqs=8, kv_fraction=0.3,
                    sync_every=32)
    V = cfg.vocab_size
    prompt = [[1] + [(j * 31) % (V - 20) + 10 for j in range(a.ctx)]]
    for r in range(a.rounds):
        for name, v in variants.items():
            hip.decode_attn_plan = base if v is None else (lambda B, hkv, ctx, v=v: v if B == 1 else base(B, hkv, ctx))
            eng._workspaces.clear()
            for attr in ("_graphs",):
                if hasattr(eng, attr):
                    getattr(eng, attr).clear()
            eng.generate(prompt, [SamplingParams(8, 0.3, 0)], ignore_eos=True)
            s0 = dict(eng.stats)
            torch.cuda.synchronize()
            eng.generate(prompt, [SamplingParams(a.new, 0.3, 0)], ignore_eos=True)
            st = eng.stats
            ms = 1000 * (st["decode_s"] - s0["decode_s"]) / max(1, st["decode_steps"] - s0["decode_steps"])
            print(json.dumps({"round": r, "variant": name, "splits_fused": base(1, 8, a.ctx + a.new) if v is None else v,
                              "ctx": a.ctx, "decode_ms_per_step": round(ms, 4)}), flush=True)
    hip.decode_attn_plan = base


if __name__ == "__main__":
    main()
