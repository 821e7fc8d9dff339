#!/usr/bin/env python3
"""A/B of the K/V prefetch into the Infinity Cache (csrc/kernels/kv_prefetch.hip, engine._prefetch_plan) on
whole decode steps of Llama-3-8B bf16: one engine, graphs re-captured per configuration, configurations
interleaved (A/B/A/B) so box drift hits them alike.  Prints one JSON line per (config, round)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--ctx", type=int, default=13500)
    ap.add_argument("--new", type=int, default=200)
    ap.add_argument("--configs", default="off,qkv:64,down:64,down:128,qkv:128")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--kv-dtype", default="bf16")
    a = ap.parse_args()
    import torch
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    cfg = get_model_config(a.model)
    eng = LLMEngine(cfg, device="cuda:0", max_model_len=a.ctx + a.new + 64, max_num_seqs=max(16, a.batch),
                    kv_fraction=0.5, sync_every=32, kv_dtype=a.kv_dtype)
    V = cfg.vocab_size
    prompts = [[1] + [(i * 7919 + j * 31) % (V - 20) + 10 for j in range(a.ctx)] for i in range(a.batch)]
    for r in range(a.rounds):
        for c in a.configs.split(","):
            mode, _, wps = c.partition(":")
            os.environ["MRSUM_KV_PREFETCH"] = mode
            os.environ["MRSUM_KV_PREFETCH_WPS"] = wps or "64"
            eng._graphs.clear()
            eng.generate(prompts, [SamplingParams(8, 0.3, i) for i in range(a.batch)], ignore_eos=True)
            s0 = dict(eng.stats)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.generate(prompts, [SamplingParams(a.new, 0.3, i) for i in range(a.batch)], ignore_eos=True)
            wall = time.perf_counter() - t0
            st = eng.stats
            steps = st["decode_steps"] - s0["decode_steps"]
            ms = 1000 * (st["decode_s"] - s0["decode_s"]) / max(1, steps)
            print(json.dumps({"round": r, "config": c, "B": a.batch, "ctx": a.ctx, "kv_dtype": a.kv_dtype,
                              "plan": bool(eng._prefetch_plan(a.batch)), "decode_ms_per_step": round(ms, 3),
                              "wall_s": round(wall, 3)}), flush=True)


if __name__ == "__main__":
    main()
