#!/usr/bin/env python3
"""Decode-step latency of the engine (Llama-3-8B bf16 by default) at the batch sizes the
summarizer runs: B=1 (final reduce), B~5 (map at DP=8), B=10 (reduce level 1), B=39 (map at DP=1).
Each sequence has a ~CTX-token prompt; reports ms per decode step (hipGraph replay, pinned length)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batches", default="1,5,10,39")
    ap.add_argument("--ctx", type=int, default=4000)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8v", "fp8"])
    ap.add_argument("--tp-shard", type=int, default=1,
                    help="run ONE rank's shard shapes of TP=K (heads, ffn and vocab / K) on this GPU with no "
                         "all-reduce: the compute + launch floor of a TP=K decode step")
    ap.add_argument("--deferred-norm", action="store_true",
                    help="with --tp-shard: keep the TP=1 deferred RMSNorm (default: the TP rank's kernel sequence, "
                         "split-K slabs -> add_rmsnorm_parts standing in for the fused P2P all-reduce kernel)")
    a = ap.parse_args()
    import torch
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    cfg = get_model_config(a.model)
    if a.tp_shard > 1:
        k = a.tp_shard
        cfg = get_model_config(a.model, n_heads=cfg.n_heads // k, n_kv_heads=cfg.n_kv_heads // k,
                               ffn=cfg.ffn // k, vocab_size=cfg.vocab_size // k)
    eng = LLMEngine(cfg, device="cuda:0", max_model_len=a.ctx + a.new + 64,
                    max_num_seqs=64, kv_fraction=0.5, weight_dtype=a.dtype, sync_every=32, kv_dtype=a.kv_dtype)
    eng.model.emulate_tp_reduce = a.tp_shard > 1 and not a.deferred_norm
    res = []
    for B in (int(b) for b in a.batches.split(",")):
        V = cfg.vocab_size
        prompts = [[1] + [(i * 7919 + j * 31) % (V - 20) + 10 for j in range(a.ctx)] for i in range(B)]
        sp = [SamplingParams(a.new, 0.3, i) for i in range(B)]
        eng.generate(prompts, [SamplingParams(8, 0.3, i) for i in range(B)], ignore_eos=True)  # capture/warm
        s0 = dict(eng.stats)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.generate(prompts, sp, ignore_eos=True)
        wall = time.perf_counter() - t0
        st = eng.stats
        steps = st["decode_steps"] - s0["decode_steps"]
        dec = st["decode_s"] - s0["decode_s"]
        res.append({"B": B, "ctx": a.ctx, "tp_shard": a.tp_shard, "kv_dtype": a.kv_dtype, "decode_ms_per_step": round(1000 * dec / max(1, steps), 3),
                    "prefill_s": round(st["prefill_s"] - s0["prefill_s"], 3), "wall_s": round(wall, 3)})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
