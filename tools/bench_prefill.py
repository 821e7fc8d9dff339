#!/usr/bin/env python3
"""Prefill wall-clock of the engine: one-pass vs chunked prefill (slices through the paged cache) and the
contiguous vs paged attention path, at the prompt lengths of the summarizer's stages (map ~4k x 39,
final reduce ~10k, the 70B aggregator's 32k).  generate(max_new=1) = prefill + one sampled token.

    python tools/bench_prefill.py [--model llama3-8b] [--dtype bf16] [--lens 32768] [--nseq 1] [--chunks 0,4096,8192]
"""
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
    ap.add_argument("--lens", default="32768")
    ap.add_argument("--nseq", type=int, default=1)
    ap.add_argument("--chunks", default="0,4096,8192")
    ap.add_argument("--paged", default="0,1")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--max-prefill-tokens", default=str(1 << 20),
                    help="comma list: packed-prefill pass budgets to compare (engine max_prefill_tokens)")
    a = ap.parse_args()
    import torch
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams
    cfg = get_model_config(a.model)
    lens = [int(x) for x in a.lens.split(",")]
    eng = LLMEngine(cfg, device="cuda:0", max_model_len=max(lens) + 64, max_num_seqs=max(64, a.nseq),
                    kv_fraction=0.3, weight_dtype=a.dtype, max_prefill_tokens=1 << 20)
    budgets = [int(b) for b in a.max_prefill_tokens.split(",")]
    V = cfg.vocab_size
    for L in lens:
        prompts = [[1] + [(i * 7919 + j * 31) % (V - 20) + 10 for j in range(L - 1)] for i in range(a.nseq)]
        sp = [SamplingParams(1, 0.0, i) for i in range(a.nseq)]
        for chunk, paged, budget in ((c, p, b) for c in (int(c) for c in a.chunks.split(","))
                                     for p in (int(p) for p in a.paged.split(",")) for b in budgets):
                if chunk and not paged:
                    continue  # chunked slices always read the paged cache
                eng.prefill_chunk, eng.paged_prefill, eng.max_prefill_tokens = chunk, bool(paged), budget
                eng.generate(prompts, sp)  # warm
                ts = []
                for _ in range(a.reps):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    eng.generate(prompts, sp)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                ts.sort()
                print(json.dumps({"model": a.model, "dtype": a.dtype, "len": L, "nseq": a.nseq, "chunk": chunk,
                                  "paged": paged, "max_prefill_tokens": budget,
                                  "s_med": round(ts[len(ts) // 2], 4), "s_min": round(ts[0], 4),
                                  "tok_s": round(L * a.nseq / ts[len(ts) // 2], 1)}), flush=True)


if __name__ == "__main__":
    main()
