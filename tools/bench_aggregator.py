#!/usr/bin/env python3
"""BASELINE config 5: the aggregator (final reduce) pass on Llama-3-70B with fp8 weights at ~32k
context -- one request: ~32k-token reduce prompt (the aggregator's own prompt format over
synthetic chunk summaries), then up to --max-new-tokens generated tokens.  TP = number of ranks
(torchrun --nproc-per-node N); on one GPU it runs TP=1 (70 GB of fp8 weights fit in 288 GB).

Prints one JSON line with prefill tok/s, decode ms/token and the wall-clock of the pass.
"""
import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--dtype", default="fp8", choices=["bf16", "fp8"])
    ap.add_argument("--context", type=int, default=32000)
    ap.add_argument("--max-new-tokens", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8v", "fp8"],
                    help="KV-cache format; fp8 is a labelled variant (bf16 KV is the credited number)")
    a = ap.parse_args()
    import torch
    from llm_map_reduce_summarizer_amd.config import LLMConfig
    from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider
    from llm_map_reduce_summarizer_amd.parallel import dist as pdist
    from llm_map_reduce_summarizer_amd.pipeline.prompts import build_aggregation_messages
    from llm_map_reduce_summarizer_amd.pipeline.providers import GenRequest
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript

    pdist.init_distributed_from_env()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    cfg = LLMConfig(MAX_TOKENS=a.max_new_tokens)
    prov = LocalEngineProvider(a.model, cfg, tp=world, dtype=a.dtype, max_model_len=a.context + a.max_new_tokens + 64,
                               ignore_eos=True, kv_dtype=a.kv_dtype,
                               engine_options={"max_num_seqs": 8})
    t0 = time.perf_counter()
    eng = prov.engine
    init_s = time.perf_counter() - t0
    # synthetic chunk summaries until the reduce prompt reaches the target context
    words = " ".join(s["text"] for s in synthetic_transcript(24.0, seed=7)["segments"]).split()
    summaries, i = [], 0
    tok = prov.tokenizer
    while True:
        summaries.append("[Time: %02d:00 - %02d:00]\n%s" % (i, i + 1, " ".join(words[i * 700:(i + 1) * 700])))
        msgs = build_aggregation_messages(summaries, None, {"File": "synthetic"})
        n = len(prov.encode_request(GenRequest(user=msgs["user"], system=msgs["system"], max_tokens=a.max_new_tokens)))
        if n >= a.context:
            break
        i += 1
    req = GenRequest(user=msgs["user"], system=msgs["system"], max_tokens=a.max_new_tokens, temperature=0.2,
                     stage="reduce_final")
    for _ in range(a.warmup):
        asyncio.run(prov.generate_batch([req]))
    pdist.barrier()
    torch.cuda.synchronize()
    s0 = dict(eng.stats)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = asyncio.run(prov.generate_batch([req]))[0]
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    s1 = eng.stats
    pf_s = (s1["prefill_s"] - s0["prefill_s"]) / a.steps
    dec_s = (s1["decode_s"] - s0["decode_s"]) / a.steps
    dec_steps = (s1["decode_steps"] - s0["decode_steps"]) / a.steps
    out = {"metric": "aggregator pass wall-clock (Llama-3-70B %s, %d-token context, %d new tokens)"
                     % (a.dtype, n, a.max_new_tokens),
           "value": round(dt, 3), "unit": "s", "higher_is_better": False, "n_gpus": world, "tp": world,
           "prompt_tokens": res.prompt_tokens, "completion_tokens": res.completion_tokens,
           "prefill_s": round(pf_s, 3), "prefill_tok_s": round(res.prompt_tokens / pf_s, 1) if pf_s else None,
           "decode_ms_per_token": round(1000 * dec_s / max(1, dec_steps), 3),
           "kv_dtype": a.kv_dtype, "weights_gib": round(eng.model.weight_bytes() / 2 ** 30, 1), "init_s": round(init_s, 1),
           "hbm_peak_gib": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1),
           "data": "synthetic summaries; random-init weights; generation pinned to max_new_tokens"}
    # the planner's cost model for this pass on an 8-GPU node (TP=8): what a TP prefill forward (RCCL
    # all-reduces of the activations) and a one-rank prefill + KV hand-off would take, and the stage
    from llm_map_reduce_summarizer_amd.parallel import plan
    d = plan.ModelDims.of(prov.model_config(), 1.0 if a.dtype == "fp8" else 2.0)
    hw = plan.HWModel()
    pl, mn = [res.prompt_tokens], [a.max_new_tokens]
    ch = plan.choose(d, hw, pl, mn, 8, handoff=True)
    out["cost_model_tp8"] = {"tp_prefill_s": round(plan.prefill_s(d, hw, pl[0], 8), 3),
                             "handoff_prefill_s": round(plan.handoff_prefill_s(d, hw, pl, 8), 3),
                             "decode_ms_per_step": round(1e3 * plan.decode_step_s(d, hw, 1, pl[0] + mn[0] / 2, 8), 3),
                             "stage_s": ch["estimates_s"], "choice": {k: v for k, v in ch.items() if k != "estimates_s"},
                             "hw": {"hbm_bw": hw.hbm_bw, "ar_lat_s": hw.ar_lat_s, "ar_bw": hw.ar_bw,
                                    "prefill_flops": hw.prefill_flops}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
