#!/usr/bin/env python3
"""The planner's view of the headline job (CPU only, no engine): the exact stage requests of the bench's
pipeline (synthetic transcript -> chunker -> map prompts -> level-1 / final reduce prompts, rendered and
tokenised as the local provider does), every generation pinned to --max-new tokens of pseudo-random ids
(what random-init weights emit), then parallel/plan.py's choice per stage at each world size and all-reduce
latency: TP degree, predicted seconds of every candidate, and the predicted end-to-end wall time.

    python tools/plan_stages.py --hours 10 --worlds 1,2,4,8 --ar-lat-us 5,10,20

One JSON line per (world, latency): {"world", "ar_lat_us", "stages": [{"stage", "requests", "tp", "handoff",
"estimates_s"}], "predicted_e2e_s", "predicted_chunks_per_s"}.  Reference fan-out / reduce:
/root/reference/llm_executor.py:133-147, /root/reference/result_aggregator.py:321-355.
"""
import argparse
import asyncio
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def stage_requests(hours: float, max_new: int, model: str, chunk_tokens: int = 4000, seed: int = 0):
    """[(stage, prompt_lens, max_new_list)] of one pipeline run, in execution order."""
    from llm_map_reduce_summarizer_amd.config import LLMConfig
    from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider
    from llm_map_reduce_summarizer_amd.pipeline.executor import LLMExecutor
    from llm_map_reduce_summarizer_amd.pipeline.orchestrator import TranscriptSummarizer
    from llm_map_reduce_summarizer_amd.pipeline.providers import GenResult
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript

    calls = []

    class Recorder(LocalEngineProvider):
        async def generate_batch(self, reqs):
            prompts = [self.encode_request(r) for r in reqs]
            calls.append((reqs[0].stage if reqs else "map", [len(p) for p in prompts], [r.max_tokens for r in reqs]))
            out = []
            for r in reqs:
                rng = random.Random(hash(r.user) & 0xffffffff)
                ids = [rng.randrange(1000, 120000) for _ in range(r.max_tokens)]
                out.append(GenResult(self.tokenizer.decode(ids), len(prompts[0]), r.max_tokens))
            return out

    cfg = LLMConfig(MAX_TOKENS=max_new, TEMPERATURE=0.3, REDUCE_TEMPERATURE=0.2)
    prov = Recorder(model, cfg, device="cpu", ignore_eos=True, parallel="dp")
    ex = LLMExecutor(config=cfg, provider_obj=prov)
    summ = TranscriptSummarizer(executor=ex, max_tokens_per_chunk=chunk_tokens)
    asyncio.run(summ.summarize(synthetic_transcript(hours, seed=seed)))
    return calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hours", type=float, default=10.0)
    ap.add_argument("--max-new", type=int, default=1000)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--ar-lat-us", default="5,10,20")
    ap.add_argument("--ar-gbps", type=float, default=100.0)
    a = ap.parse_args()
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.engine.provider import divisors
    from llm_map_reduce_summarizer_amd.parallel import plan
    calls = stage_requests(a.hours, a.max_new, a.model)
    d = plan.ModelDims.of(get_model_config(a.model), 1.0 if a.fp8 else 2.0)
    n_chunks = len(calls[0][1])
    for w in (int(x) for x in a.worlds.split(",")):
        for lat in (float(x) for x in a.ar_lat_us.split(",")):
            hw = plan.with_measurements(plan.HWModel(), ar_lat_s=lat * 1e-6, ar_bw=a.ar_gbps * 1e9)
            stages, total = [], 0.0
            for stage, lens, mn in calls:
                ch = plan.choose(d, hw, lens, mn, w, candidates=divisors(w), handoff=True)
                t = ch["estimates_s"][str(ch["tp"])]
                total += t
                stages.append({"stage": stage, "requests": len(lens), "max_prompt": max(lens), "tp": ch["tp"],
                               "handoff": ch.get("handoff", False), "estimates_s": ch["estimates_s"]})
            print(json.dumps({"world": w, "ar_lat_us": lat, "hours": a.hours, "model": a.model,
                              "stages": stages, "predicted_e2e_s": round(total, 3),
                              "predicted_chunks_per_s": round(n_chunks / total, 3)}), flush=True)
            if w == 1:
                break  # no all-reduce at world 1


if __name__ == "__main__":
    main()
