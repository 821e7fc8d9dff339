#!/usr/bin/env python3
"""Diagnose a forward-parity failure (tests/test_forward_parity_gpu.py): run the engine on the test's
random HF checkpoint under variants and report NaN / relative error of the first (prefill) logits row
against the textbook fp32 forward.  Variants: RoPE scaling on/off, chunked (paged) vs one-pass prefill,
prompt lengths, peaked vs flat attention."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tests.test_forward_parity_gpu as T  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.config import get_model_config  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams  # noqa: E402


class MP:
    def setattr(self, o, n, v):
        setattr(o, n, v)


def run(name, model, lengths, chunk, flat=False):
    cfg = get_model_config(model, n_layers=2)
    ck = T._checkpoint(cfg, 2, tied=False)
    if flat:
        for k in list(ck):
            if "q_proj" in k or "k_proj" in k:
                ck[k] = (ck[k].float() * 0.2).to(torch.bfloat16)
    prompts = T._prompts(lengths, 5)
    index = {k: "mem" for k in ck}
    T.W._open_shards = lambda path: (index, {"mem": T._Mem(ck)})
    eng = LLMEngine(cfg, device="cuda:0", weights_path="mem", use_graphs=False, max_num_seqs=8, sync_every=64,
                    max_model_len=10240, kv_pages=400, prefill_chunk=chunk)
    rec = []
    orig = eng._sample

    def spy(logits, view):
        rec.append(logits.float().clone())
        orig(logits, view)
    eng._sample = spy
    outs = eng.generate(prompts, [SamplingParams(2, 0.0, 0)] * len(prompts), ignore_eos=True)
    torch.cuda.synchronize()
    order = sorted(range(len(prompts)), key=lambda i: -len(prompts[i]))
    pre = torch.cat(rec[:-1])
    res = {"name": name, "nan_rows": [bool(torch.isnan(r).any()) for r in pre]}
    errs = []
    for slot, i in enumerate(order):
        ref = T._textbook_logits(ck, cfg, prompts[i], torch.device("cuda:0"))[-1]
        got = pre[slot]
        errs.append(round(float((got - ref).norm() / ref.norm()), 4))
    res["rel_err"] = errs
    del eng
    torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    run("3.1_chunked_9000_8193", "llama3.1-8b", (9000, 8193), 4096)
    run("3.1_onepass_9000", "llama3.1-8b", (9000,), 0)
    run("3.1_chunked_9000", "llama3.1-8b", (9000,), 4096)
    run("3_chunked_9000", "llama3-8b", (9000,), 4096)
    run("3.1_onepass_4000", "llama3.1-8b", (4000,), 0)
    run("3.1_chunked_9000_flat", "llama3.1-8b", (9000,), 4096, flat=True)
    run("3.1_chunked_5000", "llama3.1-8b", (5000,), 4096)
