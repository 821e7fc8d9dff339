"""Worker for tests/test_custom_ar_gpu.py::test_tp2_engine_one_gpu: a TP=2 engine whose two ranks
share ONE GPU (gloo process group for the eager prefill all-reduces; the decode all-reduces and the
vocab-parallel sampling key max run on the custom P2P kernel, inside the captured hipGraphs); the
chunked TP prefill (layer-major passes, async all-reduces) against the one-pass prefill."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.engine.config import get_model_config  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    cfg = get_model_config("tiny-gqa4", init_std=0.05)
    kw = dict(device="cuda:0", max_model_len=512, max_num_seqs=8, kv_pages=64, seed=7)
    prompts = [[128000] + [(i * 37 + j * 11) % 120000 + 5 for j in range(20 + 30 * i)] for i in range(3)]
    greedy = [SamplingParams(12, 0.0, i) for i in range(3)]
    sampled = [SamplingParams(12, 0.8, 100 + i) for i in range(3)]
    tp = LLMEngine(cfg, tp_rank=rank, tp_size=2, tp_group=None, use_graphs=True, **kw)
    assert tp.model.custom_ar is not None and tp.model.tp_sampling
    g2 = [o.token_ids for o in tp.generate(prompts, greedy)]
    s2 = [o.token_ids for o in tp.generate(prompts, sampled)]
    assert tp.model.custom_ar.error() == 0
    tp_eager = LLMEngine(cfg, tp_rank=rank, tp_size=2, tp_group=None, use_graphs=False, **kw)
    assert [o.token_ids for o in tp_eager.generate(prompts, greedy)] == g2, "graph vs eager TP decode"
    # chunked prefill of longer prompts: TP passes run layer-major with async all-reduces (model.prefill_passes)
    longp = [[128000] + [(i * 53 + j * 7) % 120000 + 5 for j in range(150 + 40 * i)] for i in range(3)]
    chunked = LLMEngine(cfg, tp_rank=rank, tp_size=2, tp_group=None, use_graphs=True, prefill_chunk=64, **kw)
    gc = [o.token_ids for o in chunked.generate(longp, greedy)]
    assert chunked.stats["prefill_slices"] > 3
    assert gc == [o.token_ids for o in tp.generate(longp, greedy)], "layer-major chunked TP prefill vs one pass"
    # both ranks must have produced the same tokens
    allg = [None, None]
    dist.all_gather_object(allg, (g2, s2))
    assert allg[0] == allg[1], "ranks disagree"
    if rank == 0:
        one = LLMEngine(cfg, use_graphs=True, **kw)
        g1 = [o.token_ids for o in one.generate(prompts, greedy)]
        s1 = [o.token_ids for o in one.generate(prompts, sampled)]
        first = sum(a[0] == b[0] for a, b in zip(g1, g2))
        same = sum(x == y for a, b in zip(g1 + s1, g2 + s2) for x, y in zip(a, b))
        total = sum(len(a) for a in g1 + s1)
        print("tp2 vs tp1: first tokens %d/3, all tokens %d/%d" % (first, same, total), flush=True)
        assert first == 3 and same >= 0.6 * total
    dist.barrier()
    print("rank %d tp worker ok" % rank, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
