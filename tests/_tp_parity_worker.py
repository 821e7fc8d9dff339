"""Worker for tests/test_tp_parity_gpu.py: WORLD_SIZE ranks sharing ONE GPU (gloo; the custom all-reduce's
IPC buffers map the same device).  Every rank builds the same HF-layout random checkpoint (real Llama-3-8B
dims, 2 layers, non-unit gains: tests/test_forward_parity_gpu.py) and rank 0 compares the gathered logits
of the tensor-parallel paths with the independent textbook fp32 forward, with the TP=1 bounds:

  A. TP engine, one packed prefill through the SEQUENCE-PARALLEL path (row-sharded residual, reduce-
     scatter + all-gather), then greedy decode through the TP push (row-parallel GEMM epilogues
     all-reducing their own tiles, bf16 payload) and the vocab-parallel sampler;
  B. CONTEXT-PARALLEL prefill of one prompt over the ranks' full engines (zigzag slices, per-layer K/V
     exchange) handed to the TP engine (each rank keeps its KV heads), then TP decode."""
import os
import sys

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import test_forward_parity_gpu as P  # noqa: E402
from llm_map_reduce_summarizer_amd.engine import weights as W  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.config import get_model_config  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.engine import ImportedPrefill, LLMEngine, SamplingParams  # noqa: E402
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402


def spy(eng, rec):
    orig = eng._sample

    def f(logits, view):
        rec.append(logits.float().cpu().clone())
        orig(logits, view)
    eng._sample = f


def gather_rows(rec, tp_sampling, world):
    """Every rank's recorded logits -> full-vocab rows (vocab shards concatenated in rank order)."""
    allr = [None] * world
    dist.all_gather_object(allr, rec)
    if not tp_sampling:
        return allr[0]
    return [torch.cat([allr[r][k] for r in range(world)], dim=-1) for k in range(len(rec))]


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    cfg = get_model_config("llama3-8b", n_layers=2)
    ckpt = P._checkpoint(cfg, 11)
    index = {k: "mem" for k in ckpt}
    W._open_shards = lambda path: (index, {"mem": P._Mem(ckpt)})
    tp = LLMEngine(cfg, device="cuda:0", weights_path="mem", use_graphs=False, max_num_seqs=8, sync_every=64,
                   max_model_len=4096, kv_pages=256, tp_rank=rank, tp_size=world, tp_group=None)
    assert tp.model.custom_ar is not None and tp.model.tp_sampling and tp.model.sequence_parallel
    res = {}

    # A: SP prefill + TP-push decode
    prompts = P._prompts((1, 40, 300, 129, 700), 12)
    new = 4
    rec = []
    spy(tp, rec)
    n_push = hip.STATS["tp_push"]
    outs = tp.generate(prompts, [SamplingParams(new, 0.0, 0)] * len(prompts), ignore_eos=True)
    torch.cuda.synchronize()
    pushed = hip.STATS["tp_push"] - n_push
    assert pushed > 0, "the TP push never ran"
    assert tp.model.custom_ar.error() == 0
    rows_all = gather_rows(rec, True, world)
    toks = [o.token_ids for o in outs]
    allt = [None] * world
    dist.all_gather_object(allt, toks)
    assert all(t == toks for t in allt), "TP ranks disagree on the tokens"
    if rank == 0:
        order = sorted(range(len(prompts)), key=lambda i: -len(prompts[i]))
        pre = torch.cat(rows_all[:len(rows_all) - (new - 1)])
        steps = rows_all[len(rows_all) - (new - 1):]
        rows = {i: [pre[slot].to(dev)] + [s[slot].to(dev) for s in steps] for slot, i in enumerate(order)}
        res["A"] = P._compare(cfg, ckpt, prompts, toks, rows, P.BF16_TOL, dev)

    # B: context-parallel prefill over the ranks' full engines -> TP decode
    full = LLMEngine(cfg, device="cuda:0", weights_path="mem", use_graphs=False, max_num_seqs=4, sync_every=64,
                     max_model_len=4096, kv_pages=64)
    prompt = P._prompts((1500,), 13)[0]
    frec, drec = [], []
    spy(full, frec)
    first, kv = full.prefill_export_cp(prompt, SamplingParams(1, 0.0, 0), rank, world, group=None)
    assert tp.stats.get("imported_prefills", 0) == 0
    rec.clear()
    o = tp.generate([prompt], [SamplingParams(new, 0.0, 0)], ignore_eos=True,
                    imported={0: ImportedPrefill(first, kv)})[0]
    torch.cuda.synchronize()
    assert tp.stats.get("imported_prefills", 0) == 1 and o.token_ids[0] == first
    dec = gather_rows(rec, True, world)
    firsts = [None] * world
    dist.all_gather_object(firsts, frec)
    owner = [r for r in range(world) if firsts[r]]
    assert len(owner) == 1, "exactly one rank holds the prompt's last row"
    if rank == 0:
        rows = {0: [firsts[owner[0]][0][0].to(dev)] + [d[0].to(dev) for d in dec]}
        res["B"] = P._compare(cfg, ckpt, [prompt], [o.token_ids], rows, P.BF16_TOL, dev)
        print("tp%d parity: SP prefill + TP-push decode max rel err %.4f top-1 %d/%d (%d pushes); "
              "CP prefill + hand-off + TP decode max rel err %.4f top-1 %d/%d"
              % ((world,) + res["A"] + (pushed,) + res["B"]), flush=True)
    dist.barrier()
    print("rank %d tp parity ok" % rank, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
