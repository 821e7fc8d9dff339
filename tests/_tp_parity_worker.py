"""Worker for tests/test_tp_parity_gpu.py: WORLD_SIZE ranks sharing ONE GPU (gloo; the custom all-reduce's
IPC buffers map the same device).  Every rank builds the same HF-layout random checkpoint (real Llama-3-8B
dims, 2 layers, non-unit gains: tests/test_forward_parity_gpu.py) and rank 0 compares the gathered logits
of the tensor-parallel paths with the independent textbook fp32 forward, with the TP=1 bounds:

  A. TP engine, one packed prefill through the SEQUENCE-PARALLEL path (row-sharded residual, reduce-
     scatter + all-gather), then greedy decode through the TP push (row-parallel GEMM epilogues
     all-reducing their own tiles, bf16 payload) and the vocab-parallel sampler;
  B. CONTEXT-PARALLEL prefill of one prompt over the ranks' full engines (zigzag slices, per-layer K/V
     exchange) handed to the TP engine (each rank keeps its KV heads), then TP decode.

Environment: MODEL (llama3-8b | llama3-70b, 2 layers), WDTYPE (bf16 | fp8).  fp8 weights (the config-5
aggregator's format: OCP e4m3fn, per-row scales, quantised per TP shard by the loader) are compared with the
textbook forward of the DEQUANTISED SHARDS every rank holds, rebuilt on rank 0 exactly as the loader slices,
folds and quantises them (unit gains: nothing to fold), with the TP=1 fp8 bounds; the CP part (B) needs a
full-weight engine per rank and runs for bf16 only."""
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
from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight, interleave_gate_up, split_gate_up  # noqa: E402


def unit_gain_checkpoint(cfg, seed):
    """P._checkpoint with every RMSNorm gain 1 (the fp8 comparison needs no gain folding)."""
    d = P._checkpoint(cfg, seed)
    for k in d:
        if k.endswith("norm.weight") or k.endswith("layernorm.weight"):
            d[k] = torch.ones_like(d[k])
    return d


def fp8_shard_reference(cfg, ckpt, world, dev):
    """HF-layout fp32 tensors of the model the TP ranks actually run: for every rank, its weight shards sliced
    as engine/weights.py load_hf slices them, quantised per shard with Fp8Weight.quantize on the device (as the
    loader does), dequantised and put back in place."""
    hd, H, F = cfg.head_dim, cfg.hidden, cfg.ffn
    qs, ks, f = cfg.n_heads * hd // world, cfg.n_kv_heads * hd // world, F // world
    def dq(t):
        return Fp8Weight.quantize(t.to(dev, torch.bfloat16).contiguous()).dequant(torch.float32).cpu()

    # the LM head is fp8 too (row scales: the vocab shards quantise exactly as the whole matrix does)
    ref = {"model.embed_tokens.weight": ckpt["model.embed_tokens.weight"],
           "model.norm.weight": ckpt["model.norm.weight"], "lm_head.weight": dq(ckpt["model.embed_tokens.weight"])}

    for i in range(cfg.n_layers):
        p = "model.layers.%d." % i
        wq, wk, wv = (ckpt[p + "self_attn.%s_proj.weight" % n] for n in ("q", "k", "v"))
        wo, wd = ckpt[p + "self_attn.o_proj.weight"], ckpt[p + "mlp.down_proj.weight"]
        wg, wu = ckpt[p + "mlp.gate_proj.weight"], ckpt[p + "mlp.up_proj.weight"]
        q, k, v, o, g, u, d = [], [], [], [], [], [], []
        for r in range(world):
            qkv = dq(torch.cat([wq[r * qs:(r + 1) * qs], wk[r * ks:(r + 1) * ks], wv[r * ks:(r + 1) * ks]]))
            q.append(qkv[:qs]), k.append(qkv[qs:qs + ks]), v.append(qkv[qs + ks:])
            o.append(dq(wo[:, r * qs:(r + 1) * qs]))
            gg, uu = split_gate_up(dq(interleave_gate_up(wg[r * f:(r + 1) * f], wu[r * f:(r + 1) * f])).t())
            g.append(gg.t()), u.append(uu.t())
            d.append(dq(wd[:, r * f:(r + 1) * f]))
        ref[p + "self_attn.q_proj.weight"], ref[p + "self_attn.k_proj.weight"] = torch.cat(q), torch.cat(k)
        ref[p + "self_attn.v_proj.weight"], ref[p + "self_attn.o_proj.weight"] = torch.cat(v), torch.cat(o, 1)
        ref[p + "mlp.gate_proj.weight"], ref[p + "mlp.up_proj.weight"] = torch.cat(g), torch.cat(u)
        ref[p + "mlp.down_proj.weight"] = torch.cat(d, 1)
        ref[p + "input_layernorm.weight"] = ckpt[p + "input_layernorm.weight"]
        ref[p + "post_attention_layernorm.weight"] = ckpt[p + "post_attention_layernorm.weight"]
    return ref


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
    model, wdt = os.environ.get("MODEL", "llama3-8b"), os.environ.get("WDTYPE", "bf16")
    cfg = get_model_config(model, n_layers=2)
    fp8 = wdt == "fp8"
    ckpt = unit_gain_checkpoint(cfg, 11) if fp8 else P._checkpoint(cfg, 11)
    index = {k: "mem" for k in ckpt}
    W._open_shards = lambda path: (index, {"mem": P._Mem(ckpt)})
    tp = LLMEngine(cfg, device="cuda:0", weights_path="mem", use_graphs=False, max_num_seqs=8, sync_every=64,
                   max_model_len=4096, kv_pages=256, tp_rank=rank, tp_size=world, tp_group=None, weight_dtype=wdt)
    assert tp.model.custom_ar is not None and tp.model.tp_sampling and tp.model.sequence_parallel
    rep = tp.model.custom_ar.selftest_report()
    print("rank %d p2p self-test: %s" % (rank, rep), flush=True)
    assert all(rep[p] in ("ok", "n/a") for p in tp.model.custom_ar.PATHS), rep  # self-test at these shapes
    ref_ckpt, tol, min_exact = ckpt, P.BF16_TOL, 0.9
    if fp8:
        ref_ckpt = fp8_shard_reference(cfg, ckpt, world, dev) if rank == 0 else None
        tol, min_exact = P.FP8_TOL, P.FP8_MIN_EXACT
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
        res["A"] = P._compare(cfg, ref_ckpt, prompts, toks, rows, tol, dev, min_exact=min_exact)
    if fp8:
        if rank == 0:
            print("tp%d %s fp8 parity: SP prefill (fp8 GEMMs, two-term QKV rows gathered as e4m3) + W8A16 "
                  "TP-push decode max rel err %.4f top-1 %d/%d (%d pushes); self-test %s"
                  % ((world, model) + res["A"] + (pushed, rep)), flush=True)
        dist.barrier()
        print("rank %d tp parity ok" % rank, flush=True)
        dist.destroy_process_group()
        return

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
    try:
        main()
    except BaseException:  # the launcher's report keeps only the tail of 8 ranks' stderr: say it on stdout
        import traceback
        print("RANKFAIL rank %s: %s" % (os.environ.get("RANK"), traceback.format_exc().replace("\n", " | ")),
              flush=True)
        raise
