"""Worker for tests/test_custom_ar_gpu.py::test_tp2_push_decode_one_gpu: 2 ranks sharing ONE GPU (gloo for
the handle exchange).  (1) the TP-push residual producer (ops.hip.stream_resid with a custom all-reduce
handle: the GEMM's last arriver all-reduces its tile over the group) on integer-valued operands, exact
against the rank-ordered sum; (2) a TP=2 engine with Llama-3-8B dimensions (2 layers) decoding through
the TP-push path against the same engine with the separate fused all-reduce kernel."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.engine.config import get_model_config  # noqa: E402
from llm_map_reduce_summarizer_amd.engine.engine import LLMEngine, SamplingParams  # noqa: E402
from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402
from llm_map_reduce_summarizer_amd.parallel.custom_ar import CustomAllReduce  # noqa: E402


def operands(it, r, M, N, K):
    g = torch.Generator().manual_seed(500 + 10 * it + r)
    x = torch.randint(-1, 2, (M, K), generator=g).float()
    w = torch.randint(-1, 2, (N, K), generator=g).float() * (torch.rand(N, K, generator=g) < 0.1)
    return x.to(torch.bfloat16), w.to(torch.bfloat16)


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    ar = CustomAllReduce(None, max_bytes=1 << 20)
    M, N, K = 5, 2048, 512
    for it, (wpb, S) in enumerate([(4, 4), (8, 2), (4, 1), (4, 4)]):
        g = torch.Generator().manual_seed(900 + it)
        res0 = torch.randint(-16, 17, (M, N), generator=g).to(torch.bfloat16)
        res = res0.cuda()
        x, w = operands(it, rank, M, N, K)
        ssp = hip.stream_resid(x.cuda(), w.cuda(), res, wpb, S, tp=ar.push_handle())
        torch.cuda.synchronize()
        acc = torch.zeros(M, N)
        for r in range(world):  # rank order, each rank's partial rounded to bf16 (exact: small integers)
            xr, wr = operands(it, r, M, N, K)
            acc += (xr.float() @ wr.float().t()).to(torch.bfloat16).float()
        ref = (res0.float() + acc).to(torch.bfloat16)
        assert torch.equal(res.cpu(), ref), "tp push residual it=%d (wpb %d S %d)" % (it, wpb, S)
        ss = ref.float().pow(2).reshape(M, N // (16 * wpb), 16 * wpb).sum(-1)
        assert torch.allclose(ssp.cpu(), ss, rtol=1e-5), "tp push sums of squares it=%d" % it
    assert ar.self_test(), "self-test (includes the graph-replayed TP push)"
    assert ar.error() == 0
    ar.close()

    # engine: Llama-3-8B dims, 2 layers, TP=2; decode through the TP push vs the fused all-reduce kernel
    cfg = get_model_config("llama3-8b", n_layers=2)
    kw = dict(device="cuda:0", max_model_len=512, max_num_seqs=8, kv_pages=64, seed=3, tp_rank=rank, tp_size=2,
              tp_group=None, use_graphs=True)
    prompts = [[128000] + [(i * 31 + j * 17) % 120000 + 5 for j in range(24 + 40 * i)] for i in range(3)]
    greedy = [SamplingParams(16, 0.0, i) for i in range(3)]
    push = LLMEngine(cfg, **kw)
    n0 = hip.STATS["tp_push"]  # after the engine's all-reduce self-test (which pushes too)
    gp = [o.token_ids for o in push.generate(prompts, greedy)]
    assert hip.STATS["tp_push"] > n0, "the TP-push producer never ran"
    assert push.model.custom_ar.error() == 0
    del push
    torch.cuda.empty_cache()
    os.environ["MRSUM_TP_PUSH"] = "0"
    sep = LLMEngine(cfg, **kw)
    n1 = hip.STATS["tp_push"]
    gs = [o.token_ids for o in sep.generate(prompts, greedy)]
    assert hip.STATS["tp_push"] == n1, "MRSUM_TP_PUSH=0 still pushed"
    os.environ["MRSUM_TP_PUSH"] = "1"
    allg = [None, None]
    dist.all_gather_object(allg, gp)
    assert allg[0] == allg[1], "ranks disagree under the TP push"
    same = sum(a == b for x, y in zip(gp, gs) for a, b in zip(x, y))
    total = sum(len(x) for x in gp)
    if rank == 0:
        print("tp push vs fused all-reduce kernel: first tokens %d/3, all tokens %d/%d"
              % (sum(x[0] == y[0] for x, y in zip(gp, gs)), same, total), flush=True)
    assert all(x[0] == y[0] for x, y in zip(gp, gs)) and same >= 0.7 * total
    dist.barrier()
    print("rank %d tp push ok" % rank, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
