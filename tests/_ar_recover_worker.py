"""Worker for tests/test_custom_ar_gpu.py::test_custom_ar_timeout_recovery: 2 ranks sharing ONE GPU (gloo).
TP rank 1 sleeps 5 s on the host before its first decode window (MRSUM_FAULT_AR_DELAY), so rank 0's P2P
all-reduce waits time out (4 s bound) and set the sticky error word.  The engine must agree on the error
across the group, reset the P2P buffers and re-run the requests on the torch.distributed path: the tokens
equal a run with the custom all-reduce disabled, the error word is clear afterwards, and the next generate
runs on the reset P2P path again without a recovery."""
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
    os.environ["MRSUM_FAULT_AR_DELAY"] = "1:5"
    eng = LLMEngine(get_model_config("tiny-gqa4", init_std=0.05), device="cuda:0", max_model_len=1024,
                    max_num_seqs=8, kv_pages=64, sync_every=4, seed=5, tp_rank=rank, tp_size=2, tp_group=None)
    assert eng.model.custom_ar is not None, "no custom all-reduce on the shared GPU"
    prompts = [[128000] + [(i * 31 + j * 17) % 120000 + 5 for j in range(20 + 30 * i)] for i in range(3)]
    sp = [SamplingParams(12, 0.0, i) for i in range(3)]
    got = [o.token_ids for o in eng.generate(prompts, sp, ignore_eos=True)]
    assert eng.stats.get("custom_ar_recoveries", 0) == 1, eng.stats
    assert eng.model.custom_ar.error() == 0, "error word not cleared by the reset"
    assert all(len(t) == 12 for t in got)
    # reference: the same engine on the torch.distributed path, eager
    ar, eng.model.custom_ar, eng.use_graphs = eng.model.custom_ar, None, False
    ref = [o.token_ids for o in eng.generate(prompts, sp, ignore_eos=True)]
    eng.model.custom_ar, eng.use_graphs = ar, True
    assert got == ref, "recovered run differs from the RCCL-path run"
    # the reset P2P path works again: no recovery, no error, ranks agree
    again = [o.token_ids for o in eng.generate(prompts, sp, ignore_eos=True)]
    assert eng.stats.get("custom_ar_recoveries", 0) == 1 and ar.error() == 0
    allg = [None, None]
    dist.all_gather_object(allg, again)
    assert allg[0] == allg[1], "ranks disagree after the reset"
    same = sum(a == b for x, y in zip(again, ref) for a, b in zip(x, y))
    assert same >= 0.7 * sum(len(x) for x in ref), (again, ref)
    dist.barrier()
    print("rank %d ar recovery ok (%d/%d tokens as the RCCL path after reset)" % (rank, same, 36), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
