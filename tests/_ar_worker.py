"""Worker for tests/test_custom_ar_gpu.py: 2 ranks on ONE GPU (gloo for the handle exchange),
custom P2P all-reduce eager and replayed from a hipGraph, checked against the exact sum."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.parallel.custom_ar import CustomAllReduce  # noqa: E402


def data(rank, n, it):
    g = torch.Generator().manual_seed(1000 * it + rank)
    return torch.randint(-64, 64, (n,), generator=g).float()  # exact in fp32 sums


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    ar = CustomAllReduce(None, max_bytes=1 << 20)
    for it, n in enumerate([4, 4096, 12288, 65536, 200000]):
        x = data(rank, n, it).cuda()
        ar.all_reduce(x)
        ref = sum(data(r, n, it) for r in range(world))
        torch.cuda.synchronize()
        assert torch.equal(x.cpu(), ref), "eager n=%d" % n
    # graph: the same buffer re-filled and reduced 5 times per replay-set
    x = torch.zeros(16384, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ar.all_reduce(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ar.all_reduce(x)
    for it in range(5):
        x.copy_(data(rank, 16384, 100 + it).cuda())
        g.replay()
        torch.cuda.synchronize()
        ref = sum(data(r, 16384, 100 + it) for r in range(world))
        assert torch.equal(x.cpu(), ref), "graph replay %d" % it
    # u64 max (sampler keys): values above 2^63 must compare as unsigned
    def i64(u):
        return u - (1 << 64) if u >= 1 << 63 else u

    keys = torch.tensor([i64((rank + 1) << 62), 5 + rank, -1 if rank == 1 else 7], dtype=torch.int64, device="cuda")
    ar.max_u64_(keys)
    torch.cuda.synchronize()
    assert keys.tolist() == [i64(world << 62), 5 + world - 1, -1], keys.tolist()
    assert ar.error() == 0
    dist.barrier()
    ar.close()
    print("rank %d custom all-reduce ok" % rank, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
