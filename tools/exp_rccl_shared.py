#!/usr/bin/env python3
"""Can two RCCL ranks share one GPU (rehearsal of TP collectives on a 1-GPU box)?  Eager
all_reduce, then the same all_reduce captured in a CUDA(HIP) graph and replayed.
Run: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/exp_rccl_shared.py"""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    x = torch.full((4096,), float(rank + 1), device="cuda:0")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    ok = bool((x == world * (world + 1) / 2).all())
    print("rank %d eager all_reduce ok=%s" % (rank, ok), flush=True)
    s = torch.cuda.Stream()
    y = torch.full((4096,), float(rank + 1), device="cuda:0")
    with torch.cuda.stream(s):
        dist.all_reduce(y)  # warm on the capture stream
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        dist.all_reduce(y)
    y.fill_(float(rank + 1))
    g.replay()
    torch.cuda.synchronize()
    print("rank %d graph all_reduce ok=%s" % (rank, bool((y == world * (world + 1) / 2).all())), flush=True)
    t = time.perf_counter()
    for _ in range(100):
        g.replay()
    torch.cuda.synchronize()
    print("rank %d graph all_reduce %.1f us" % (rank, (time.perf_counter() - t) * 1e4), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
