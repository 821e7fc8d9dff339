#!/usr/bin/env python3
"""Fused all-reduce + add_rmsnorm latency (parallel/custom_ar.py measure_latency) of the ranks of this
job -- run with torchrun; ranks may share one GPU (gloo process group, IPC-mapped P2P buffers).
MRSUM_AR_WT=0/1 selects the fenced / write-through publish."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_map_reduce_summarizer_amd.parallel.custom_ar import AR_WT, CustomAllReduce  # noqa: E402


def main():
    dist.init_process_group(os.environ.get("MRSUM_DIST_BACKEND", "gloo"))
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    ar = CustomAllReduce(None)
    ok = ar.self_test(iters=8)
    lat, per_row = ar.measure_latency(rows=(1, 64), hidden=4096)
    if dist.get_rank() == 0:
        print(json.dumps({"world": dist.get_world_size(), "write_through": AR_WT, "self_test": ok,
                          "lat_us": round(lat * 1e6, 2), "per_row_us": round(per_row * 1e6, 3)}), flush=True)
    ar.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
