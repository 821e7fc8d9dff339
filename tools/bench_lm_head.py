#!/usr/bin/env python3
"""Back-to-back cost of the decode LM head (ops.hip.linear, [M, 4096] x [128256, 4096]^T, bf16) at decode
batch sizes.  Rotates two weight copies (2 x 1.05 GB) so nothing stays in the 256 MiB Infinity Cache.
Imports the package from the tree given by --tree (default: this repo), so an A/B against an older
worktree uses the same driver: ``python tools/bench_lm_head.py --tree .ab_old``."""
import argparse
import json
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--tree", default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap.add_argument("--ms", default="1,10,16,39")
ap.add_argument("--n", type=int, default=128256)
ap.add_argument("--k", type=int, default=4096)
ap.add_argument("--iters", type=int, default=40)
args = ap.parse_args()
sys.path.insert(0, os.path.abspath(args.tree))

import torch  # noqa: E402

from llm_map_reduce_summarizer_amd.ops import hip  # noqa: E402

dev = "cuda:0"
ws = [torch.randn(args.n, args.k, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(2)]
for M in (int(m) for m in args.ms.split(",")):
    x = torch.randn(M, args.k, device=dev, dtype=torch.bfloat16)
    ref = (x.float() @ ws[0].float().t())
    got = hip.linear(x, ws[0]).float()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    for i in range(4):
        hip.linear(x, ws[i % 2])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(args.iters):
        hip.linear(x, ws[i % 2])
    e.record()
    e.synchronize()
    t = s.elapsed_time(e) * 1e-3 / args.iters
    nb = args.n * args.k * 2
    print(json.dumps({"tree": args.tree, "M": M, "N": args.n, "K": args.k, "us": round(t * 1e6, 1),
                      "TBps": round(nb / t / 1e12, 2), "rel_err": round(err, 5)}), flush=True)
