#!/usr/bin/env python3
"""Fit parallel/plan.py HWModel's decode constants to measured decode steps (minimax relative error).

    python tools/fit_hwmodel.py profiles/r6_decode_steps.jsonl

Each line: {"model", "dtype", "B", "ctx", "tp_shard", "decode_ms_per_step"} (tools/bench_decode.py; TP shards
measured on one GPU with the TP kernel sequence over a group of one rank; "model" / "dtype" default to
llama3-8b / bf16).  The model is linear in its constants:

    t = (W + B ctx kv) / TP / hbm_bw
        + L/32 (step_floor + tp_row B log2(TP) + [TP > 1] tp_shard / TP + [fp8] (fp8_floor + fp8_row B))

so the fit is a linear program minimising the worst relative error over the points (scipy linprog, all
constants >= 0); prints the constants and every point's error."""
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COLS = ("inv_bw", "step_floor_s", "tp_row_s", "tp_shard_s", "fp8_floor_s", "fp8_row_s")


def features(r):
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.parallel import plan
    fp8 = r.get("dtype") == "fp8"
    d = plan.ModelDims.of(get_model_config(r.get("model", "llama3-8b")), 1.0 if fp8 else 2.0)
    tp, B, ctx = r["tp_shard"], r["B"], r["ctx"] + 128
    L = d.n_layers / 32.0
    return [(d.weight_bytes + B * ctx * d.kv_bytes_per_token) / tp, L, L * B * math.log2(tp),
            L * (tp > 1) / tp, L * fp8, L * B * fp8]


def main():
    from scipy.optimize import linprog

    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.parallel import plan
    rows = [json.loads(l) for p in sys.argv[1:] for l in open(p) if l.startswith("{")]
    pts = {}
    for r in rows:  # mean over repeated rounds of one point
        key = (r.get("model", "llama3-8b"), r.get("dtype", "bf16"), r["tp_shard"], r["B"], r["ctx"])
        pts.setdefault(key, []).append(r)
    A, b = [], []
    for key, rs in sorted(pts.items()):
        t = sum(x["decode_ms_per_step"] for x in rs) / len(rs) * 1e-3
        row = [f / t for f in features(rs[0])]
        A.append(row + [-1.0])
        b.append(1.0)
        A.append([-v for v in row] + [-1.0])
        b.append(-1.0)
    n = len(COLS)
    res = linprog([0.0] * n + [1.0], A_ub=A, b_ub=b, bounds=[(0, None)] * (n + 1), method="highs")
    if not res.success:
        raise SystemExit("fit failed: %s" % res.message)
    x = res.x[:n]
    hw = plan.HWModel(hbm_bw=1.0 / x[0], step_floor_s=x[1], tp_row_s=x[2], tp_shard_s=x[3], fp8_floor_s=x[4],
                      fp8_row_s=x[5], ar_lat_s=0.0)
    print("hbm_bw %.3g B/s  step_floor %.3g s  tp_row %.3g s  tp_shard %.3g s  fp8_floor %.3g s  fp8_row %.3g s"
          % (hw.hbm_bw, x[1], x[2], x[3], x[4], x[5]))
    worst = 0.0
    for (model, dtype, tp, B, ctx), rs in sorted(pts.items()):
        t = sum(r["decode_ms_per_step"] for r in rs) / len(rs)
        d = plan.ModelDims.of(get_model_config(model), 1.0 if dtype == "fp8" else 2.0)
        est = plan.decode_step_s(d, hw, B, ctx + 128, tp) * 1e3
        worst = max(worst, abs(est - t) / t)
        print("%s %s tp %d B %2d ctx %5d  measured %.3f ms  model %.3f ms  %+.1f %%"
              % (model, dtype, tp, B, ctx, t, est, 100 * (est - t) / t))
    print("worst %.1f %%" % (100 * worst))


if __name__ == "__main__":
    main()
