#!/usr/bin/env python3
"""Fit parallel/plan.py HWModel's decode constants to measured decode steps.

    python tools/fit_hwmodel.py profiles/r3_decode_steps_push.jsonl

Each line: {"B", "ctx", "tp_shard", "decode_ms_per_step"} (tools/bench_decode.py; TP shards measured on one
GPU with the TP kernel sequence).  The model is linear in (1 / hbm_bw, step_floor, tp_floor, tp_row):

    t = (W + B ctx kv) / TP / hbm_bw + step_floor + [TP > 1] tp_floor + tp_row B log2(TP)

so the fit is a relative-error weighted least squares; prints the constants and every point's error."""
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llm_map_reduce_summarizer_amd.engine.config import get_model_config
    from llm_map_reduce_summarizer_amd.parallel import plan
    rows = [json.loads(l) for p in sys.argv[1:] for l in open(p) if l.startswith("{")]
    d = plan.ModelDims.of(get_model_config("llama3-8b"))
    # mean over repeated rounds of one point
    pts = {}
    for r in rows:
        pts.setdefault((r["tp_shard"], r["B"], r["ctx"]), []).append(r["decode_ms_per_step"] * 1e-3)
    keys = sorted(pts)
    A, y = [], []
    for tp, B, ctx in keys:
        t = sum(pts[(tp, B, ctx)]) / len(pts[(tp, B, ctx)])
        stream = (d.weight_bytes + B * (ctx + 128) * d.kv_bytes_per_token) / tp
        A.append([stream / t, 1.0 / t, (1.0 if tp > 1 else 0.0) / t, B * math.log2(tp) / t])
        y.append(1.0)
    x, *_ = np.linalg.lstsq(np.array(A), np.array(y), rcond=None)
    inv_bw, c0, c1, c2 = x
    hw = plan.HWModel(hbm_bw=1.0 / inv_bw, step_floor_s=c0, tp_floor_s=c1, tp_row_s=c2, ar_lat_s=0.0)
    print("hbm_bw %.3g B/s  step_floor %.3g s  tp_floor %.3g s  tp_row %.3g s" % (hw.hbm_bw, c0, c1, c2))
    worst = 0.0
    for tp, B, ctx in keys:
        t = sum(pts[(tp, B, ctx)]) / len(pts[(tp, B, ctx)])
        est = plan.decode_step_s(d, hw, B, ctx + 128, tp)
        worst = max(worst, abs(est - t) / t)
        print("tp %d B %2d  measured %.3f ms  model %.3f ms  %+.1f %%" % (tp, B, t * 1e3, est * 1e3, 100 * (est - t) / t))
    print("worst %.1f %%" % (100 * worst))


if __name__ == "__main__":
    main()
