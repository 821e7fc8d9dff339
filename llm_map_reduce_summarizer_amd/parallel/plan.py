"""Per-stage parallelism planner: data-parallel replicas vs. one tensor-parallel engine.

Every stage of the summarizer is a batch of independent generations pinned to ``max_new`` tokens
(map: one per chunk; reduce level 1: one per batch of summaries; final: one).  On N GPUs a stage can
run either

* **DP**: the requests are split over N replicas of the model (one per GPU), or
* **TP**: every request runs on ONE engine whose weights and KV heads are sharded over the N GPUs
  (two all-reduces per layer on the custom P2P kernel, parallel/custom_ar.py).

Decode is a 1000-step serial loop whose step time is bounded by streaming the weights plus the
batch's KV cache from HBM, so DP does not shorten it (each replica still streams the full 15 GB of
weights per step) while TP divides both streams by N at the price of the per-layer all-reduce
latency.  Prefill is compute-bound: DP divides it by N for free, TP adds RCCL all-reduces of the
activations.  Which is faster depends on the batch, the context and the all-reduce latency of the
node, so the choice is a cost model whose hardware constants are *measured*:

* ``hbm_bw``, ``step_floor_s``, ``tp_row_s``, ``tp_shard_s``, ``fp8_row_s``, ``fp8_floor_s``: one MINIMAX fit
  (tools/fit_hwmodel.py) over the round-6 decode steps of TP=1 and of one rank's TP=2/4/8 shard with the TP
  kernel sequence over a group of one rank (TP push in the row-parallel GEMM epilogues), Llama-3-8B bf16 at
  B=1/10/39 x 4k and Llama-3-70B fp8 at TP=1 / TP=8 (profiles/r6_decode_steps_final.jsonl):
  t = (W + B ctx kv) / TP / 6.02 TB/s + L/32 x (0.858 ms + 7.43 us x B log2(TP) + [TP > 1] 0.384 ms / TP
  + [fp8] (86.8 us + 5.28 us x B)), every point within 3.9 % (tests/test_plan.py pins that; the fp8 per-row
  term fell from 46.4 us with the split-K SwiGLU of the narrow fp8 gate_up);
* ``prefill_flops``: the engine's prefill rate in the 10 h bench (~76k tok/s of Llama-3-8B);
* ``ar_lat_s`` / ``ar_lat_row_s`` and ``ar_bw``: timed at start-up on the job's own GPUs (the fused
  all-reduce inside a replayed hipGraph at 1 and 64 rows against the same kernel over a group of one
  rank -- the cross-GPU part the shard fit above does not contain: a latency and a per-row link cost;
  one RCCL all-reduce of a prefill-sized activation), MAX-reduced over the ranks so every rank takes
  the same decision.

A TP stage may also prefill *disaggregated* (``handoff``): data-parallel on every rank's full
TP=1 engine, then one all-to-all moves each prompt's KV heads to their TP owner -- the KV of a
prompt is 128 KiB/token for Llama-3-8B, far less than the 2 x 32 activation all-reduces of
8 KiB/token each that a TP prefill forward needs.  A single prompt is prefilled *context-parallel*
instead (zigzag slices on every rank, per-layer K/V all-gather; every rank ends with the whole KV).

The reference has a single form of parallelism, a semaphore-bounded fan-out of HTTPS calls
(reference llm_executor.py:133-147); this module is the MI355X replacement for choosing how the
fan-out maps onto GPUs.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, replace
from typing import Dict, List, Sequence


@dataclass(frozen=True)
class HWModel:
    hbm_bw: float = 6.02e12         # bytes/s streamed by the decode GEMM + attention kernels
    step_floor_s: float = 0.858e-3  # fixed per-step cost of the decode graph (kernel latencies), per 32 layers
    tp_shard_s: float = 0.384e-3    # a TP shard's extra fixed cost per 32 layers, divided by TP ...
    tp_row_s: float = 7.43e-6       # ... plus this per decode row per log2(TP) (few-kv-head attention is latency-bound)
    fp8_floor_s: float = 86.8e-6    # W8A16 decode kernels: extra fixed cost per 32 layers ...
    fp8_row_s: float = 5.28e-6      # ... and per decode row (the e4m3 -> bf16 conversion grows with the rows)
    prefill_flops: float = 1.1e15   # effective prefill FLOP/s (MFMA GEMMs + flash attention)
    ar_lat_s: float = 20e-6         # one decode all-reduce (custom P2P kernel), measured at start-up ...
    ar_lat_row_s: float = 0.0       # ... plus this per decode row (the push sends every row to every peer)
    ar_bw: float = 100e9            # RCCL all-reduce algorithm bandwidth (bytes/s), measured at start-up
    tp_ok: bool = True              # False when the TP engine has no graph-safe all-reduce


@dataclass(frozen=True)
class ModelDims:
    weight_bytes: float
    kv_bytes_per_token: float
    flops_per_token: float
    n_layers: int
    hidden: int
    fp8: bool = False  # W8A16 decode kernels (1-byte weights)

    @classmethod
    def of(cls, cfg, weight_bytes_per_param: float = 2.0) -> "ModelDims":
        n = cfg.n_params()
        emb = cfg.vocab_size * cfg.hidden  # the embedding table is gathered, not streamed
        return cls(weight_bytes=(n - emb) * weight_bytes_per_param, kv_bytes_per_token=cfg.kv_bytes_per_token(),
                   flops_per_token=2.0 * (n - 2 * emb), n_layers=cfg.n_layers, hidden=cfg.hidden,
                   fp8=weight_bytes_per_param < 2.0)


def decode_step_s(d: ModelDims, hw: HWModel, batch: int, ctx: float, tp: int) -> float:
    """One decode step of ``batch`` sequences at mean context ``ctx`` on a TP=``tp`` engine."""
    if batch <= 0:
        return 0.0
    stream = (d.weight_bytes + batch * ctx * d.kv_bytes_per_token) / tp / hw.hbm_bw
    floor = (hw.step_floor_s + (hw.tp_shard_s / tp if tp > 1 else 0.0) + hw.tp_row_s * batch * math.log2(tp)
             + ((hw.fp8_floor_s + hw.fp8_row_s * batch) if d.fp8 else 0.0)) * d.n_layers / 32.0
    comm = (2 * d.n_layers + 1) * (hw.ar_lat_s + hw.ar_lat_row_s * batch) if tp > 1 else 0.0
    return stream + floor + comm


from ..engine.config import PREFILL_CHUNK  # noqa: E402 -- the engine's default slice (engine/engine.py)


def prefill_s(d: ModelDims, hw: HWModel, tokens: int, tp: int, longest: int = 0,
              chunk: int = PREFILL_CHUNK) -> float:
    """TP=``tp`` prefill of ``tokens`` rows whose longest prompt has ``longest`` tokens (default: one
    prompt).  The engine cuts prompts into end-aligned ``chunk``-token slices (n passes for the longest),
    and a TP prefill of n > 1 passes runs layer-major with every pass's all-reduces under the next pass's
    GEMMs (engine/model.py prefill_passes): the longer of compute and communication, plus the shorter
    one's last-pass share."""
    compute = tokens * d.flops_per_token / tp / hw.prefill_flops
    if tp == 1:
        return compute
    comm = 2 * d.n_layers * tokens * d.hidden * 2 / hw.ar_bw
    n = max(1, -(-(longest or tokens) // chunk)) if chunk else 1
    return max(compute, comm) + min(compute, comm) / n


def _lpt(costs: Sequence[int], bins: int) -> List[List[int]]:
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load, out = [0] * bins, [[] for _ in range(bins)]
    for i in order:
        b = min(range(bins), key=lambda j: (load[j], j))
        out[b].append(i)
        load[b] += costs[i]
    return out


def cp_prefill_s(d: ModelDims, hw: HWModel, tokens: int, world: int) -> float:
    """Context-parallel prefill of ONE prompt over ``world`` ranks (engine.prefill_export_cp): each rank
    runs 1 / world of the prompt (zigzag slices, balanced causal attention) through all layers and every
    layer's K/V rows are all-gathered, so each rank receives (world - 1) / world of the prompt's KV."""
    compute = prefill_s(d, hw, tokens, 1) / world
    return compute + tokens * d.kv_bytes_per_token * (world - 1) / world / hw.ar_bw


def handoff_prefill_s(d: ModelDims, hw: HWModel, prompt_lens: Sequence[int], world: int) -> float:
    """Disaggregated prefill of a TP=``world`` stage: the prompts are prefilled data-parallel on the
    ranks' full (TP=1) engines, then every rank sends each TP peer its KV heads (one all-to-all).  One
    prompt (the final reduce) is prefilled context-parallel over all the ranks instead (cp_prefill_s)."""
    if len(prompt_lens) == 1 and world > 1 and prompt_lens[0] >= 2 * world:
        return cp_prefill_s(d, hw, prompt_lens[0], world)
    bins = _lpt(list(prompt_lens), world)
    compute = max(prefill_s(d, hw, sum(prompt_lens[i] for i in b), 1) for b in bins)
    kv = sum(prompt_lens) * d.kv_bytes_per_token
    per_rank = kv / world * (world - 1) / world  # what one rank sends (and receives)
    return compute + per_rank / hw.ar_bw


def stage_seconds(d: ModelDims, hw: HWModel, prompt_lens: Sequence[int], max_new: Sequence[int], tp: int,
                  world: int, handoff: bool = False) -> float:
    """Estimated wall-clock of one stage on ``world`` GPUs as ``world // tp`` replicas of TP=``tp``
    (requests LPT-balanced over replicas, every generation pinned to its ``max_new``).  ``handoff``:
    a TP stage may prefill through handoff_prefill_s inside its own TP group (the cheaper of the two),
    whatever the group size -- so TP=world is not favoured over intermediate TP x DP layouts."""
    if not prompt_lens:
        return 0.0
    dp = max(1, world // tp)
    bins = _lpt([p + m for p, m in zip(prompt_lens, max_new)], dp)
    use_handoff = handoff and tp > 1
    worst = 0.0
    for idx in bins:
        if not idx:
            continue
        pl = [prompt_lens[i] for i in idx]
        mn = [max_new[i] for i in idx]
        t = prefill_s(d, hw, sum(pl), tp, max(pl))
        if use_handoff:  # the cheaper of the TP forward and the disaggregated prefill
            t = min(t, handoff_prefill_s(d, hw, pl, tp))
        # sequences retire as they reach their max_new: walk the decode in segments of equal batch
        order = sorted(range(len(idx)), key=lambda k: mn[k])
        done = 0
        for k in order:
            steps = mn[k] - done
            if steps > 0:
                live = [j for j in range(len(idx)) if mn[j] > done]
                ctx = sum(pl[j] for j in live) / len(live) + done + steps / 2.0
                t += steps * decode_step_s(d, hw, len(live), ctx, tp)
                done = mn[k]
        worst = max(worst, t)
    return worst


def choose(d: ModelDims, hw: HWModel, prompt_lens: Sequence[int], max_new: Sequence[int], world: int,
           candidates: Sequence[int] = (), handoff: bool = False) -> Dict[str, object]:
    """Best TP degree for a stage among ``candidates`` (default: 1 and ``world``)."""
    cands = list(candidates) or ([1, world] if world > 1 else [1])
    if not hw.tp_ok:
        cands = [1]
    est = {tp: stage_seconds(d, hw, prompt_lens, max_new, tp, world, handoff) for tp in cands}
    best = min(cands, key=lambda tp: (est[tp], tp))
    out = {"tp": best, "estimates_s": {str(k): round(v, 3) for k, v in est.items()}}
    if best > 1 and best == world:
        # disaggregated prefill only where it beats the TP forward: many prompts split over the ranks;
        # one prompt (the final reduce) context-parallel, whose per-layer K/V all-gather moves a quarter
        # of the TP forward's activation all-reduce bytes (Llama-3: 4 vs 16 KiB per token and layer)
        out["handoff"] = bool(handoff) and handoff_prefill_s(d, hw, prompt_lens, world) < \
            prefill_s(d, hw, sum(prompt_lens), world, max(prompt_lens))
    return out


def with_measurements(hw: HWModel, ar_lat_s=None, ar_bw=None, tp_ok=None, ar_lat_row_s=None) -> HWModel:
    kw = {}
    if ar_lat_s is not None:
        kw["ar_lat_s"] = float(ar_lat_s)
    if ar_lat_row_s is not None:
        kw["ar_lat_row_s"] = float(ar_lat_row_s)
    if ar_bw is not None:
        kw["ar_bw"] = float(ar_bw)
    if tp_ok is not None:
        kw["tp_ok"] = bool(tp_ok)
    return replace(hw, **kw)
