#!/usr/bin/env python3
"""Headline benchmark: end-to-end map-reduce summarisation of a 10 h
transcript with Llama-3-8B (BASELINE.json: "chunks/sec (whole node) +
end-to-end wall-clock, 10h transcript, Llama-3-8B").

One step = the full pipeline of the reference's ``TranscriptSummarizer.
summarize`` (reference main.py:82-257) on a synthetic 10 h transcript:
preprocess -> chunk (4000-token budget) -> map (one 1000-token summary per
chunk, temperature 0.3) -> hierarchical reduce (level-1 batches + final pass,
temperature 0.2), all generation on the local engine (random-init
Llama-3-8B weights, bf16).  Chunks are data-parallel over the N ranks
(one process per GPU, RCCL all-gather of the summaries); every rank runs
the same SPMD pipeline.

value = chunks / end-to-end seconds (whole job; the transcript is fixed, so
scaling is strong).  ms_per_step = end-to-end wall-clock of one summary.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N

``python bench.py --gpus N`` (N > 1) without a torchrun environment launches the N ranks itself (a child
``torch.distributed.run``), so both forms measure N ranks; the JSON reports the world size and backend
the process group actually saw (``ranks_seen``, ``backend``) and a hash of the final summary.
"""

from __future__ import annotations

import argparse
import asyncio
import hashlib
import json
import logging
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# RCCL and the custom all-reduce share device memory across processes through dmabuf IPC, the only
# IPC mode the host driver supports; set before anything initialises HIP
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

BASELINE_VALUE = None  # the reference publishes no number


def _parallelism(provider, world: int) -> str:
    """e.g. "dp1", or per stage "map:tp2xdp4,reduce_l1:dp8,reduce_final:tp8" (tpK = one engine sharded
    over K GPUs, dpK = K data-parallel replicas, tpKxdpD = D replicas of a TP=K engine)."""
    plan = getattr(provider, "stage_plan", {}) or {}
    if world == 1 or not plan:
        return "dp%d" % world

    def lay(k: int) -> str:
        return "dp%d" % world if k <= 1 else ("tp%d" % k if k == world else "tp%dxdp%d" % (k, world // k))
    return ",".join("%s:%s" % (s, lay(int(c["tp"]))) for s, c in plan.items())


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n: int) -> int:
    """``--gpus N > 1`` without a torchrun environment: start ``torch.distributed.run`` with N ranks as a
    CHILD process (never an exec: nothing here has touched the GPU, and none of it may before the ranks
    own it), let rank 0's JSON line through, and exit with the child's code.  So ``python bench.py
    --gpus 8`` measures 8 ranks instead of silently timing one process N times."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ, MRSUM_BENCH_SELF_LAUNCHED="1")
    print("bench: --gpus %d without WORLD_SIZE: launching %d ranks (%s)" % (n, n, " ".join(cmd[:8])),
          file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--hours", type=float, default=10.0)
    ap.add_argument("--max-new-tokens", type=int, default=1000)
    ap.add_argument("--chunk-tokens", type=int, default=4000)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--stop-at-eos", action="store_true",
                    help="honour EOS (default: pin every generation to --max-new-tokens so the timed work is fixed)")
    ap.add_argument("--parallel", default=os.environ.get("MRSUM_PARALLEL", "auto"),
                    help="dp: every stage data-parallel over the ranks; reduce_tp: map data-parallel, reduce stages "
                         "tensor-parallel over all ranks; tp: every stage on one engine sharded over all ranks; "
                         "tpK: TP=K x DP=N/K for every stage; a per-stage layout such as "
                         "map:tp2,reduce_l1:tp4,reduce_final:tp8; auto: per stage, the cheapest TP degree (divisors "
                         "of N) under parallel/plan.py's cost model fed with the all-reduce latency and bandwidth "
                         "measured on these GPUs at start-up")
    ap.add_argument("--no-hierarchical", action="store_true",
                    help="single-pass reduce over every summary (use a long-context model, e.g. llama3.1-8b)")
    ap.add_argument("--stream-reduce", action="store_true",
                    help="start each level-1 reduce batch as soon as its chunks are summarised (no map barrier)")
    ap.add_argument("--kv-dtype", choices=["bf16", "fp8v"], default="bf16",
                    help="KV cache format; fp8v (V rows e4m3 with power-of-two row scales, K bf16) is a LABELLED "
                         "variant: the headline is bf16 KV")
    ap.add_argument("--reduce-batch-tokens", type=int, default=None,
                    help="rehearsal knob: the aggregator's token budget per reduce call (default 6000, with 1000 "
                         "reserved); a small value forces a multi-level reduce with short pinned summaries "
                         "(labelled variant, never the headline)")
    ap.add_argument("--profile", default=None, metavar="DIR", help="torch.profiler trace of the timed steps")
    ap.add_argument("--log-level", default="WARNING")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _self_launch(args.gpus)
    # a hung collective must end the job well inside the driver's slot (a rank waits for its peers at
    # most one 1000-token generate of the slowest stage: seconds)
    os.environ.setdefault("MRSUM_DIST_TIMEOUT", "240")

    logging.basicConfig(level=getattr(logging, args.log_level.upper()), stream=sys.stderr,
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    import torch

    from llm_map_reduce_summarizer_amd.config import LLMConfig
    from llm_map_reduce_summarizer_amd.engine.provider import LocalEngineProvider
    from llm_map_reduce_summarizer_amd.parallel import dist as pdist
    from llm_map_reduce_summarizer_amd.pipeline.executor import LLMExecutor
    from llm_map_reduce_summarizer_amd.pipeline.orchestrator import TranscriptSummarizer
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript

    pdist.init_distributed_from_env()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    if torch.cuda.is_available():  # one rank per GPU (modulo: rehearsal runs share one GPU over gloo)
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))

    cfg = LLMConfig(MAX_TOKENS=args.max_new_tokens, TEMPERATURE=0.3, REDUCE_TEMPERATURE=0.2)
    provider = LocalEngineProvider(args.model, cfg, use_graphs=not args.no_graphs, ignore_eos=not args.stop_at_eos,
                                   parallel=args.parallel, kv_dtype=args.kv_dtype)
    executor = LLMExecutor(config=cfg, provider_obj=provider)
    agg_opts = ({"max_tokens_per_batch": args.reduce_batch_tokens, "reserved_tokens": 0}
                if args.reduce_batch_tokens else None)
    summarizer = TranscriptSummarizer(executor=executor, max_tokens_per_chunk=args.chunk_tokens,
                                      hierarchical_aggregation=not args.no_hierarchical,
                                      stream_reduce=args.stream_reduce, aggregator_options=agg_opts)
    transcript = synthetic_transcript(args.hours, seed=0)
    # weight init, KV allocation, planner measurements and the decode graphs of every batch bucket a
    # stage of this transcript can use: engine start-up, outside the timed region
    n_chunks_est = max(64, int(args.hours * 8))
    provider.warm(capture_batch=n_chunks_est if not args.no_graphs else None)

    def one():
        return asyncio.run(summarizer.summarize(transcript))

    for i in range(args.warmup):
        t = time.perf_counter()
        rep = one()
        if rank == 0:
            print("warmup %d: %.2f s, %d chunks" % (i, time.perf_counter() - t, rep["chunks"]), file=sys.stderr)

    pdist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    from llm_map_reduce_summarizer_amd.utils.profiling import maybe_profile
    work0 = dict(provider.work)
    stages0 = {k: dict(v) for k, v in provider.stage_seconds.items()}
    t0 = time.perf_counter()
    reports = []
    with maybe_profile(args.profile, rank):
        for i in range(args.steps):
            ts = time.perf_counter()
            reports.append(one())
            if rank == 0:  # progress on stderr (a 20-step run is minutes long); stdout keeps the one JSON line
                print("step %d: %.2f s" % (i, time.perf_counter() - ts), file=sys.stderr, flush=True)
    pdist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    elapsed = pdist.all_reduce_max(time.perf_counter() - t0)

    # what the process group itself saw (not what the flags claim)
    if pdist.is_initialized():
        import torch.distributed as tdist
        ranks_seen, backend = tdist.get_world_size(), tdist.get_backend()
    else:
        ranks_seen, backend = 1, "none"
    # the timed work must be the pinned work: every generation of every timed step produced exactly its
    # max_new_tokens and none failed (the provider counts from the all-gathered results, same on every rank)
    work = {k: provider.work[k] - work0[k] for k in work0}
    work_ok = work["errors"] == 0 and (args.stop_at_eos or work["completion_tokens"] == work["requested_tokens"])
    rep = reports[-1]
    ms = elapsed / max(1, args.steps) * 1000.0
    # the P2P all-reduce paths of every TP engine this job built (start-up self-test at the model's shapes,
    # per path) and how many generates fell back to RCCL after a timed-out P2P wait
    pstats = provider.stats()
    tp_engs = dict(pstats.get("tp_engines", {}))
    if "tp_engine" in pstats:
        tp_engs[str(world)] = pstats["tp_engine"]
    p2p = {("tp%s" % k): e.get("p2p_selftest") for k, e in sorted(tp_engs.items())}
    ar_recoveries = sum(int(e.get("custom_ar_recoveries", 0)) for e in tp_engs.values())
    n_chunks = rep["chunks"]
    value = n_chunks / (ms / 1000.0)
    # per stage and timed step: the planner's prediction at the layout the stage ran next to its measured wall
    # time (parallel/plan.py stage_seconds vs the provider's generate calls; rank 0's clock), and the measured
    # cross-GPU cost of one decode all-reduce per path and TP degree -- what a first multi-GPU run needs to
    # tell which stage missed its model and whether the xGMI push latency is the reason
    stages = {}
    for st, r in provider.stage_seconds.items():
        r0 = stages0.get(st, {"calls": 0, "predicted_s": 0.0, "measured_s": 0.0})
        n = max(1, args.steps)
        pred = None if r.get("predicted_s") is None or r0.get("predicted_s") is None else \
            round((r["predicted_s"] - r0["predicted_s"]) / n, 6)
        stages[st] = {"tp": r["tp"], "calls_per_step": (r["calls"] - r0["calls"]) / n, "predicted_s": pred,
                      "measured_s": round((r["measured_s"] - r0["measured_s"]) / n, 4)}
    eng = rep.get("engine", {})
    out = {
        "metric": "chunks/sec (whole node) + end-to-end wall-clock, 10h transcript, Llama-3-8B"
                  + ("" if args.model == "llama3-8b" and args.hours == 10.0 and not args.no_hierarchical
                     and not args.stream_reduce and args.kv_dtype == "bf16" and not args.reduce_batch_tokens
                     else " [variant: %s, %gh%s%s%s%s]" % (args.model, args.hours,
                                                         ", single-pass reduce" if args.no_hierarchical else "",
                                                         ", streamed level-1 reduce" if args.stream_reduce else "",
                                                         (", reduce batches of %d tokens" % args.reduce_batch_tokens)
                                                         if args.reduce_batch_tokens else "",
                                                         {"fp8": ", fp8 KV cache", "fp8v": ", fp8 V cache (bf16 K)"}
                                                         .get(args.kv_dtype, ""))),
        "value": round(value, 4),
        "unit": "chunks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 2),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
        "dtype": "bf16",
        "kv_dtype": args.kv_dtype,
        "data": ("synthetic %gh transcript (utils/synth.py, seed 0); random-init weights; every generation "
                 "pinned to max_new_tokens%s" % (args.hours, " (EOS honoured)" if args.stop_at_eos else "")),
        "config": {"model": args.model, "global_batch": n_chunks, "seq_len": args.chunk_tokens,
                   "parallelism": _parallelism(provider, world),
                   "max_new_tokens": args.max_new_tokens,
                   "transcript_hours": args.hours},
        "ranks_seen": ranks_seen,
        "summary_sha16": hashlib.sha256(rep.get("summary", "").encode("utf-8")).hexdigest()[:16],
        "backend": backend,
        "e2e_wall_s": round(ms / 1000.0, 3),
        "phases_s": {k: round(v, 3) for k, v in rep.get("timings", {}).items()},
        "map_chunks_per_s": round(rep["chunks_per_second"] or 0.0, 3),
        "reduce_plan": rep.get("reduce_plan"),
        "tokens_used": rep.get("tokens_used"),
        "timed_work": dict(work, pinned_ok=work_ok),
        "p2p_selftest": p2p or None,
        "stages": stages,
        "p2p_latency_us": pstats.get("p2p_latency") or None,
        "planner_hw": pstats.get("planner_hw"),
        "ar_recoveries": ar_recoveries,
        "engine_rank0": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in eng.items()},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    rc = 0
    if not work_ok:
        print("bench: timed work is not the pinned work: %d of %d requested tokens generated, %d failed requests"
              % (work["completion_tokens"], work["requested_tokens"], work["errors"]), file=sys.stderr)
        rc = 3
    # the measurement is complete and printed: a teardown error must not turn it into a failed run
    try:
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        print("bench: process-group teardown raised after the result was printed: %r" % (e,), file=sys.stderr)
    return rc


if __name__ == "__main__":
    # one exit path with the CLI: flush, then os._exit for a rank of a multi-process job (no backend C++
    # destructors after the printed result), sys.exit otherwise (parallel/dist.py exit_process)
    code = main()
    from llm_map_reduce_summarizer_amd.parallel import dist as _pdist
    _pdist.exit_process(code)
