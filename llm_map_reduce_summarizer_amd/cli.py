"""Command-line interface (layer L8).

Reference: ``main.py:334-480``.  Every reference flag is accepted with the same
meaning; new flags select and size the on-node engine.

    python -m llm_map_reduce_summarizer_amd --input talk.json --output out/summary.md --report
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m llm_map_reduce_summarizer_amd -i talk.json -o s.md

Differences: ``--provider`` defaults to ``$DEFAULT_PROVIDER`` (``local`` = the
MI355X engine) and also accepts ``local`` / ``mock``;
``--max-concurrent-requests`` defaults to ``$MAX_CONCURRENT_REQUESTS`` for
hosted providers (the reference's hard default of 5 made the env var dead,
SURVEY Q10) and caps in-flight sequences per rank for the local engine; logs
go to stderr through one logging setup (Q11), the summary to stdout.
"""

from __future__ import annotations

import os as _os

_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL, P2P all-reduce), before HIP init

import argparse
import asyncio
import json
import logging
import os
import sys
from pathlib import Path
from typing import List, Optional

log = logging.getLogger("mrsum.cli")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Summarize a long transcript with map-reduce on an on-node "
                                            "MI355X LLM engine (or a hosted/mock provider)")
    p.add_argument("--input", "-i", required=True, help="transcript JSON ({'segments': [...]})")
    p.add_argument("--output", "-o", help="write the summary here (parent directories are created)")
    p.add_argument("--provider", choices=["local", "mock", "openai", "anthropic"], default=None,
                   help="generation back-end (default: $DEFAULT_PROVIDER, i.e. local)")
    p.add_argument("--model", help="model name (local: llama3-8b | llama3-70b | tiny | <config.json>)")
    p.add_argument("--max-tokens-per-chunk", type=int, default=4000)
    p.add_argument("--max-concurrent-requests", type=int, default=None)
    p.add_argument("--max-segment-duration", type=int, default=120)
    p.add_argument("--no-merge", action="store_true")
    p.add_argument("--no-hierarchical", action="store_true")
    p.add_argument("--limit-segments", type=int)
    p.add_argument("--report", action="store_true", help="also write <output>.report.json")
    p.add_argument("--prompt-file")
    p.add_argument("--system-prompt-file")
    p.add_argument("--save-chunks", help="write per-chunk summaries JSON before the reduce")
    p.add_argument("--aggregator-prompt-file")
    p.add_argument("--quiet", "-q", action="store_true")
    g = p.add_argument_group("extensions")
    g.add_argument("--resume-chunks", help="load a --save-chunks file and skip the map stage")
    g.add_argument("--time-interval", type=float, default=None, help="bucket segments into N-second windows")
    g.add_argument("--no-timestamps", action="store_true", help="merged text without inline [MM:SS] marks")
    g.add_argument("--reduce-levels", type=int, default=2,
                   help="max reduce depth incl. the final pass (0 = recursive until it fits)")
    g.add_argument("--stream-reduce", action="store_true",
                   help="start each level-1 reduce batch as soon as its chunks are summarised (no map barrier)")
    g.add_argument("--chunk-overlap", type=int, default=0, help="tokens of previous-chunk context to prepend")
    g.add_argument("--position-mode", choices=["transcript", "reference"], default="transcript")
    g.add_argument("--max-new-tokens", type=int, default=None, help="override $MAX_TOKENS")
    g.add_argument("--temperature", type=float, default=None, help="override $TEMPERATURE (map)")
    g.add_argument("--fault-inject", type=float, default=0.0, help="mock provider: failure probability")
    g.add_argument("--profile", default=None, metavar="DIR",
                   help="torch.profiler trace of the run: DIR/trace_rank{r}.json + top-kernel table")
    g.add_argument("--log-level", default=os.environ.get("MRSUM_LOG_LEVEL", "INFO"))
    g.add_argument("--debug-sync", action="store_true",
                   help="debug mode: serialised kernels (AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING=1) and a "
                        "device sync + error check after every HIP kernel launch, so a fault names its op")
    e = p.add_argument_group("local engine")
    e.add_argument("--dtype", choices=["bf16", "fp8"], default=None)
    e.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (ranks per model replica)")
    e.add_argument("--seed", type=int, default=None)
    e.add_argument("--kv-fraction", type=float, default=None, help="fraction of free HBM for the KV cache")
    e.add_argument("--kv-dtype", choices=["bf16", "fp8v"], default=None,
                   help="KV cache format: bf16 (default, $ENGINE_KV_DTYPE); fp8v = V rows as OCP e4m3fn with "
                        "power-of-two row scales, K bf16 (3/4 of the KV bytes per decode step, 8 %% logit error on "
                        "the parity checkpoint; no context-parallel prefill)")
    e.add_argument("--no-graphs", action="store_true", help="disable hipGraph capture of decode steps")
    e.add_argument("--max-model-len", type=int, default=None,
                   help="context budget per request (default: 32k for llama3-*, the model window for llama3.1-*); "
                        "longer prompts are truncated with a warning")
    e.add_argument("--tokenizer", default=None, help="tiktoken-format vocabulary file (default: bundled)")
    e.add_argument("--weights", default=os.environ.get("MRSUM_WEIGHTS"),
                   help="Hugging Face Llama safetensors checkpoint (file or dir) for the map model; "
                        "default: seeded random init.  With a non-preset --model the dir's config.json is used")
    e.add_argument("--aggregator-weights", default=None, help="safetensors checkpoint of the aggregator model")
    e.add_argument("--reduce-tp", dest="reduce_tp", action="store_const", const=True, default=None,
                   help="reduce stages tensor-parallel over all ranks (map stays data-parallel); default: on with "
                        "several GPUs when the P2P all-reduce passes its self-test")
    e.add_argument("--no-reduce-tp", dest="reduce_tp", action="store_const", const=False,
                   help="keep every stage data-parallel")
    e.add_argument("--parallel", default=None,
                   help="multi-GPU policy per stage: dp replicas, one TP=world engine (tp), map dp + reduce tp "
                        "(reduce_tp), TP=K x DP=N/K (tpK), an explicit per-stage layout (e.g. "
                        "map:tp2,reduce_l1:tp4,reduce_final:tp8), or auto: the cheapest TP degree per stage under "
                        "parallel/plan.py's cost model with the all-reduce latency/bandwidth measured at start-up "
                        "(default; overrides --reduce-tp)")
    e.add_argument("--aggregator-model", default=None,
                   help="separate local model for the reduce stage (e.g. llama3-70b); default: the map model")
    e.add_argument("--aggregator-dtype", choices=["bf16", "fp8"], default=None,
                   help="weight dtype of the aggregator model (fp8 = OCP e4m3fn, per-row scales)")
    e.add_argument("--aggregator-tp", type=int, default=None, help="TP degree of the aggregator model")
    return p


def setup_logging(level: str) -> None:
    root = logging.getLogger()
    for h in list(root.handlers):
        root.removeHandler(h)
    h = logging.StreamHandler(sys.stderr)
    rank = os.environ.get("RANK")
    prefix = "[rank %s] " % rank if rank is not None and os.environ.get("WORLD_SIZE", "1") != "1" else ""
    h.setFormatter(logging.Formatter("%(asctime)s " + prefix + "%(name)s %(levelname)s %(message)s"))
    root.addHandler(h)
    root.setLevel(getattr(logging, str(level).upper(), logging.INFO))


async def async_main(args: argparse.Namespace) -> int:
    from .config import LLMConfig
    from .pipeline.executor import LLMExecutor
    from .pipeline.orchestrator import TranscriptSummarizer, _is_writer

    try:
        with open(args.input, "r", encoding="utf-8") as f:
            transcript = json.load(f)
    except (OSError, ValueError) as e:
        log.error("failed to load transcript %s: %s", args.input, e)
        return 1

    cfg = LLMConfig()
    if args.max_new_tokens is not None:
        cfg.MAX_TOKENS = args.max_new_tokens
    if args.temperature is not None:
        cfg.TEMPERATURE = args.temperature
    provider = args.provider or cfg.DEFAULT_PROVIDER
    popts = {}
    if provider == "mock":
        popts["fault_rate"] = args.fault_inject
    if provider == "local":
        popts.update({"dtype": args.dtype, "tp": args.tp, "seed": args.seed, "kv_fraction": args.kv_fraction,
                      "kv_dtype": args.kv_dtype,
                      "use_graphs": not args.no_graphs, "tokenizer": args.tokenizer,
                      "max_num_seqs": args.max_concurrent_requests, "reduce_tp": args.reduce_tp,
                      "parallel": args.parallel,
                      "weights": args.weights})
        if args.max_model_len:
            popts["max_model_len"] = args.max_model_len
    agg_executor = None
    if args.aggregator_model:
        if provider != "local":
            log.error("--aggregator-model needs the local provider")
            return 1
        if popts.get("kv_fraction") is None:
            popts["kv_fraction"] = 0.3  # leave HBM for the second engine
        aopts = dict(popts, dtype=args.aggregator_dtype, tp=args.aggregator_tp or args.tp, kv_fraction=0.6,
                     max_model_len=args.max_model_len or 40960, weights=args.aggregator_weights)
        agg_executor = LLMExecutor(config=cfg, provider="local", model=args.aggregator_model, **aopts)
    executor = LLMExecutor(config=cfg, provider=provider, model=args.model,
                           max_concurrent_requests=args.max_concurrent_requests, **popts)
    summarizer = TranscriptSummarizer(
        provider=provider, model=args.model, max_tokens_per_chunk=args.max_tokens_per_chunk,
        max_concurrent_requests=args.max_concurrent_requests, hierarchical_aggregation=not args.no_hierarchical,
        executor=executor, aggregator_executor=agg_executor,
        chunker_options={"position_mode": args.position_mode, "overlap_tokens": args.chunk_overlap,
                         "apply_overlap": args.chunk_overlap > 0},
        aggregator_options={"max_levels": args.reduce_levels or None}, stream_reduce=args.stream_reduce)
    from .utils.profiling import maybe_profile
    with maybe_profile(args.profile, int(os.environ.get("RANK", "0"))):
        result = await summarizer.summarize(
            transcript, merge_same_speaker=not args.no_merge, max_segment_duration=args.max_segment_duration,
            prompt_file=args.prompt_file, system_prompt_file=args.system_prompt_file,
            limit_segments=args.limit_segments, save_intermediate_chunks=args.save_chunks,
            aggregator_prompt_file=args.aggregator_prompt_file, resume_chunks=args.resume_chunks,
            time_interval_seconds=args.time_interval, preserve_timestamps=not args.no_timestamps)
    executor.backend.close()
    if not _is_writer():
        return 0
    summary = result["summary"]
    if not args.quiet:
        bar = "=" * 80
        print("\n%s\nTRANSCRIPT SUMMARY\n%s\n\n%s\n\n%s" % (bar, bar, summary, bar))
        print("Processing time: %.2f seconds" % result["processing_time"])
        print("Tokens used: %d" % result["tokens_used"])
        print("Estimated cost: $%.4f" % result["cost"])
        if result.get("chunks_per_second"):
            print("Map throughput: %.2f chunks/s (%d chunks)" % (result["chunks_per_second"], result["chunks"]))
        print(bar + "\n")
    if args.output:
        try:
            out = Path(args.output)
            out.parent.mkdir(parents=True, exist_ok=True)
            out.write_text(summary, encoding="utf-8")
            if args.report:
                rp = out.with_suffix(".report.json")
                rp.write_text(json.dumps(result, indent=2, default=str), encoding="utf-8")
                log.info("saved report to %s", rp)
            log.info("saved summary to %s", out)
        except OSError as e:
            log.error("failed to save output: %s", e)
            return 1
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    if args.debug_sync:  # must precede the first HIP call of the process
        os.environ.update(AMD_SERIALIZE_KERNEL="3", HIP_LAUNCH_BLOCKING="1", MRSUM_DEBUG_SYNC="1")
    setup_logging(args.log_level)
    from .parallel.dist import init_distributed_from_env, shutdown
    init_distributed_from_env()
    try:
        return asyncio.run(async_main(args))
    finally:
        shutdown()


if __name__ == "__main__":
    from .parallel.dist import exit_process
    exit_process(main())
