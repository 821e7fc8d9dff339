"""Orchestrator (layer L7): transcript -> preprocess -> chunk -> map -> reduce.

Reference: ``TranscriptSummarizer`` (``main.py:45-332``), ``summarize``
(``:82-257``).  Kept: constructor and ``summarize`` signatures, prompt
precedence (explicit template > file > default; ``main.py:155-167``), the
``--save-chunks`` JSON schema (``:178-201``), metadata ``File`` /
``Total Duration`` (``:219-231``) and the returned report keys
(``:248-257``).

Added: ``resume_chunks`` (load a saved chunk-summaries JSON and skip the map
stage), per-phase wall-clock timers and engine metrics under
``report["timings"]`` / ``report["engine"]``, counters
reset per run (Q17), and tokenizer injection so chunks are sized with the
engine's vocabulary.

``stream_reduce``: the level-1 reduce batches are planned before the map
and each starts as soon as its own chunks are summarised (the
reference's map ends with a full ``gather``, ``llm_executor.py:147``) --
see ``ResultAggregator.stream_plan`` and ``LLMExecutor.process_chunks_streamed``.
It needs the reduce on the map's executor; ``timings["map"]`` then covers
the map and the streamed level 1.

Under ``torch.distributed`` every rank runs this same code (SPMD): the
CPU front-end is deterministic, the local provider scatters each generate
batch over the data-parallel ranks and all-gathers the results, so every rank
ends with the same summary; only rank 0 writes files.
"""

from __future__ import annotations

import datetime
import json
import logging
import os
import time
from typing import Any, Dict, List, Optional

from .aggregator import ResultAggregator
from .chunker import Chunker
from .executor import LLMExecutor
from .preprocess import preprocess_transcript
from .prompts import load_map_prompt, load_optional_prompt

log = logging.getLogger("mrsum.orchestrator")


def _is_writer() -> bool:
    try:
        import torch.distributed as dist
        return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
    except Exception:
        return True


def format_duration(seconds: float) -> str:
    h, rem = divmod(int(seconds), 3600)
    m, s = divmod(rem, 60)
    return "%dh %dm %ds" % (h, m, s) if h > 0 else "%dm %ds" % (m, s)


def load_chunk_summaries(path: str) -> List[Dict[str, Any]]:
    with open(path, "r", encoding="utf-8") as f:
        data = json.load(f)
    return data["chunks"] if isinstance(data, dict) else data


class TranscriptSummarizer:
    def __init__(self, provider: Optional[str] = None, model: Optional[str] = None,
                 max_tokens_per_chunk: int = 4000, max_concurrent_requests: Optional[int] = None,
                 hierarchical_aggregation: bool = True, executor: Optional[LLMExecutor] = None,
                 chunker_options: Optional[Dict[str, Any]] = None, aggregator_options: Optional[Dict[str, Any]] = None,
                 provider_options: Optional[Dict[str, Any]] = None,
                 aggregator_executor: Optional[LLMExecutor] = None, stream_reduce: bool = False):
        """``aggregator_executor``: optional separate back-end for the reduce stage (e.g. the fp8
        Llama-3-70B aggregator of BASELINE config 5 while the map runs on Llama-3-8B); by default the
        reduce uses the map executor (the reference borrows its executor, result_aggregator.py:225)."""
        self.provider = provider
        self.model = model
        self.max_tokens_per_chunk = max_tokens_per_chunk
        self.max_concurrent_requests = max_concurrent_requests
        self.hierarchical_aggregation = hierarchical_aggregation
        self.executor = executor
        self.chunker: Optional[Chunker] = None
        self.aggregator: Optional[ResultAggregator] = None
        self.chunker_options = chunker_options or {}
        self.aggregator_options = aggregator_options or {}
        self.provider_options = provider_options or {}
        self.aggregator_executor = aggregator_executor
        self.stream_reduce = stream_reduce

    def _ensure_components(self) -> None:
        if self.executor is None:
            self.executor = LLMExecutor(provider=self.provider, model=self.model,
                                        max_concurrent_requests=self.max_concurrent_requests,
                                        **self.provider_options)
        self.provider = self.executor.provider
        tok = getattr(self.executor.backend, "tokenizer", None)
        if self.chunker is None:
            self.chunker = Chunker(max_tokens_per_chunk=self.max_tokens_per_chunk, tokenizer=tok,
                                   **self.chunker_options)
        if self.aggregator is None:
            self.aggregator = ResultAggregator(executor=self.aggregator_executor or self.executor,
                                               hierarchical=self.hierarchical_aggregation,
                                               tokenizer=tok, **self.aggregator_options)

    def _get_prompt_template(self, prompt_file: Optional[str] = None) -> str:
        return load_map_prompt(prompt_file)

    def _get_system_prompt(self, system_prompt_file: Optional[str] = None) -> Optional[str]:
        return load_optional_prompt(system_prompt_file, "system prompt")

    def _format_duration(self, seconds: float) -> str:
        return format_duration(seconds)

    async def summarize(self, transcript_data: Dict[str, Any], merge_same_speaker: bool = True,
                        max_segment_duration: int = 120, prompt_template: Optional[str] = None,
                        prompt_file: Optional[str] = None, system_prompt: Optional[str] = None,
                        system_prompt_file: Optional[str] = None, metadata: Optional[Dict[str, Any]] = None,
                        limit_segments: Optional[int] = None, save_intermediate_chunks: Optional[str] = None,
                        aggregator_prompt_file: Optional[str] = None, resume_chunks: Optional[str] = None,
                        time_interval_seconds: Optional[float] = None, preserve_timestamps: bool = True
                        ) -> Dict[str, Any]:
        t_start = time.perf_counter()
        timings: Dict[str, float] = {}
        self._ensure_components()
        ex = self.executor
        ex.reset_counters()
        if self.aggregator_executor is not None:
            self.aggregator_executor.reset_counters()

        segments = transcript_data.get("segments", [])
        if limit_segments:
            segments = segments[:limit_segments]
        log.info("summarizing transcript with %d segments", len(segments))

        t = time.perf_counter()
        processed = preprocess_transcript(segments, merge_same_speaker=merge_same_speaker,
                                          max_segment_duration=max_segment_duration,
                                          time_interval_seconds=time_interval_seconds,
                                          preserve_timestamps=preserve_timestamps)
        timings["preprocess"] = time.perf_counter() - t

        t = time.perf_counter()
        chunks = self.chunker.postprocess_chunks(self.chunker.chunk_transcript(processed))
        timings["chunk"] = time.perf_counter() - t
        log.info("%d segments -> %d processed -> %d chunks", len(segments), len(processed), len(chunks))

        if not prompt_template:
            prompt_template = self._get_prompt_template(prompt_file)
        sys_prompt = system_prompt or (self._get_system_prompt(system_prompt_file) if system_prompt_file else None)

        agg_prompt = load_optional_prompt(aggregator_prompt_file, "aggregator prompt")
        metadata = dict(metadata or {})
        file_info = transcript_data.get("file_info") if hasattr(transcript_data, "get") else None
        metadata.update({"File": file_info or "Unknown",
                         "Total Duration": format_duration(chunks[-1]["end_time"] if chunks else 0)})

        groups = None
        if self.stream_reduce and not resume_chunks:
            if self.aggregator_executor is not None:
                log.warning("--stream-reduce needs the reduce on the map's back-end: running the stages apart")
            else:
                chunks = sorted(chunks, key=lambda c: c["chunk_index"])
                groups = self.aggregator.stream_plan(chunks)
        level1 = None
        t = time.perf_counter()
        if groups:
            n = len(groups)
            processed_chunks, l1 = await ex.process_chunks_streamed(
                chunks, prompt_template, groups,
                lambda g, recs: self.aggregator.level1_request(g, n, recs, metadata), system_prompt=sys_prompt)
            level1 = (groups, l1)
        elif resume_chunks:
            saved = {c["chunk_index"]: c for c in load_chunk_summaries(resume_chunks)}
            processed_chunks = []
            for c in chunks:
                s = saved.get(c["chunk_index"])
                if s is None:
                    raise ValueError("resume file %s has no chunk %d" % (resume_chunks, c["chunk_index"]))
                d = dict(c)
                d.update({"summary": s.get("summary", ""), "tokens_used": s.get("tokens_used", 0), "cost": 0.0,
                          "processing_index": c["chunk_index"]})
                processed_chunks.append(d)
            log.info("resumed %d chunk summaries from %s (map stage skipped)", len(processed_chunks), resume_chunks)
        else:
            processed_chunks = await ex.process_chunks(chunks, prompt_template, system_prompt=sys_prompt)
        timings["map"] = time.perf_counter() - t

        if save_intermediate_chunks and _is_writer():
            try:
                out = {"timestamp": datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S"),
                       "chunks": [{"chunk_index": c.get("chunk_index", -1), "start_time": c.get("start_time", ""),
                                   "end_time": c.get("end_time", ""), "summary": c.get("summary", ""),
                                   "tokens_used": c.get("tokens_used", 0)} for c in processed_chunks]}
                parent = os.path.dirname(os.path.abspath(save_intermediate_chunks))
                os.makedirs(parent, exist_ok=True)
                with open(save_intermediate_chunks, "w", encoding="utf-8") as f:
                    json.dump(out, f, indent=2)
                log.info("saved %d chunk summaries to %s", len(processed_chunks), save_intermediate_chunks)
            except OSError as e:
                log.error("failed to save chunk summaries to %s: %s", save_intermediate_chunks, e)

        t = time.perf_counter()
        result = await self.aggregator.aggregate(processed_chunks, prompt_template=agg_prompt, metadata=metadata,
                                                 level1=level1)
        timings["reduce"] = time.perf_counter() - t

        elapsed = time.perf_counter() - t_start
        timings["total"] = elapsed
        n_failed = sum(1 for c in processed_chunks if c.get("error"))
        report = {
            "summary": result["summary"],
            "processing_time": elapsed,
            "tokens_used": ex.total_tokens_used + (self.aggregator_executor.total_tokens_used
                                                   if self.aggregator_executor is not None else 0),
            "cost": ex.total_cost + (self.aggregator_executor.total_cost if self.aggregator_executor is not None else 0.0),
            "segments": len(segments),
            "chunks": len(chunks),
            "provider": self.provider,
            "model": ex.model,
            "failed_chunks": n_failed,
            "chunks_per_second": (len(chunks) / timings["map"]) if timings["map"] > 0 else None,
            "timings": timings,
            "reduce_plan": result.get("plan", {}),
            "engine": ex.backend.stats(),
            "aggregator_engine": (self.aggregator_executor.backend.stats()
                                  if self.aggregator_executor is not None else None),
        }
        log.info("summarization done in %.2f s; tokens=%d", elapsed, ex.total_tokens_used)
        return report
