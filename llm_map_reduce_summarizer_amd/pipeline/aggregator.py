"""Reduce stage (layer L6): combine chunk summaries into one summary.

Reference: ``ResultAggregator`` (``result_aggregator.py:26-498``).  Kept:

* summaries sorted by ``chunk_index`` and prefixed ``"[Time: a - b]\\n"``
  (``:79-90``); empty summaries skipped;
* single pass when hierarchical is off or the summaries total
  ``<= max_tokens_per_batch`` (6000) tokens (``:95``);
* otherwise two levels: contiguous batches of
  ``min(10, max(1, int((6000 - 1000) / avg_tokens)))`` summaries (``:357-380``)
  reduced concurrently with ``Batch: i/n`` / ``Position`` metadata
  (``:325-342``), then one final pass (``:346-355``);
* return ``{"summary", "chunks_aggregated", "processing_time"}``, error text
  ``"Error generating summary: ..."`` on failure (``:256-259``).

Changed: the reduce calls go through the *executor's*
provider (Q1: the reference always POSTs to OpenAI), the batch/final
templates and custom prompts are rendered (Q2/Q3), the reduce temperature is
configurable (``REDUCE_TEMPERATURE``, default 0.2 as the reference
hard-codes), and ``max_levels=None`` enables a recursive reduce that keeps
batching until one prompt fits (the reference stops at 2 levels).

With the local engine every level is ONE batched generate call, so level-1
batches are spread over the data-parallel ranks and prefilled together.

Streamed level 1 (``stream_plan`` / ``level1_request`` / ``aggregate(...,
level1=...)``): the level-1 batches are fixed BEFORE the map
runs, from the token cap of a summary (``MAX_TOKENS`` + the ``[Time: ...]``
prefix) instead of the measured average, so each batch's reduce can start as
soon as its own chunks are summarised.  With capped (pinned-length) summaries
the plan equals the reference's; with shorter ones it may use more, smaller
batches than the reference would (never a batch over the token budget); and
when the real summaries total no more than ``max_tokens_per_batch`` the
streamed level-1 outputs are dropped and the reduce is the reference's single
pass (the structure never gains a level the reference would not have).
"""

from __future__ import annotations

import logging
import time
from typing import Any, Dict, List, Optional

from .executor import LLMExecutor
from .preprocess import format_timestamp
from .prompts import AGG_BATCH_PROMPT, AGG_FINAL_PROMPT, build_aggregation_messages
from .providers import GenRequest

log = logging.getLogger("mrsum.aggregator")


class ResultAggregator:
    def __init__(self, executor: Optional[LLMExecutor] = None, max_tokens_per_batch: int = 6000,
                 tokenizer_name: Optional[str] = None, hierarchical: bool = True, tokenizer=None,
                 max_levels: Optional[int] = 2, reserved_tokens: int = 1000, max_batch_size: int = 10):
        self.executor = executor or LLMExecutor()
        self.max_tokens_per_batch = max_tokens_per_batch
        if tokenizer is None:
            tokenizer = getattr(self.executor.backend, "tokenizer", None)
        if tokenizer is None:
            from ..engine.tokenizer import get_tokenizer
            tokenizer = get_tokenizer(tokenizer_name)
        self.tokenizer = tokenizer
        self.hierarchical = hierarchical
        self.max_levels = max_levels
        self.level_seconds: List[float] = []
        self.reserved_tokens = reserved_tokens
        self.max_batch_size = max_batch_size
        self.last_plan: Dict[str, Any] = {}

    # --------------------------------------------------------------- helpers
    def _format_time(self, seconds: float) -> str:
        return format_timestamp(seconds)

    def _total_tokens(self, texts: List[str]) -> int:
        return sum(self.tokenizer.count(t) for t in texts)

    def _calculate_batch_size(self, summaries: List[str]) -> int:
        if not summaries:
            return 1
        avg = self._total_tokens(summaries) / len(summaries)
        per = max(1, int((self.max_tokens_per_batch - self.reserved_tokens) / max(avg, 1e-9)))
        return min(per, self.max_batch_size)

    def _request(self, summaries: List[str], template: Optional[str], metadata: Optional[Dict[str, Any]],
                 stage: str) -> GenRequest:
        msgs = build_aggregation_messages(summaries, template, metadata)
        cfg = self.executor.config
        return GenRequest(user=msgs["user"], system=msgs["system"], max_tokens=cfg.MAX_TOKENS,
                          temperature=cfg.REDUCE_TEMPERATURE, stage=stage)

    async def _run(self, reqs: List[GenRequest], stage: str) -> List[str]:
        results = await self.executor.generate(reqs, stage=stage)
        out = []
        for r in results:
            if r.error:
                log.error("aggregation call failed: %s", r.error)
                out.append("Error generating summary: %s" % r.error)
            else:
                out.append(r.text)
        return out

    async def _single_aggregation(self, summaries: List[str], prompt_template: Optional[str] = None,
                                  metadata: Optional[Dict[str, Any]] = None) -> str:
        return (await self._run([self._request(summaries, prompt_template, metadata, "reduce_final")],
                                "reduce_final"))[0]

    @staticmethod
    def _summaries(chunks: List[Dict[str, Any]]) -> List[str]:
        out = []
        for c in chunks:
            if c.get("summary"):
                out.append("[Time: %s - %s]\n%s" % (format_timestamp(c.get("start_time", 0)),
                                                    format_timestamp(c.get("end_time", 0) or 0), c["summary"]))
            else:
                log.warning("chunk %s has no summary", c.get("chunk_index", "?"))
        return out

    def _batch_request(self, batch: List[str], i: int, n: int, metadata: Optional[Dict[str, Any]],
                       level: int) -> GenRequest:
        meta = dict(metadata or {})
        meta.update({"Batch": "%d/%d" % (i + 1, n),
                     "Position": "Covering approximately %.0f%% - %.0f%% of the transcript"
                                 % (100 * i / n, 100 * (i + 1) / n)})
        return self._request(batch, AGG_BATCH_PROMPT, meta, "reduce_l%d" % level)

    # ------------------------------------------------------- streamed level 1
    def stream_plan(self, chunks: List[Dict[str, Any]]) -> Optional[List[List[int]]]:
        """Level-1 batches (positions in ``chunks``, chunk_index order) fixed before the map runs, or
        None when the reduce would not be hierarchical even with every summary at the token cap."""
        if not self.hierarchical or self.max_levels == 1 or len(chunks) < 2:
            return None
        cap = self.executor.config.MAX_TOKENS + self.tokenizer.count("[Time: 00:00:00 - 00:00:00]\n")
        if len(chunks) * cap <= self.max_tokens_per_batch:
            return None
        bs = min(self.max_batch_size, max(1, int((self.max_tokens_per_batch - self.reserved_tokens) / cap)))
        order = sorted(range(len(chunks)), key=lambda i: chunks[i].get("chunk_index", 0))
        return [order[i:i + bs] for i in range(0, len(order), bs)]

    def level1_request(self, g: int, n: int, records: List[Dict[str, Any]],
                       metadata: Optional[Dict[str, Any]] = None) -> Optional[GenRequest]:
        """Level-1 reduce request of batch ``g`` of ``n`` from its chunk records (None: no summaries)."""
        batch = self._summaries(sorted(records, key=lambda c: c.get("chunk_index", 0)))
        return self._batch_request(batch, g, n, metadata, 1) if batch else None

    # ------------------------------------------------------------------ main
    async def aggregate(self, processed_chunks: List[Dict[str, Any]], prompt_template: Optional[str] = None,
                        metadata: Optional[Dict[str, Any]] = None, level1=None) -> Dict[str, Any]:
        """``level1``: ``(groups, results)`` of a streamed level 1 (stream_plan groups as positions in
        ``processed_chunks`` sorted by chunk_index, one GenResult or None per group); missing or failed
        batches are re-run here, then the reduce continues at level 2."""
        t0 = time.perf_counter()
        if not processed_chunks:
            return {"summary": "", "error": "No chunks provided for aggregation"}
        processed_chunks = sorted(processed_chunks, key=lambda c: c.get("chunk_index", 0))
        summaries = self._summaries(processed_chunks)
        log.info("aggregating %d summaries", len(summaries))
        self.level_seconds = []
        single = not self.hierarchical or self._total_tokens(summaries) <= self.max_tokens_per_batch
        if level1 is not None and single:
            # the real summaries fit one reduce call (stream_plan sized its groups for summaries at the
            # token cap): the reference does one pass here, so the streamed level-1 outputs are dropped
            log.info("streamed level 1 not needed: %d summaries fit one reduce pass", len(summaries))
            level1 = None
        if level1 is not None:
            final = await self._hierarchical_aggregation(summaries, prompt_template, metadata,
                                                         level1=(level1[0], level1[1], processed_chunks))
        elif single:
            self.last_plan = {"levels": 1, "calls": [1]}
            t1 = time.perf_counter()
            final = await self._single_aggregation(summaries, prompt_template, metadata)
            self.level_seconds.append(time.perf_counter() - t1)
        else:
            final = await self._hierarchical_aggregation(summaries, prompt_template, metadata)
        dt = time.perf_counter() - t0
        log.info("aggregation done in %.2f s (%s)", dt, self.last_plan)
        plan = dict(self.last_plan)
        plan["seconds"] = [round(x, 3) for x in self.level_seconds]  # wall-clock of every reduce level
        if level1 is not None:
            plan["level1_streamed"] = True  # level 1 ran inside the map pass (seconds[0]: re-runs only)
        return {"summary": final, "chunks_aggregated": len(processed_chunks), "processing_time": dt,
                "plan": plan}

    async def _streamed_level1(self, groups, results, chunks, metadata) -> List[str]:
        """Level-1 outputs of a streamed level 1: the streamed results, with missing / failed batches
        re-run (executor retry policy) from the final chunk records."""
        n = len(groups)
        redo = []
        for g in range(n):
            r = results[g]
            if r is None or r.error:
                req = self.level1_request(g, n, [chunks[i] for i in groups[g]], metadata)
                if req is not None:
                    redo.append((g, req))
        out: Dict[int, str] = {g: r.text for g, r in enumerate(results) if r is not None and not r.error}
        if redo:
            log.warning("re-running %d of %d streamed level-1 batches", len(redo), n)
            for (g, _), text in zip(redo, await self._run([r for _, r in redo], "reduce_l1")):
                out[g] = text
        return [out[g] for g in range(n) if g in out]

    async def _hierarchical_aggregation(self, summaries: List[str], prompt_template: Optional[str] = None,
                                        metadata: Optional[Dict[str, Any]] = None, level1=None) -> str:
        calls: List[int] = []
        current = summaries
        while True:
            level = len(calls) + 1
            before = self._total_tokens(current) if self.max_levels is None else 0
            t1 = time.perf_counter()
            if level == 1 and level1 is not None:
                groups, results, chunks = level1
                n = len(groups)
                log.info("reduce level 1 (streamed with the map): %d chunks -> %d batches", len(chunks), n)
                current = await self._streamed_level1(groups, results, chunks, metadata)
            else:
                bs = self._calculate_batch_size(current)
                batches = [current[i:i + bs] for i in range(0, len(current), bs)]
                n = len(batches)
                reqs = [self._batch_request(b, i, n, metadata, level) for i, b in enumerate(batches)]
                log.info("reduce level %d: %d summaries -> %d batches of <=%d", level, len(current), n, bs)
                current = await self._run(reqs, "reduce_l%d" % level)
            self.level_seconds.append(time.perf_counter() - t1)
            calls.append(n)
            if len(current) == 1:
                self.last_plan = {"levels": len(calls), "calls": calls}
                return current[0]
            if self.max_levels is not None:
                if len(calls) + 1 >= self.max_levels:  # the final pass is the last allowed level
                    break
            else:
                after = self._total_tokens(current)
                if after <= self.max_tokens_per_batch or after >= before:
                    break  # recursive mode: stop once everything fits (or a level no longer shrinks it)
        template = prompt_template or AGG_FINAL_PROMPT
        calls.append(1)
        self.last_plan = {"levels": len(calls), "calls": calls}
        t1 = time.perf_counter()
        out = (await self._run([self._request(current, template, metadata, "reduce_final")], "reduce_final"))[0]
        self.level_seconds.append(time.perf_counter() - t1)
        return out


def aggregate_results(processed_chunks: List[Dict[str, Any]], prompt_template: Optional[str] = None,
                      metadata: Optional[Dict[str, Any]] = None, hierarchical: bool = True,
                      executor: Optional[LLMExecutor] = None) -> str:
    """Synchronous wrapper (reference ``result_aggregator.py:501-524``)."""
    import asyncio
    agg = ResultAggregator(executor=executor, hierarchical=hierarchical)
    return asyncio.run(agg.aggregate(processed_chunks, prompt_template, metadata))["summary"]
