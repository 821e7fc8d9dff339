"""Map stage executor (layer L5): one generation per chunk.

Reference: ``LLMExecutor`` (``llm_executor.py:54-432``).  The public surface is
kept -- constructor ``(config, provider, model, max_concurrent_requests)``,
``await process_chunks(chunks, prompt_template, summary_type, system_prompt)``
returning the chunks plus ``processing_index``, ``summary``, ``tokens_used``,
``cost`` (and ``error`` / ``system_prompt`` when relevant), sorted by
``chunk_index``; counters ``total_tokens_used``, ``total_cost``,
``total_requests``, ``failed_requests``; retries (``RETRY_ATTEMPTS`` x
``RETRY_DELAY``) with the ``"[Error processing chunk: ...]"`` summary on final
failure (``:196-228``).

What changes is the transport.  A *batched* provider (the local MI355X
engine) receives every chunk prompt of the stage at once -- continuous
batching on the GPU replaces the reference's ``asyncio.Semaphore`` fan-out,
and the engine shards the batch over data-parallel ranks.  Hosted providers
still use a semaphore of ``max_concurrent_requests`` in-flight requests.  The
reduce stage borrows :meth:`LLMExecutor.generate`, so map and reduce always
use the same provider (SURVEY Q1 fix).
"""

from __future__ import annotations

import asyncio
import logging
import time
from typing import Any, Dict, List, Optional, Sequence

from ..config import LLMConfig
from .prompts import render_template
from .providers import GenRequest, GenResult, Provider, make_provider

log = logging.getLogger("mrsum.executor")


class LLMExecutor:
    def __init__(self, config: Optional[LLMConfig] = None, provider: Optional[str] = None,
                 model: Optional[str] = None, max_concurrent_requests: Optional[int] = None,
                 provider_obj: Optional[Provider] = None, **provider_kwargs):
        self.config = config or LLMConfig()
        if provider_obj is not None:
            self._provider = provider_obj
            self.provider = provider_obj.name
        else:
            self.provider = provider or self.config.DEFAULT_PROVIDER
            self._provider = make_provider(self.provider, model, self.config, **provider_kwargs)
        self.model = self._provider.model
        self.max_concurrent_requests = max_concurrent_requests or self.config.MAX_CONCURRENT_REQUESTS
        self.reset_counters()
        if self.provider in ("openai", "anthropic") and not self.config.api_key(self.provider):
            log.warning("%s API key not found; responses will be mocked", self.provider)
        log.info("LLM executor ready: provider=%s model=%s", self.provider, self.model)

    def reset_counters(self) -> None:
        self.total_tokens_used = 0
        self.total_cost = 0.0
        self.total_requests = 0
        self.failed_requests = 0
        self.retried_requests = 0  # failed attempts that were retried (final failures: failed_requests)
        self.phase_seconds: Dict[str, float] = {}

    @property
    def backend(self) -> Provider:
        return self._provider

    def _get_api_key(self) -> str:
        return self.config.api_key(self.provider)

    # ------------------------------------------------------------ generation
    async def _one_with_retries(self, req: GenRequest, sem: asyncio.Semaphore) -> GenResult:
        attempts = max(1, self.config.RETRY_ATTEMPTS)
        async with sem:
            for attempt in range(1, attempts + 1):
                try:
                    return await self._provider.generate(req)
                except Exception as e:  # provider errors are per request
                    log.warning("request failed (attempt %d/%d): %s", attempt, attempts, e)
                    if attempt == attempts:
                        return GenResult("", error=str(e))
                    self.retried_requests += 1
                    await asyncio.sleep(self.config.RETRY_DELAY)
        raise AssertionError("unreachable")

    def _account(self, results: Sequence[Optional[GenResult]]) -> None:
        for r in results:
            if r is None:
                continue
            self.total_requests += 1
            if r.error:
                self.failed_requests += 1
            else:
                self.total_tokens_used += r.tokens_used
                self.total_cost += r.cost

    async def generate(self, reqs: Sequence[GenRequest], stage: str = "map",
                       attempts: Optional[int] = None) -> List[GenResult]:
        """Run requests through the provider with the executor's retry policy and accounting."""
        t0 = time.perf_counter()
        if not reqs:
            return []
        if self._provider.batched:
            results: List[Optional[GenResult]] = [None] * len(reqs)
            pending = list(range(len(reqs)))
            attempts = max(1, self.config.RETRY_ATTEMPTS if attempts is None else attempts)
            for attempt in range(1, attempts + 1):
                try:
                    out = await self._provider.generate_batch([reqs[i] for i in pending])
                except Exception as e:
                    out = [GenResult("", error=str(e)) for _ in pending]
                nxt = []
                for i, r in zip(pending, out):
                    results[i] = r
                    if r.error:
                        nxt.append(i)
                if not nxt:
                    break
                log.warning("%d/%d requests failed (attempt %d/%d)", len(nxt), len(reqs), attempt, attempts)
                pending = nxt
                if attempt < attempts:
                    self.retried_requests += len(nxt)
                    await asyncio.sleep(self.config.RETRY_DELAY)
            final = [r for r in results if r is not None]
        else:
            sem = asyncio.Semaphore(max(1, self.max_concurrent_requests))
            final = list(await asyncio.gather(*[self._one_with_retries(r, sem) for r in reqs]))
        self._account(final)
        self.phase_seconds[stage] = self.phase_seconds.get(stage, 0.0) + time.perf_counter() - t0
        return final

    def _map_requests(self, chunks: List[Dict[str, Any]], prompt_template: str, summary_type: str,
                      system_prompt: Optional[str]):
        reqs, outs = [], []
        for idx, chunk in enumerate(chunks):
            res = dict(chunk)
            if system_prompt:
                res["system_prompt"] = system_prompt
            res["processing_index"] = idx
            prompt = render_template(prompt_template, transcript=chunk["text_with_context"],
                                     summary_type=summary_type)
            reqs.append(GenRequest(user=prompt, system=system_prompt, max_tokens=self.config.MAX_TOKENS,
                                   temperature=self.config.TEMPERATURE, stage="map", tag=idx))
            outs.append(res)
        return reqs, outs

    @staticmethod
    def _apply(res: Dict[str, Any], r: GenResult) -> Dict[str, Any]:
        """Fill a chunk record from its map result (reference llm_executor.py:196-228 error text)."""
        if r.error:
            res["summary"] = "[Error processing chunk: %s]" % r.error
            res["error"] = r.error
            res["tokens_used"] = 0
            res["cost"] = 0
        else:
            res["summary"] = r.text
            res["tokens_used"] = r.tokens_used
            res["cost"] = r.cost
        return res

    def _log_map(self, n: int, dt: float) -> None:
        log.info("map stage done: %d chunks in %.2f s (%.2f chunks/s); tokens=%d failed=%d/%d", n, dt,
                 n / dt if dt > 0 else 0.0, self.total_tokens_used, self.failed_requests, self.total_requests)

    async def process_chunks(self, chunks: List[Dict[str, Any]], prompt_template: str,
                             summary_type: str = "summary", system_prompt: Optional[str] = None
                             ) -> List[Dict[str, Any]]:
        t0 = time.perf_counter()
        log.info("map stage: %d chunks via %s", len(chunks), self.provider)
        reqs, outs = self._map_requests(chunks, prompt_template, summary_type, system_prompt)
        results = await self.generate(reqs, stage="map")
        for res, r in zip(outs, results):
            self._apply(res, r)
        outs.sort(key=lambda c: c["chunk_index"])
        self._log_map(len(chunks), time.perf_counter() - t0)
        return outs

    async def process_chunks_streamed(self, chunks: List[Dict[str, Any]], prompt_template: str,
                                      groups: Sequence[Sequence[int]], build, summary_type: str = "summary",
                                      system_prompt: Optional[str] = None):
        """Map stage with a follow-up request per group of chunks, started as soon as the group's
        chunks are summarised (the streamed map -> level-1 reduce of SURVEY §2.5; the reference waits for
        every chunk, llm_executor.py:147).  ``groups`` holds positions in ``chunks``;
        ``build(g, records)`` gets the group's chunk records (as process_chunks returns them) and returns
        a GenRequest or None.

        Returns ``(records, follow_ups)``: the chunk records sorted by chunk_index and one GenResult (or
        None) per group.  A group with a chunk that failed in the streamed pass gets None -- its chunks
        are retried like process_chunks' and the caller re-runs the group from the final records.

        Transports: the local engine streams inside one continuous batch (``generate_groups``); a
        per-request provider (hosted HTTP, mock) runs one asyncio task per group under the
        ``max_concurrent_requests`` semaphore, so a group's follow-up is sent the moment its last chunk
        returns; any other batched provider falls back to map, then follow-ups (a barrier)."""
        t0 = time.perf_counter()
        log.info("map stage (streamed into %d follow-ups): %d chunks via %s", len(groups), len(chunks), self.provider)
        reqs, outs = self._map_requests(chunks, prompt_template, summary_type, system_prompt)
        first: List[Optional[GenResult]] = [None] * len(reqs)
        second: List[Optional[GenResult]] = [None] * len(groups)
        records = lambda g, res: build(g, [self._apply(dict(outs[i]), r) for i, r in zip(groups[g], res)])
        streamed = None
        if self._provider.batched and hasattr(self._provider, "generate_groups"):
            streamed = await self._provider.generate_groups(reqs, groups, records)
        if streamed is not None:
            first, second = list(streamed[0]), list(streamed[1])
            self._account(first)
            # groups built from a failed chunk are dropped (below) and re-run by the aggregator, which
            # accounts them then: count only the follow-ups that are kept
            self._account([r for g, r in enumerate(second)
                           if not any(first[i].error for i in groups[g])])
        elif not self._provider.batched:
            sem = asyncio.Semaphore(max(1, self.max_concurrent_requests))

            async def run_group(g: int) -> None:
                res = await asyncio.gather(*[self._one_with_retries(reqs[i], sem) for i in groups[g]])
                for i, r in zip(groups[g], res):
                    first[i] = r
                r2 = records(g, list(res))
                if r2 is not None:
                    second[g] = await self._one_with_retries(r2, sem)

            await asyncio.gather(*[run_group(g) for g in range(len(groups))])
            self._account(first)
            self._account(second)
        else:  # batched provider without a streaming path: map, then the follow-ups
            first = await self.generate(reqs, stage="map")
            follow = [(g, records(g, [first[i] for i in groups[g]])) for g in range(len(groups))]
            follow = [(g, r) for g, r in follow if r is not None]
            res2 = await self.generate([r for _, r in follow], stage=follow[0][1].stage if follow else "reduce_l1")
            for (g, _), r in zip(follow, res2):
                second[g] = r
        self.phase_seconds["map+follow_ups"] = time.perf_counter() - t0
        if streamed is not None:  # per-request transports retried inside the pass already
            bad = [i for i, r in enumerate(first) if r.error]
            if bad:
                log.warning("%d/%d chunks failed in the streamed pass: retrying them", len(bad), len(reqs))
                for g, members in enumerate(groups):
                    if any(first[i].error for i in members):
                        second[g] = None  # built from an error text: the caller re-runs it
                retry = await self.generate([reqs[i] for i in bad], stage="map",
                                            attempts=max(1, self.config.RETRY_ATTEMPTS - 1))
                for i, r in zip(bad, retry):
                    first[i] = r
                # the failed pass's records were accounted above; keep failed_requests = final failures
                self.failed_requests -= len(bad)
                self.total_requests -= len(bad)
        for res, r in zip(outs, first):
            self._apply(res, r)
        outs.sort(key=lambda c: c["chunk_index"])
        self._log_map(len(chunks), time.perf_counter() - t0)
        return outs, second


async def process_chunks_parallel(chunks: List[Dict[str, Any]], prompt_template: str,
                                  provider: Optional[str] = None, model: Optional[str] = None,
                                  summary_type: str = "summary") -> List[Dict[str, Any]]:
    """Reference helper ``llm_executor.py:435-457``."""
    return await LLMExecutor(provider=provider, model=model).process_chunks(chunks, prompt_template, summary_type)
