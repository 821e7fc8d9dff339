"""One-shot reducer (the reference's alternative ``SimpleAggregator``).

Reference: ``simple_aggregator.py:26-189`` -- one call over all chunk
summaries with a fixed "summary only" system message, a fixed
Overview / Main Topics / Key Points / Notable Quotes user prompt, temperature
0.2, 1000 tokens, ``"Error generating summary: ..."`` on failure, and a sync
wrapper ``aggregate_summaries``.  Not wired into the orchestrator (same as the
reference).

Difference: instead of raising when no OpenAI key is set (reference ``:41-42``)
it goes through an executor, i.e. any provider -- by default the local
engine, or the mock.
"""

from __future__ import annotations

import asyncio
import logging
from typing import Any, Dict, List, Optional

from .executor import LLMExecutor
from .prompts import format_metadata_block
from .providers import GenRequest

log = logging.getLogger("mrsum.simple_aggregator")

SIMPLE_SYSTEM = """
You are a professional transcript summarizer that ONLY creates summaries.

IMPORTANT RULES:
1. DO NOT include any greeting in your response
2. DO NOT introduce yourself or explain what you're doing
3. DO NOT ask how you can help
4. ONLY output the requested summary in the specified format
5. Your response MUST start with "# Transcript Summary"
6. DO NOT make up information - use ONLY what's in the provided summaries
"""

SIMPLE_USER = """
I need you to combine these transcript segment summaries into a final summary.

{metadata}

Here are the summaries from different parts of the transcript:

{summaries}

Your summary must accurately reflect ONLY the content in these summaries.

Format your response with these exact headings:

# Transcript Summary

## Overview
[2-3 sentence high-level description of the transcript content]

## Main Topics
[Bullet list of key themes and topics discussed]

## Key Points
[Bullet list of important details and takeaways]

## Notable Quotes
[Direct quotes from the transcript that were mentioned in the summaries]
"""


class SimpleAggregator:
    def __init__(self, executor: Optional[LLMExecutor] = None, model: Optional[str] = None,
                 provider: Optional[str] = None, temperature: float = 0.2, max_tokens: int = 1000):
        self.executor = executor or LLMExecutor(provider=provider, model=model)
        self.model = self.executor.model
        self.temperature = temperature
        self.max_tokens = max_tokens

    @staticmethod
    def _format_summaries(summaries: List[str]) -> str:
        bar = "=" * 40
        return "".join("SUMMARY %d:\n%s\n%s\n%s\n\n" % (i + 1, bar, s.strip(), bar) for i, s in enumerate(summaries))

    def build_request(self, chunk_summaries: List[str], metadata: Optional[Dict[str, Any]] = None) -> GenRequest:
        user = SIMPLE_USER.replace("{metadata}", format_metadata_block(metadata)).replace(
            "{summaries}", self._format_summaries(chunk_summaries))
        return GenRequest(user=user, system=SIMPLE_SYSTEM, max_tokens=self.max_tokens,
                          temperature=self.temperature, stage="reduce_final")

    async def aggregate(self, chunk_summaries: List[str], metadata: Optional[Dict[str, Any]] = None) -> str:
        log.info("aggregating %d summaries", len(chunk_summaries))
        res = (await self.executor.generate([self.build_request(chunk_summaries, metadata)], stage="reduce_final"))[0]
        if res.error:
            log.error("error generating aggregated summary: %s", res.error)
            return "Error generating summary: %s" % res.error
        return res.text


def aggregate_summaries(chunk_summaries: List[str], metadata: Optional[Dict[str, Any]] = None,
                        executor: Optional[LLMExecutor] = None) -> str:
    """Synchronous wrapper (reference ``simple_aggregator.py:177-189``)."""
    return asyncio.run(SimpleAggregator(executor=executor).aggregate(chunk_summaries, metadata))
