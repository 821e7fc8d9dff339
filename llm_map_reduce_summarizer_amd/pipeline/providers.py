"""Generation back-ends ("providers") behind the map and reduce stages.

Reference: the executor's provider adapters (``llm_executor.py:232-432``) --
OpenAI chat completions (``:250-326``), Anthropic messages (``:328-409``) and
the no-key mock (``:411-432``).

Here a provider turns a *batch* of chat requests into results:

* ``local``  -- the on-node MI355X engine (``engine/``), data-parallel over the
  ranks of the process group; the default.
* ``mock``   -- deterministic canned responses with the reference mock's
  text / token schema, optional fault injection and an
  optional simulated latency; runs anywhere.
* ``openai`` / ``anthropic`` -- thin HTTPS adapters kept for capability
  parity; with no API key they fall back to the mock response exactly like
  the reference.  The Anthropic adapter sends the system prompt as the
  top-level ``system`` field (SURVEY Q8 fix).
"""

from __future__ import annotations

import asyncio
import hashlib
import logging
import random
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

from ..config import LLMConfig

log = logging.getLogger("mrsum.providers")


@dataclass
class GenRequest:
    user: str
    system: Optional[str] = None
    max_tokens: int = 1000
    temperature: float = 0.3
    stage: str = "map"
    tag: Any = None
    # a whole chat ([{"role": "system" | "user" | "assistant", "content": str}, ...]) instead of the
    # reference's [system?, user] pair -- the HTTP front-end (serve.py) passes multi-turn requests here
    messages: Optional[List[Dict[str, str]]] = None


@dataclass
class GenResult:
    text: str
    prompt_tokens: int = 0
    completion_tokens: int = 0
    cost: float = 0.0
    is_mock: bool = False
    error: Optional[str] = None
    extra: Dict[str, Any] = field(default_factory=dict)

    @property
    def tokens_used(self) -> int:
        return self.prompt_tokens + self.completion_tokens


class ProviderError(RuntimeError):
    pass


class Provider:
    """Base class.  ``batched`` providers receive whole batches at once."""

    name = "base"
    batched = False

    def __init__(self, model: str, config: Optional[LLMConfig] = None):
        self.model = model
        self.config = config or LLMConfig()

    async def generate(self, req: GenRequest) -> GenResult:  # pragma: no cover - abstract
        raise NotImplementedError

    async def generate_batch(self, reqs: Sequence[GenRequest]) -> List[GenResult]:
        return [await self.generate(r) for r in reqs]

    def stats(self) -> Dict[str, Any]:
        return {}

    def close(self) -> None:
        pass


def mock_map_text(provider: str, model: str) -> str:
    # reference llm_executor.py:422
    return ("[Mock %s Response using %s]\n\nThis is a simulated summary generated because no API key was "
            "provided. In a real scenario, this would contain a summary of the transcript chunk."
            % (provider.capitalize(), model))


MOCK_REDUCE_TEXT = ("# Transcript Summary\n\n## Overview\nThis is a mock summary for testing without an API key.\n\n"
                    "## Main Topics\n- Topic 1\n- Topic 2\n\n## Key Points\n- Key point 1\n- Key point 2\n\n"
                    "## Notable Quotes\n- 'This is a mock quote.'")


def mock_result(provider: str, model: str, stage: str) -> GenResult:
    if stage == "map":
        return GenResult(mock_map_text(provider, model), prompt_tokens=75, completion_tokens=25, is_mock=True)
    return GenResult(MOCK_REDUCE_TEXT, prompt_tokens=0, completion_tokens=0, is_mock=True)


class MockProvider(Provider):
    """Canned responses; ``fault_rate`` makes attempts fail (deterministically per request+attempt)."""

    name = "mock"

    def __init__(self, model: str = "mock", config: Optional[LLMConfig] = None, fault_rate: float = 0.0,
                 latency_s: float = 0.0, seed: int = 0, label: str = "mock"):
        super().__init__(model, config)
        self.fault_rate = fault_rate
        self.latency_s = latency_s
        self.seed = seed
        self.label = label
        self._attempts: Dict[str, int] = {}
        self.calls = 0
        self.peak_in_flight = 0
        self._in_flight = 0

    def _should_fail(self, req: GenRequest) -> bool:
        if self.fault_rate <= 0:
            return False
        key = hashlib.sha1((req.system or "").encode() + req.user.encode()).hexdigest()
        n = self._attempts.get(key, 0)
        self._attempts[key] = n + 1
        return random.Random("%s:%d:%d" % (key, n, self.seed)).random() < self.fault_rate

    async def generate(self, req: GenRequest) -> GenResult:
        self.calls += 1
        self._in_flight += 1
        self.peak_in_flight = max(self.peak_in_flight, self._in_flight)
        try:
            if self.latency_s:
                await asyncio.sleep(self.latency_s)
            if self._should_fail(req):
                raise ProviderError("injected fault")
            return mock_result(self.label, self.model, req.stage)
        finally:
            self._in_flight -= 1


class _HTTPProvider(Provider):
    path = ""

    @property
    def url(self) -> str:
        base = self.config.OPENAI_BASE_URL if self.name == "openai" else self.config.ANTHROPIC_BASE_URL
        return base.rstrip("/") + self.path

    def _key(self) -> str:
        return self.config.api_key(self.name)

    async def _post(self, headers: Dict[str, str], body: Dict[str, Any]) -> Dict[str, Any]:
        import aiohttp  # only needed for the hosted providers
        timeout = aiohttp.ClientTimeout(total=self.config.REQUEST_TIMEOUT)
        async with aiohttp.ClientSession(timeout=timeout) as session:
            async with session.post(self.url, headers=headers, json=body) as resp:
                try:
                    data = await resp.json(content_type=None)
                except ValueError:
                    data = {"error": {"message": (await resp.text())[:200]}}
                if resp.status != 200:
                    msg = (data.get("error") or {}).get("message", "Unknown error") if isinstance(data, dict) else data
                    raise ProviderError("%s API Error: %s" % (self.name, msg))
                return data


class OpenAIProvider(_HTTPProvider):
    name = "openai"
    path = "/chat/completions"  # reference llm_executor.py:292

    async def generate(self, req: GenRequest) -> GenResult:
        if not self._key():
            log.warning("no OpenAI API key: using the mock response")
            return mock_result("openai", self.model, req.stage)
        headers = {"Content-Type": "application/json", "Authorization": "Bearer %s" % self._key()}
        if self.config.OPENAI_ORG_ID:
            headers["OpenAI-Organization"] = self.config.OPENAI_ORG_ID
        msgs = ([{"role": "system", "content": req.system}] if req.system else []) + [
            {"role": "user", "content": req.user}]
        data = await self._post(headers, {"model": self.model, "messages": msgs, "temperature": req.temperature,
                                          "max_tokens": req.max_tokens})
        usage = data.get("usage", {})
        pt, ct = usage.get("prompt_tokens", 0), usage.get("completion_tokens", 0)
        # reference llm_executor.py:310-317
        rate_in, rate_out = (0.00003, 0.00006) if "gpt-4" in self.model else (0.000001, 0.000002)
        return GenResult(data["choices"][0]["message"]["content"], pt, ct, pt * rate_in + ct * rate_out)


class AnthropicProvider(_HTTPProvider):
    name = "anthropic"
    path = "/messages"

    async def generate(self, req: GenRequest) -> GenResult:
        if not self._key():
            log.warning("no Anthropic API key: using the mock response")
            return mock_result("anthropic", self.model, req.stage)
        headers = {"Content-Type": "application/json", "x-api-key": self._key(),
                   "anthropic-version": "2023-06-01"}
        body: Dict[str, Any] = {"model": self.model, "messages": [{"role": "user", "content": req.user}],
                                "temperature": req.temperature, "max_tokens": req.max_tokens}
        if req.system:
            body["system"] = req.system
        data = await self._post(headers, body)
        text = data["content"][0]["text"]
        usage = data.get("usage") or {}
        pt = usage.get("input_tokens", len(req.user) // 4)
        ct = usage.get("output_tokens", len(text) // 4)
        return GenResult(text, pt, ct, pt * 0.000003 + ct * 0.000015)


def make_provider(name: str, model: Optional[str] = None, config: Optional[LLMConfig] = None,
                  **engine_kwargs) -> Provider:
    config = config or LLMConfig()
    if name == "openai":
        return OpenAIProvider(model or config.OPENAI_MODEL, config)
    if name == "anthropic":
        return AnthropicProvider(model or config.ANTHROPIC_MODEL, config)
    if name == "mock":
        return MockProvider(model or "mock", config, fault_rate=engine_kwargs.get("fault_rate", 0.0),
                            latency_s=engine_kwargs.get("latency_s", 0.0))
    if name == "local":
        from ..engine.provider import LocalEngineProvider
        return LocalEngineProvider(model or config.LOCAL_MODEL, config, **engine_kwargs)
    raise ValueError("unsupported provider: %s" % name)
