"""Configuration from the environment / ``.env`` (layer L0).

Reference: ``LLMConfig`` class attributes read once at import
(``llm_executor.py:31-52``) after ``load_dotenv()`` (``:29``, ``main.py:43``);
keys documented in ``.env.template:1-22``.

Here the same keys are recognised (plus engine keys), a minimal ``.env``
reader replaces python-dotenv (not installed offline; existing environment
variables win, as with ``load_dotenv(override=False)``), and an
``LLMConfig()`` *instance* re-reads the environment so settings changed after
import take effect (reference values stay available as class attributes).
Defaults follow the code / ``.env.template``, not the README.
"""

from __future__ import annotations

import os
from typing import Optional

_DOTENV_LOADED = False


def load_dotenv(path: Optional[str] = None) -> bool:
    """Populate ``os.environ`` from ``KEY=VALUE`` lines (inline ``#`` comments stripped)."""
    global _DOTENV_LOADED
    path = path or os.path.join(os.getcwd(), ".env")
    if not os.path.isfile(path):
        return False
    with open(path, "r", encoding="utf-8") as f:
        for raw in f:
            line = raw.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            key, val = line.split("=", 1)
            key = key.strip()
            if key.startswith("export "):
                key = key[7:].strip()
            val = val.strip()
            if val[:1] in "\"'" and val[-1:] == val[:1] and len(val) >= 2:
                val = val[1:-1]
            elif " #" in val:
                val = val.split(" #", 1)[0].rstrip()
            os.environ.setdefault(key, val)
    _DOTENV_LOADED = True
    return True


def _env(key: str, default: str) -> str:
    return os.environ.get(key, default)


class LLMConfig:
    """Provider + generation settings.  Class attributes = values at import time."""

    _FIELDS = {
        "OPENAI_API_KEY": ("", str), "OPENAI_ORG_ID": ("", str), "OPENAI_MODEL": ("gpt-3.5-turbo", str),
        "ANTHROPIC_API_KEY": ("", str), "ANTHROPIC_MODEL": ("claude-3-sonnet-20240229", str),
        "MAX_CONCURRENT_REQUESTS": ("5", int), "TEMPERATURE": ("0.3", float), "MAX_TOKENS": ("1000", int),
        "REQUEST_TIMEOUT": ("60", int), "RETRY_ATTEMPTS": ("3", int), "RETRY_DELAY": ("5", float),
        "DEFAULT_PROVIDER": ("local", str),
        # engine (new)
        "LOCAL_MODEL": ("llama3-8b", str), "ENGINE_DTYPE": ("bf16", str), "ENGINE_SEED": ("0", int),
        "ENGINE_MAX_NUM_SEQS": ("256", int), "ENGINE_KV_FRACTION": ("0.6", float),
        "ENGINE_KV_DTYPE": ("bf16", str),
        "REDUCE_TEMPERATURE": ("0.2", float),
        # hosted-provider endpoints (new): point the adapters at any compatible server
        "OPENAI_BASE_URL": ("https://api.openai.com/v1", str),
        "ANTHROPIC_BASE_URL": ("https://api.anthropic.com/v1", str),
    }

    def __init__(self, **overrides):
        for k, (d, typ) in self._FIELDS.items():
            setattr(self, k, typ(_env(k, d)))
        for k, v in overrides.items():
            if k not in self._FIELDS:
                raise TypeError("unknown config key %s" % k)
            setattr(self, k, v)

    def api_key(self, provider: str) -> str:
        return {"openai": self.OPENAI_API_KEY, "anthropic": self.ANTHROPIC_API_KEY}.get(provider, "")


load_dotenv()
for _k, (_d, _t) in LLMConfig._FIELDS.items():
    setattr(LLMConfig, _k, _t(_env(_k, _d)))
