"""Llama-3 chat template.

The reference sends ``[{"role": "system"}, {"role": "user"}]`` chat messages
to hosted APIs (``llm_executor.py:274-281``; aggregator
``result_aggregator.py:225-231``).  The local engine renders the same
messages with the Llama-3 instruct format and tokenises them with the
engine tokenizer (special tokens at their Llama-3 ids)::

    <|begin_of_text|><|start_header_id|>system<|end_header_id|>\\n\\n{system}<|eot_id|>
    <|start_header_id|>user<|end_header_id|>\\n\\n{user}<|eot_id|>
    <|start_header_id|>assistant<|end_header_id|>\\n\\n
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence

from .tokenizer import LLAMA3_SPECIALS, BPETokenizer

BOT = LLAMA3_SPECIALS["<|begin_of_text|>"]
SH = LLAMA3_SPECIALS["<|start_header_id|>"]
EH = LLAMA3_SPECIALS["<|end_header_id|>"]
EOT = LLAMA3_SPECIALS["<|eot_id|>"]


def _header(tok: BPETokenizer, role: str) -> List[int]:
    return [SH] + tok.encode_ordinary(role) + [EH] + tok.encode_ordinary("\n\n")


def render_chat(tok: BPETokenizer, user: str, system: Optional[str] = None) -> List[int]:
    ids = [BOT]
    if system:
        ids += _header(tok, "system") + tok.encode_ordinary(system) + [EOT]
    ids += _header(tok, "user") + tok.encode_ordinary(user) + [EOT]
    ids += _header(tok, "assistant")
    return ids


def render_messages(tok: BPETokenizer, messages: Sequence[Dict[str, str]]) -> List[int]:
    """Any chat ([{"role", "content"}, ...]: system / user / assistant turns in order), rendered the same
    way turn by turn, ending with the assistant header (the turn to generate)."""
    ids = [BOT]
    for m in messages:
        ids += _header(tok, m["role"]) + tok.encode_ordinary(m["content"]) + [EOT]
    ids += _header(tok, "assistant")
    return ids
