"""Prompt management (layer L4).

* map prompts: ``{transcript}`` (+ optional ``{summary_type}``) -- reference
  ``llm_executor.py:187-190``; file loading with auto-appended ``{transcript}``
  -- ``main.py:259-300``; system-prompt files -- ``main.py:302-322``.
* reduce prompts: ``{summaries}`` / ``{metadata}`` / ``{num_summaries}`` --
  reference ``result_aggregator.py:146-219`` (single pass), ``:404-498``
  (default / batch / final templates).

Deviations:

* Q7 -- templates are rendered with :func:`render_template`, which substitutes
  only known placeholders and leaves any other ``{...}`` text alone, so a JSON
  example inside a prompt file no longer aborts the run with ``KeyError``.
  ``{{`` / ``}}`` still produce literal braces, as with ``str.format``.
* Q2/Q3 -- the batch and final templates are actually rendered (the reference
  builds them but always sends its default user prompt), and a custom
  aggregator prompt is honoured in every mode (at the final level when the
  reduce is hierarchical).
* The built-in prompts are stored without the reference's 8-space source
  indentation, which only cost prompt tokens.
"""

from __future__ import annotations

import logging
import re
from typing import Any, Dict, Iterable, Mapping, Optional

log = logging.getLogger("mrsum.prompts")

DEFAULT_MAP_PROMPT = """Please summarize the following transcript segment:

{transcript}

Provide:

### 1. Concise Summary
[A 3-5 sentence overview of what this segment covers]

### 2. Key Topics Discussed
[Bullet list of the main topics]

### 3. Notable Quotes or Statements
[2-3 important or representative quotes]"""

_RULES = """IMPORTANT RULES:
1. DO NOT include any greeting or introduction
2. DO NOT ask how you can help
3. {rule3}
4. {rule4}
5. The summary MUST ONLY contain information from the provided summaries
6. DO NOT make up information not contained in the summaries
7. DO NOT discuss general impacts of technology - stay focused on the transcript content"""

AGG_SYSTEM_DEFAULT = (
    "You are a professional transcript summarizer. Your ONLY job is to create a structured summary that "
    "combines information from multiple transcript segment summaries.\n\n"
    + _RULES.format(rule3="ONLY produce the summary in the requested format",
                    rule4='START your response with "# Transcript Summary"'))

AGG_SYSTEM_VIDEO = (
    "You are a professional transcript summarizer specializing in video editing formats. Your job is to "
    "create a structured summary that combines information from multiple transcript segment summaries.\n\n"
    + _RULES.format(rule3="Follow EXACTLY the format specified in the user prompt",
                    rule4="Preserve ALL timestamps in [HH:MM:SS] format"))

AGG_USER_DEFAULT = """I need you to combine multiple transcript summaries into a single coherent summary.

{metadata}

Here are the summaries from different segments of the transcript:

{summaries}

Your summary must accurately reflect ONLY the content in these summaries.

Format your response with these exact headings:

# Transcript Summary

## Overview
[2-3 sentence high-level description of what the transcript contains]

## Main Topics
[Bullet list of key themes and topics discussed]

## Key Points
[Bullet list of important details and takeaways]

## Notable Quotes
[Direct quotes from the transcript that were mentioned in the summaries]"""

AGG_BATCH_PROMPT = """Create an intermediate summary for this section of a transcript.

{metadata}

Here are {num_summaries} summaries from consecutive segments:

{summaries}

IMPORTANT INSTRUCTIONS:
1. DO NOT introduce yourself or add any greeting
2. DO NOT ask how you can help
3. ONLY provide the summary in the format below
4. START your response with "# Intermediate Summary"

Your intermediate summary must:
- Combine key information from these segment summaries
- Preserve important details, quotes, and themes
- Maintain chronological order and context
- Be thorough rather than brief at this stage

Format your summary as:
# Intermediate Summary

[Your detailed summary content here]"""

AGG_FINAL_PROMPT = """Create the FINAL SUMMARY of a complete transcript by combining these section summaries.

{metadata}

Here are {num_summaries} section summaries covering the entire transcript:

{summaries}

IMPORTANT INSTRUCTIONS:
1. DO NOT introduce yourself or add any greeting
2. DO NOT ask how you can help
3. ONLY provide the summary in the format below
4. START your response with "# Transcript Summary"

Your final summary must:
- Synthesize key information from all sections
- Present a cohesive narrative of the entire transcript
- Highlight important themes, insights, and quotes
- Organize information in a logical structure

Format your summary with these headings:
# Transcript Summary

## Overview
[2-3 sentence high-level description]

## Main Topics
[Bullet list of key themes discussed]

## Important Points
[Key details and takeaways]

## Notable Quotes
[Direct quotes from the transcript]"""

VIDEO_EDITOR_MARKER = "TIMELINE SUMMARY"

_PLACEHOLDER = re.compile(r"\{\{|\}\}|\{(\w+)\}")


def render_template(template: str, **values: Any) -> str:
    """``str.format``-like substitution that never raises on unknown fields."""

    def sub(m: "re.Match[str]") -> str:
        tok = m.group(0)
        if tok == "{{":
            return "{"
        if tok == "}}":
            return "}"
        name = m.group(1)
        if name in values:
            return str(values[name])
        return tok

    return _PLACEHOLDER.sub(sub, template)


def read_text_file(path: str) -> str:
    with open(path, "r", encoding="utf-8") as f:
        return f.read().strip()


def load_map_prompt(prompt_file: Optional[str]) -> str:
    """Map prompt from file (``{transcript}`` appended when missing) or the default."""
    if prompt_file:
        try:
            content = read_text_file(prompt_file)
            if "{transcript}" not in content:
                log.warning("prompt file %s has no {transcript} placeholder; appending it", prompt_file)
                content += "\n\n{transcript}"
            return content
        except OSError as e:
            log.error("cannot read prompt file %s (%s); using the default prompt", prompt_file, e)
    return DEFAULT_MAP_PROMPT


def load_optional_prompt(path: Optional[str], what: str = "prompt") -> Optional[str]:
    if not path:
        return None
    try:
        return read_text_file(path)
    except OSError as e:
        log.error("cannot read %s file %s (%s); ignoring it", what, path, e)
        return None


def format_metadata_block(metadata: Optional[Mapping[str, Any]]) -> str:
    if not metadata:
        return ""
    return "Additional Information:\n" + "".join("- %s: %s\n" % (k, v) for k, v in metadata.items())


def format_summaries_block(summaries: Iterable[str]) -> str:
    bar = "=" * 40
    return "".join("SUMMARY %d:\n%s\n%s\n%s\n\n" % (i + 1, bar, s, bar) for i, s in enumerate(summaries))


def build_aggregation_messages(summaries: list, template: Optional[str],
                               metadata: Optional[Mapping[str, Any]]) -> Dict[str, str]:
    """System + user message for one reduce call (see module docstring)."""
    meta = format_metadata_block(metadata)
    block = format_summaries_block(summaries)
    if template and VIDEO_EDITOR_MARKER in template:
        system = AGG_SYSTEM_VIDEO
    else:
        system = AGG_SYSTEM_DEFAULT
    if not template:
        template = AGG_USER_DEFAULT
    user = render_template(template, summaries=block, metadata=meta, num_summaries=len(summaries))
    if meta and "{metadata}" not in template:
        user = meta + "\n\n" + user  # reference result_aggregator.py:184-188
    return {"system": system, "user": user}
