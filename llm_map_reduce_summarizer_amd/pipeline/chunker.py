"""Token-bounded, sentence-aware transcript chunker (layer L3).

Behavioural contract: reference ``big_chunkeroosky.py`` (class
``BigChunkeroosky``, ``:20-567``).  Chunks are packed greedily from formatted
segment lines ``"[MM:SS] SPEAKER: text"`` (``:244-265``) until the next line
would push the *sum of per-line token counts* past
``max_tokens_per_chunk - context_tokens`` (``:42``, ``:86``); separators and
the context header are not counted (kept).  Oversize segments are
split by their merged sub-segments, then by sentences, then by clauses /
20-word groups (``:267-542``).  Every chunk gets the context header of
``:197-232`` and the keys listed in SURVEY.md §2.2.

The tokenizer is injected (``tokenizer=`` an object with ``count(str)``, or a
name for :func:`engine.tokenizer.get_tokenizer`) so chunks are sized against
the same vocabulary the engine prefills with -- the north-star requirement.

Documented deviations (each switchable for reference parity):

* ``position_mode="transcript"`` (default): ``position_percentage`` is the
  chunk start's offset over the *whole transcript* duration.  The reference
  divides by the chunk's own end; ``position_mode="reference"``
  reproduces that.
* Clause-level sub-chunks inherit the parent segment's speaker;
  ``reference_quirks=True`` restores the empty speaker.
* ``_split_long_sentence`` keeps text after the last clause punctuation (the
  reference's ``findall`` silently drops it); ``reference_quirks=True``
  restores the drop.
* ``overlap_tokens`` is honoured when ``apply_overlap=True``: the tail of the
  previous chunk is added to ``text_with_context`` as a clearly marked
  "previous context" block (chunk boundaries and ``token_count`` unchanged).
  The reference stores but never uses it (``:26,40``).
* Sentence splitting uses a rule-based splitter equivalent to an untrained
  Punkt model on transcript text (split after ``.?!`` + closing quotes when
  followed by whitespace).  NLTK is not available offline; exact Punkt parity
  is unpinned.
"""

from __future__ import annotations

import logging
import re
from typing import Any, Dict, List, Optional

from .preprocess import format_timestamp

log = logging.getLogger("mrsum.chunker")

Segment = Dict[str, Any]
Chunk = Dict[str, Any]

_SENT_SPLIT = re.compile(r"(?<=[.!?])[\"'”’)\]]*\s+")
_CLAUSE = re.compile(r"([^,.;:?!]+[,.;:?!]+)")


def split_sentences(text: str) -> List[str]:
    """Split after sentence-final punctuation followed by whitespace."""
    out: List[str] = []
    pos = 0
    for m in _SENT_SPLIT.finditer(text):
        end = m.start() + len(m.group(0).rstrip())
        out.append(text[pos:end])
        pos = m.end()
    if pos < len(text):
        out.append(text[pos:])
    return [s for s in out if s.strip()]


def _resolve_tokenizer(tokenizer):
    if tokenizer is None or isinstance(tokenizer, str):
        from ..engine.tokenizer import get_tokenizer
        return get_tokenizer(tokenizer)
    return tokenizer


class Chunker:
    """Packs processed segments into LLM-sized chunks (reference ``BigChunkeroosky``)."""

    def __init__(self, max_tokens_per_chunk: int = 4000, overlap_tokens: int = 200,
                 tokenizer_name: Optional[str] = None, context_tokens: int = 150, tokenizer=None,
                 position_mode: str = "transcript", reference_quirks: bool = False,
                 apply_overlap: bool = False):
        if max_tokens_per_chunk <= context_tokens:
            raise ValueError("max_tokens_per_chunk must exceed context_tokens")
        if position_mode not in ("transcript", "reference"):
            raise ValueError("position_mode must be 'transcript' or 'reference'")
        self.max_tokens_per_chunk = max_tokens_per_chunk
        self.overlap_tokens = overlap_tokens
        self.context_tokens = context_tokens
        self.effective_max_tokens = max_tokens_per_chunk - context_tokens
        self.tokenizer = _resolve_tokenizer(tokenizer if tokenizer is not None else tokenizer_name)
        self.position_mode = position_mode
        self.reference_quirks = reference_quirks
        self.apply_overlap = apply_overlap
        self._transcript_end: float = 0.0

    # --------------------------------------------------------------- helpers
    def _count(self, text: str) -> int:
        return self.tokenizer.count(text)

    @staticmethod
    def _format_time(seconds: float) -> str:
        return format_timestamp(seconds)

    def _format_segment_for_chunk(self, seg: Segment) -> str:
        # reference :244-265 -- combined segments keep their inline [ts] prefixes
        # (so the first one is doubled, SURVEY Q5, kept for token-count parity).
        return "[%s] %s: %s" % (format_timestamp(seg["start"]), seg["speaker"], seg["text"])

    @staticmethod
    def _new_chunk(start: float) -> Chunk:
        return {"segments": [], "text": "", "token_count": 0, "start_time": start, "end_time": None,
                "speakers": set()}

    @staticmethod
    def _append(chunk: Chunk, seg: Segment, text: str, tokens: int) -> None:
        chunk["segments"].append(seg)
        if chunk["text"]:
            chunk["text"] += "\n\n"
        chunk["text"] += text
        chunk["token_count"] += tokens
        chunk["end_time"] = seg["end"]
        chunk["speakers"].add(seg["speaker"])

    # ------------------------------------------------------------------ main
    def chunk_transcript(self, processed_segments: List[Segment], add_context: bool = True) -> List[Chunk]:
        chunks: List[Chunk] = []
        if not processed_segments:
            return chunks
        log.info("Chunker: processing %d segments (budget %d tokens)", len(processed_segments),
                 self.effective_max_tokens)
        self._transcript_end = max(s["end"] for s in processed_segments)
        total = len(processed_segments)
        eff = self.effective_max_tokens
        cur = self._new_chunk(processed_segments[0]["start"])
        for idx, seg in enumerate(processed_segments):
            text = self._format_segment_for_chunk(seg)
            ntok = self._count(text)
            if cur["token_count"] + ntok > eff and cur["segments"]:
                self._finalize_chunk(cur, chunks, idx, total, add_context)
                cur = self._new_chunk(seg["start"])
            if ntok > eff:
                for sub in self._chunk_large_segment(seg):
                    if cur["token_count"] > 0 and cur["token_count"] + sub["token_count"] > eff:
                        self._finalize_chunk(cur, chunks, idx, total, add_context)
                        s = sub["segment"]
                        cur = {"segments": [s], "text": sub["text"], "token_count": sub["token_count"],
                               "start_time": s["start"], "end_time": s["end"], "speakers": {s["speaker"]}}
                    else:
                        self._append(cur, sub["segment"], sub["text"], sub["token_count"])
            else:
                self._append(cur, seg, text, ntok)
        if cur["segments"]:
            self._finalize_chunk(cur, chunks, total, total, add_context)
        log.info("Chunker: created %d chunks from %d segments", len(chunks), total)
        return chunks

    def _finalize_chunk(self, chunk: Chunk, chunks: List[Chunk], current_segment_index: int,
                        total_segments: int, add_context: bool) -> None:
        chunk["speakers"] = sorted(chunk["speakers"])
        chunk["chunk_index"] = len(chunks)
        chunk["total_chunks"] = None
        first = chunk["segments"][0]["start"]
        t0 = chunks[0]["segments"][0]["start"] if chunks else first
        if self.position_mode == "reference":
            denom_end = chunk["segments"][-1]["end"]
        else:
            denom_end = self._transcript_end
        chunk["position_percentage"] = ((first - t0) / (denom_end - t0) * 100.0) if denom_end > t0 else 0
        if add_context:
            header = self._create_context_header(chunk, current_segment_index, total_segments)
            prev = self._overlap_block(chunks) if self.apply_overlap else ""
            chunk["text_with_context"] = header + "\n\n" + prev + chunk["text"]
        else:
            chunk["text_with_context"] = chunk["text"]
        chunks.append(chunk)

    def _overlap_block(self, chunks: List[Chunk]) -> str:
        if not chunks or self.overlap_tokens <= 0:
            return ""
        ids = self.tokenizer.encode_ordinary(chunks[-1]["text"])
        tail = self.tokenizer.decode(ids[-self.overlap_tokens:])
        return "--- PREVIOUS CONTEXT (end of chunk %d) ---\n%s\n--- END PREVIOUS CONTEXT ---\n\n" % (
            chunks[-1]["chunk_index"] + 1, tail.strip())

    def _create_context_header(self, chunk: Chunk, current_segment_index: int, total_segments: int) -> str:
        return ("--- TRANSCRIPT CHUNK INFORMATION ---\n"
                "Time Range: %s - %s\n"
                "Speakers: %s\n"
                "Position: Chunk %d (approximately %.1f%% through the transcript)\n"
                "--- TRANSCRIPT CHUNK CONTENT ---") % (
                    format_timestamp(chunk["start_time"]), format_timestamp(chunk["end_time"]),
                    ", ".join(chunk["speakers"]), chunk["chunk_index"] + 1, chunk["position_percentage"])

    # --------------------------------------------------------- large segments
    @staticmethod
    def _sub(start: float, end: Optional[float], speaker: str, text: str, tokens: int, parent: Segment,
             clause: bool = False, with_parent: bool = True) -> Dict[str, Any]:
        seg = {"start": start, "end": end, "speaker": speaker, "text": text, "is_sub_chunk": True}
        if clause:
            seg["is_clause"] = True
        if with_parent:
            seg["parent_segment_start"] = parent["start"]
            seg["parent_segment_end"] = parent["end"]
        return {"segment": seg, "text": text, "token_count": tokens}

    def _chunk_large_segment(self, segment: Segment) -> List[Dict[str, Any]]:
        eff = self.effective_max_tokens
        subs: List[Dict[str, Any]] = []
        spk = segment["speaker"]
        if "segment_timestamps" in segment and segment.get("is_combined", False):
            parts = segment["segment_timestamps"]
            cur = self._sub(parts[0]["start"], None, spk, "", 0, segment)
            for ts in parts:
                t = "[%s] %s" % (format_timestamp(ts["start"]), ts["text"])
                n = self._count(t)
                if cur["token_count"] + n > eff and cur["token_count"] > 0:
                    subs.append(cur)
                    cur = self._sub(ts["start"], None, spk, "", 0, segment)
                if cur["text"]:
                    cur["text"] += " "
                cur["text"] += t
                cur["token_count"] += n
                cur["segment"]["end"] = ts["end"]
                cur["segment"]["text"] = cur["text"]
            if cur["token_count"] > 0:
                subs.append(cur)
            return subs

        text = segment["text"]
        span = segment["end"] - segment["start"]
        tpc = span / len(text) if text else 0.0
        done = 0
        cur = self._sub(segment["start"], None, spk, "", 0, segment)
        for sentence in split_sentences(text):
            s = sentence.strip()
            if not s:
                continue
            s_start = segment["start"] + tpc * done
            s_end = s_start + tpc * len(s)
            done += len(s)
            ft = "[%s] %s" % (format_timestamp(s_start), s)
            n = self._count(ft)
            if n > eff:
                clauses = self._split_long_sentence(s, s_start, s_end, speaker=spk, parent=segment)
                if cur["token_count"] > 0:
                    cur["segment"]["end"] = s_start
                    cur["segment"]["text"] = cur["text"]
                    subs.append(cur)
                subs.extend(clauses)
                cur = self._sub(s_end, None, spk, "", 0, segment)
            elif cur["token_count"] + n > eff and cur["token_count"] > 0:
                cur["segment"]["end"] = s_start
                cur["segment"]["text"] = cur["text"]
                subs.append(cur)
                cur = self._sub(s_start, s_end, spk, ft, n, segment)
            else:
                if cur["text"]:
                    cur["text"] += " "
                cur["text"] += ft
                cur["token_count"] += n
                cur["segment"]["end"] = s_end
                cur["segment"]["text"] = cur["text"]
        if cur["token_count"] > 0:
            subs.append(cur)
        return subs

    def _split_long_sentence(self, sentence: str, start_time: float, end_time: float, speaker: str = "",
                             parent: Optional[Segment] = None) -> List[Dict[str, Any]]:
        eff = self.effective_max_tokens
        matches = list(_CLAUSE.finditer(sentence))
        clauses = [m.group(0) for m in matches]
        if matches and not self.reference_quirks:
            tail = sentence[matches[-1].end():]  # unpunctuated tail the reference drops
            if tail.strip():
                clauses.append(tail)
        if not clauses:
            words = sentence.split()
            clauses = [" ".join(words[i:i + 20]) for i in range(0, len(words), 20)]
        tpc = (end_time - start_time) / len(sentence) if sentence else 0.0
        quirk = self.reference_quirks
        spk = "" if quirk else speaker
        par = parent or {"start": start_time, "end": end_time}
        subs: List[Dict[str, Any]] = []
        cur = self._sub(start_time, None, spk, "", 0, par, clause=True, with_parent=not quirk)
        done = 0
        for c in clauses:
            ct = c.strip()
            if not ct:
                continue
            c_start = start_time + tpc * done
            c_end = c_start + tpc * len(ct)
            done += len(ct)
            ft = "[%s] %s" % (format_timestamp(c_start), ct)
            n = self._count(ft)
            if cur["token_count"] + n > eff and cur["token_count"] > 0:
                subs.append(cur)
                cur = self._sub(c_start, c_end, spk, ft, n, par, clause=True, with_parent=not quirk)
            else:
                if cur["text"]:
                    cur["text"] += " "
                cur["text"] += ft
                cur["token_count"] += n
                cur["segment"]["end"] = c_end
                cur["segment"]["text"] = cur["text"]
        if cur["token_count"] > 0:
            subs.append(cur)
        return subs

    # ------------------------------------------------------------ post-pass
    def postprocess_chunks(self, chunks: List[Chunk]) -> List[Chunk]:
        n = len(chunks)
        for c in chunks:
            c["total_chunks"] = n
        for c in chunks:
            for seg in c["segments"]:
                if seg.get("is_clause", False) and not seg["speaker"] and "parent_segment_start" in seg:
                    seg["speaker"] = c["speakers"][0] if c["speakers"] else "UNKNOWN"
        return chunks


# Reference-compatible name (reference big_chunkeroosky.py:20).
BigChunkeroosky = Chunker
