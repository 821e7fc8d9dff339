"""Transcript preprocessing (layer L2 of the pipeline).

Behavioural contract (reference ``preprocessor.py``):

* ``preprocess_transcript``  -- reference ``preprocessor.py:15-67``
* ``clean_text``             -- ``preprocessor.py:69-89``
* ``format_timestamp``       -- ``preprocessor.py:91-107``
* ``combine_same_speaker_segments`` / ``create_combined_segment``
                             -- ``preprocessor.py:109-215``
* ``aggregate_by_time_interval`` -- ``preprocessor.py:217-324``
* ``extract_speakers`` / ``get_transcript_duration`` -- ``:326-361``

The output dictionaries (keys, text formats, timestamp formats) are kept
identical to the reference because the chunker, the prompts and the saved
JSON files all depend on them.  Golden numbers for the
bundled example transcript are pinned in ``tests/test_preprocess.py``.

Differences from the reference (documented deviations):

* progress messages go through :mod:`logging` (logger ``mrsum.preprocess``)
  instead of ``print`` so ``--quiet`` runs are quiet;
* ``aggregate_by_time_interval`` buckets segments with a sort + two-pointer
  sweep instead of the reference's O(intervals x segments) scan; the
  resulting segments are identical.
"""

from __future__ import annotations

import bisect
import logging
import math
import re
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

log = logging.getLogger("mrsum.preprocess")

Segment = Dict[str, Any]

_REPEATED_WORD = re.compile(r"\b(\w+)( \1\b)+")
_MISSING_SPACE = re.compile(r"([.!?])([A-Za-z])")


def format_timestamp(seconds: float) -> str:
    """``MM:SS`` below one hour, ``HH:MM:SS`` above; truncates to whole seconds."""
    total = int(seconds)
    hours, rem = divmod(total, 3600)
    minutes, secs = divmod(rem, 60)
    if hours > 0:
        return "%02d:%02d:%02d" % (hours, minutes, secs)
    return "%02d:%02d" % (minutes, secs)


def clean_text(text: str) -> str:
    """Collapse whitespace, drop stuttered repeats ("the the"), add a space after
    sentence punctuation glued to a following letter."""
    out = " ".join(text.split())
    out = _REPEATED_WORD.sub(r"\1", out)
    out = _MISSING_SPACE.sub(r"\1 \2", out)
    return out


def _base_segment(raw: Segment) -> Optional[Segment]:
    text = raw.get("text", "")
    if not text.strip():
        return None
    start = raw.get("start", 0)
    end = raw.get("end", 0)
    return {
        "start": start,
        "end": end,
        "start_formatted": format_timestamp(start),
        "end_formatted": format_timestamp(end),
        "speaker": raw.get("speaker", ""),
        "text": clean_text(text),
    }


def create_combined_segment(group: Sequence[Segment], preserve_timestamps: bool = True) -> Segment:
    """Merge a run of same-speaker segments.  A run of one is returned unchanged."""
    if not group:
        return {}
    if len(group) == 1:
        return group[0]
    first, last = group[0], group[-1]
    if preserve_timestamps:
        text = " ".join("[%s] %s" % (format_timestamp(s["start"]), s["text"]) for s in group)
    else:
        text = " ".join(s["text"] for s in group)
    return {
        "start": first["start"],
        "end": last["end"],
        "start_formatted": format_timestamp(first["start"]),
        "end_formatted": format_timestamp(last["end"]),
        "speaker": first["speaker"],
        "text": text,
        "is_combined": True,
        "original_segments": len(group),
        "segment_timestamps": [{"start": s["start"], "end": s["end"], "text": s["text"]} for s in group],
    }


def combine_same_speaker_segments(
    segments: Sequence[Segment],
    max_duration: Optional[float] = 120,
    preserve_timestamps: bool = True,
) -> List[Segment]:
    """Greedy merge of consecutive same-speaker segments.

    A new group starts when the speaker changes or when adding the next
    segment's *spoken* duration (end - start, gaps excluded) would exceed
    ``max_duration`` (reference ``preprocessor.py:136-154``).
    """
    if not segments:
        return []
    n_speakers = len({s["speaker"] for s in segments})
    log.info("Preprocessing: found %d unique speakers in transcript", n_speakers)

    merged: List[Segment] = []
    group: List[Segment] = [segments[0]]
    duration = segments[0]["end"] - segments[0]["start"]
    speaker = segments[0]["speaker"]
    for seg in segments[1:]:
        seg_dur = seg["end"] - seg["start"]
        if seg["speaker"] != speaker or (max_duration is not None and duration + seg_dur > max_duration):
            merged.append(create_combined_segment(group, preserve_timestamps))
            group, duration, speaker = [seg], seg_dur, seg["speaker"]
        else:
            group.append(seg)
            duration += seg_dur
    merged.append(create_combined_segment(group, preserve_timestamps))

    log.info("Preprocessing: combined %d segments into %d segments (ratio %.2f)",
             len(segments), len(merged), len(merged) / len(segments))
    return merged


def _overlaps(start: float, end: float, lo: float, hi: float) -> bool:
    # reference preprocessor.py:249-252 -- starts inside [lo, hi) or spans lo.
    return (lo <= start < hi) or (start <= lo and end > lo)


def aggregate_by_time_interval(segments: Sequence[Segment], interval_seconds: float) -> List[Segment]:
    """Bucket segments into fixed windows of ``interval_seconds``.

    Semantics follow reference ``preprocessor.py:217-324`` exactly: a segment
    belongs to every window it starts in or spans the start of; combined
    segments keep only their component parts that overlap the window; windows
    with no content are dropped.
    """
    if not segments:
        return []
    t0 = segments[0]["start"]
    t1 = segments[-1]["end"]
    n_int = math.ceil((t1 - t0) / interval_seconds)
    log.info("Creating %d time intervals of %s seconds each (%s - %s)", n_int, interval_seconds,
             format_timestamp(t0), format_timestamp(t1))

    # Candidates for window [lo, hi): segments with start < hi and end > lo, or
    # start >= lo.  Sorting by start lets us skip everything that starts at/after hi.
    order = sorted(range(len(segments)), key=lambda i: segments[i]["start"])
    starts = [segments[i]["start"] for i in order]
    max_len = max((s["end"] - s["start"]) for s in segments)

    out: List[Segment] = []
    for k in range(n_int):
        lo = t0 + k * interval_seconds
        hi = min(lo + interval_seconds, t1)
        # any overlapping segment starts in [lo - max_len, hi)
        a = bisect.bisect_left(starts, lo - max_len - 1e-9)
        b = bisect.bisect_left(starts, hi)
        picked: List[Tuple[int, Segment]] = []
        for pos in range(a, b):
            idx = order[pos]
            seg = segments[idx]
            if not _overlaps(seg["start"], seg["end"], lo, hi):
                continue
            piece = dict(seg)
            if "segment_timestamps" in seg:
                parts = [ts for ts in seg["segment_timestamps"] if _overlaps(ts["start"], ts["end"], lo, hi)]
                if not parts:
                    continue
                piece["segment_timestamps"] = parts
                piece["text"] = " ".join("[%s] %s" % (format_timestamp(ts["start"]), ts["text"])
                                         for ts in sorted(parts, key=lambda x: x["start"]))
            picked.append((idx, piece))
        if not picked:
            continue
        # keep original list order among equal starts (matches the reference's
        # stable sort over the input order)
        picked.sort(key=lambda p: (p[1]["start"], p[0]))
        ordered = [p[1] for p in picked]
        speakers = set(p["speaker"] for p in ordered)
        text = "\n\n".join("[%s %s] %s" % (format_timestamp(p["start"]), p["speaker"], p["text"]) for p in ordered)
        out.append({
            "start": lo,
            "end": hi,
            "start_formatted": format_timestamp(lo),
            "end_formatted": format_timestamp(hi),
            "speaker": ", ".join(speakers) if len(speakers) > 1 else next(iter(speakers)),
            "text": text,
            "is_aggregated": True,
            "interval_index": k,
            "original_segments": len(ordered),
            "segment_timestamps": [{"start": p["start"], "end": p["end"], "speaker": p["speaker"], "text": p["text"]}
                                   for p in ordered],
        })
    log.info("Created %d time-interval segments", len(out))
    return out


def preprocess_transcript(
    segments: Iterable[Segment],
    merge_same_speaker: bool = True,
    time_interval_seconds: Optional[float] = None,
    max_segment_duration: Optional[float] = 120,
    preserve_timestamps: bool = True,
) -> List[Segment]:
    """Clean -> (optionally) merge same-speaker runs -> (optionally) bucket by time."""
    result = [p for p in (_base_segment(s) for s in segments) if p is not None]
    if merge_same_speaker and result:
        result = combine_same_speaker_segments(result, max_segment_duration, preserve_timestamps)
    if time_interval_seconds and result:
        result = aggregate_by_time_interval(result, time_interval_seconds)
    return result


def extract_speakers(segments: Iterable[Segment]) -> List[str]:
    """Sorted unique non-empty speaker labels."""
    return sorted({s["speaker"] for s in segments if s.get("speaker")})


def get_transcript_duration(segments: Sequence[Segment]) -> Tuple[float, str]:
    """(last end - first start, formatted)."""
    if not segments:
        return 0.0, "00:00"
    dur = segments[-1]["end"] - segments[0]["start"]
    return dur, format_timestamp(dur)
