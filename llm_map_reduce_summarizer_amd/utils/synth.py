"""Deterministic synthetic transcripts.

The benchmark configs in BASELINE.json (1 h / 10 h / 24 h transcripts) need
input data of the reference's input schema (``{"segments": [{start, end,
text, speaker}]}``, reference README.md:162-175) on machines that have no
datasets.  This generator reproduces the statistics of the reference's
bundled example talk (measured in SURVEY.md §2.1 C11 / our own probe):

* segment duration: log-normal, mean 4.18 s, median 3.12 s, clipped to
  [0.16, 29.4] s;
* inter-segment gap: 0 s with p=0.6, else exponential (overall mean 1.38 s);
* ~2.6 spoken words per second, unigram word distribution from
  ``assets/wordfreq.tsv``, '.', ',', '?' at the measured rates, occasional
  numbers, sentence-initial capitalisation.

A 10 h transcript therefore has ~6.4k raw segments, like the 10 h config of
SURVEY.md §6.  Output is a pure function of ``(hours, seed, n_speakers)``.
"""

from __future__ import annotations

import bisect
import math
import os
import random
from functools import lru_cache
from typing import Any, Dict, List, Tuple

_ASSET = os.path.join(os.path.dirname(os.path.dirname(__file__)), "assets", "wordfreq.tsv")


@lru_cache(maxsize=1)
def _vocab() -> Tuple[List[str], List[int]]:
    words: List[str] = []
    cum: List[int] = []
    total = 0
    with open(_ASSET, "r", encoding="utf-8") as f:
        for line in f:
            if line.startswith("#"):
                continue
            w, n = line.rstrip("\n").split("\t")
            total += int(n)
            words.append(w)
            cum.append(total)
    return words, cum


def _word(rng: random.Random) -> str:
    words, cum = _vocab()
    return words[bisect.bisect_right(cum, rng.randrange(cum[-1]))]


def synthetic_transcript(hours: float = 1.0, seed: int = 0, n_speakers: int = 1,
                         turn_prob: float = 0.15) -> Dict[str, Any]:
    """Return ``{"segments": [...], "file_info": {...}}`` covering ``hours``."""
    rng = random.Random(seed * 1000003 + int(hours * 3600))
    horizon = hours * 3600.0
    t = 0.0
    speaker = 0
    capital = True
    segments: List[Dict[str, Any]] = []
    while t < horizon:
        dur = min(29.4, max(0.16, math.exp(rng.gauss(1.138, 0.765))))
        n_words = max(1, int(round(dur * 2.6 * rng.uniform(0.6, 1.4))))
        parts: List[str] = []
        for _ in range(n_words):
            if rng.random() < 0.007:
                w = str(rng.randint(1, 2030))
            else:
                w = _word(rng)
            if capital:
                w = w[:1].upper() + w[1:]
                capital = False
            r = rng.random()
            if r < 0.088:
                w += "."
                capital = True
            elif r < 0.162:
                w += ","
            elif r < 0.173:
                w += "?"
                capital = True
            parts.append(w)
        end = min(horizon, t + dur)
        segments.append({"start": round(t, 2), "end": round(end, 2), "text": " ".join(parts),
                         "speaker": "SPEAKER_%02d" % speaker})
        gap = 0.0 if rng.random() < 0.6 else min(156.0, rng.expovariate(1.0 / 3.45))
        t = end + gap
        if n_speakers > 1 and rng.random() < turn_prob:
            speaker = (speaker + rng.randrange(1, n_speakers)) % n_speakers
    return {"segments": segments, "file_info": "synthetic-%gh-seed%d.json" % (hours, seed)}
