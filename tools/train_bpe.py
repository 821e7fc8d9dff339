#!/usr/bin/env python3
"""Train the bundled byte-level BPE vocabulary (``assets/mrsum-bpe.tiktoken``).

Offline, deterministic, build-time only (the runtime never imports
``tokenizers``).  The corpus is chunk-formatted synthetic transcript text
(``utils/synth.py``) plus the bundled prompt files, i.e. exactly the kind of
text the chunker and the aggregator count.  ``--merges`` is calibrated so that
the token count of a transcript is close to cl100k's (see tokenizer.py).

    python tools/train_bpe.py --merges 4000
"""

import argparse
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llm_map_reduce_summarizer_amd.engine.tokenizer import (CL100K_PATTERN, DEFAULT_VOCAB_FILE,  # noqa: E402
                                                            save_tiktoken_file)
from llm_map_reduce_summarizer_amd.pipeline.preprocess import preprocess_transcript, format_timestamp  # noqa: E402
from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript  # noqa: E402


def bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def corpus(hours: float, seeds: int):
    for seed in range(seeds):
        data = synthetic_transcript(hours, seed=1000 + seed, n_speakers=1 + seed % 3)
        for seg in preprocess_transcript(data["segments"]):
            yield "[%s] %s: %s" % (format_timestamp(seg["start"]), seg["speaker"], seg["text"])
    root = os.path.dirname(DEFAULT_VOCAB_FILE)
    for p in sorted(glob.glob(os.path.join(os.path.dirname(root), "prompts", "*.txt"))):
        with open(p, encoding="utf-8") as f:
            yield f.read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--merges", type=int, default=4000)
    ap.add_argument("--hours", type=float, default=10.0)
    ap.add_argument("--seeds", type=int, default=6)
    ap.add_argument("--out", default=DEFAULT_VOCAB_FILE)
    a = ap.parse_args()
    from tokenizers import Regex, Tokenizer, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(CL100K_PATTERN), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False),
    ])
    alphabet = pre_tokenizers.ByteLevel.alphabet()
    trainer = trainers.BpeTrainer(vocab_size=len(alphabet) + a.merges, initial_alphabet=alphabet,
                                  min_frequency=2, show_progress=False)
    tok.train_from_iterator(list(corpus(a.hours, a.seeds)), trainer)
    merges = json.loads(tok.to_str())["model"]["merges"]
    dec = {u: b for b, u in bytes_to_unicode().items()}
    ranks = {bytes([b]): b for b in range(256)}
    for m in merges:
        left, right = (m.split(" ") if isinstance(m, str) else m)
        tb = bytes(dec[c] for c in left + right)
        if tb not in ranks:
            ranks[tb] = len(ranks)
    save_tiktoken_file(a.out, ranks)
    print("wrote %s: %d tokens" % (a.out, len(ranks)))


if __name__ == "__main__":
    main()
