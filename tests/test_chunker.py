import importlib.util
import os
import sys
import types

import pytest

from llm_map_reduce_summarizer_amd.engine.tokenizer import get_tokenizer
from llm_map_reduce_summarizer_amd.pipeline.chunker import Chunker, split_sentences
from llm_map_reduce_summarizer_amd.pipeline.preprocess import preprocess_transcript

KEYS = {"chunk_index", "end_time", "position_percentage", "segments", "speakers", "start_time", "text",
        "text_with_context", "token_count", "total_chunks"}


def test_budget_and_schema(example_transcript):
    segs = preprocess_transcript(example_transcript["segments"])
    c = Chunker(4000)
    chunks = c.postprocess_chunks(c.chunk_transcript(segs))
    assert 25 <= len(chunks) <= 40
    for i, ch in enumerate(chunks):
        assert set(ch) == KEYS
        assert ch["chunk_index"] == i and ch["total_chunks"] == len(chunks)
        assert ch["token_count"] <= 3850
        assert ch["text_with_context"].startswith("--- TRANSCRIPT CHUNK INFORMATION ---\nTime Range: ")
    # every segment lands in exactly one chunk, in order
    flat = [s for ch in chunks for s in ch["segments"]]
    assert flat == segs
    assert chunks[-1]["position_percentage"] < 100 and chunks[0]["position_percentage"] == 0


def test_chunk_count_scales_with_budget(example_transcript):
    segs = preprocess_transcript(example_transcript["segments"])
    counts = [len(Chunker(m).chunk_transcript(segs)) for m in (2000, 4000, 8000, 16000)]
    assert counts == sorted(counts, reverse=True) and counts[0] > 2 * counts[2]


def test_large_uncombined_segment_split_by_sentences():
    words = " ".join("word%d is here." % i for i in range(600))
    seg = preprocess_transcript([{"start": 0, "end": 600, "text": words, "speaker": "A"}])[0]
    c = Chunker(400, context_tokens=100)
    chunks = c.postprocess_chunks(c.chunk_transcript([seg]))
    assert len(chunks) > 3
    for ch in chunks:
        assert ch["token_count"] <= 300
        for s in ch["segments"]:
            assert s["is_sub_chunk"] and s["speaker"] == "A"


def test_clause_split_keeps_speaker_and_tail():
    long_sentence = ", ".join("clause number %d" % i for i in range(300)) + " unpunctuated tail"
    seg = {"start": 0, "end": 100, "text": long_sentence, "speaker": "SPK", "start_formatted": "00:00",
           "end_formatted": "01:40"}
    c = Chunker(300, context_tokens=50)
    chunks = c.postprocess_chunks(c.chunk_transcript([seg]))
    assert all(s["speaker"] == "SPK" for ch in chunks for s in ch["segments"])
    assert "unpunctuated tail" in chunks[-1]["text"]
    q = Chunker(300, context_tokens=50, reference_quirks=True)
    qchunks = q.postprocess_chunks(q.chunk_transcript([seg]))
    assert any(s["speaker"] == "" for ch in qchunks for s in ch["segments"])  # SURVEY Q9 reproduced
    assert "unpunctuated tail" not in qchunks[-1]["text"]


def test_split_sentences():
    assert split_sentences("Hi there. How are you? Fine!  ok") == ["Hi there.", "How are you?", "Fine!", "ok"]
    assert split_sentences("Pi is 3.14 right.") == ["Pi is 3.14 right."]


def test_overlap_block():
    segs = preprocess_transcript([{"start": i * 10, "end": i * 10 + 9, "text": "sentence %d here." % i,
                                   "speaker": "A" if i % 2 else "B"} for i in range(200)])
    c = Chunker(300, context_tokens=50, overlap_tokens=20, apply_overlap=True)
    chunks = c.chunk_transcript(segs)
    assert "PREVIOUS CONTEXT" not in chunks[0]["text_with_context"]
    assert "PREVIOUS CONTEXT" in chunks[1]["text_with_context"]


def _reference_chunker_module():
    path = "/root/reference/big_chunkeroosky.py"
    if not os.path.isfile(path):
        pytest.skip("reference sources not mounted")
    tok = get_tokenizer()

    class Enc:
        def encode(self, text):
            return tok.encode_ordinary(text)

    fake_tiktoken = types.SimpleNamespace(get_encoding=lambda name: Enc())

    class Punkt:
        def tokenize(self, text):
            return split_sentences(text)

    fake_nltk = types.ModuleType("nltk")
    fake_nltk.data = types.SimpleNamespace(find=lambda *_: True)
    fake_nltk.tokenize = types.SimpleNamespace(PunktSentenceTokenizer=Punkt)
    saved = {k: sys.modules.get(k) for k in ("nltk", "tiktoken")}
    sys.modules["nltk"], sys.modules["tiktoken"] = fake_nltk, fake_tiktoken
    try:
        spec = importlib.util.spec_from_file_location("ref_chunker", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod


@pytest.mark.parametrize("budget", [600, 2000, 4000])
def test_differential_vs_reference(example_transcript, budget, capsys):
    """Same tokenizer + sentence splitter injected into the reference: identical chunks."""
    ref = _reference_chunker_module()
    segs = preprocess_transcript(example_transcript["segments"][:2500], max_segment_duration=600)
    a = Chunker(budget, position_mode="reference", reference_quirks=True)
    mine = a.postprocess_chunks(a.chunk_transcript(segs))
    r = ref.BigChunkeroosky(max_tokens_per_chunk=budget)
    theirs = r.postprocess_chunks(r.chunk_transcript(segs))
    assert mine == theirs
