import pytest

from llm_map_reduce_summarizer_amd.engine.tokenizer import (BPETokenizer, CL100K_PATTERN, LLAMA3_SPECIALS,
                                                            bpe_merge_py, get_tokenizer, load_tiktoken_file,
                                                            DEFAULT_VOCAB_FILE)

TEXTS = ["Hello world!", "  leading spaces and\ttabs\n\nnewlines", "[14:20] SPEAKER_00: [14:20] So yeah, I mean.",
         "Ünïcödé — émojis 😀🚀 and CJK 漢字", "numbers 1234567 and 3.14159", "it's we've they'll I'M", ""]


@pytest.fixture(scope="module")
def ranks():
    return load_tiktoken_file(DEFAULT_VOCAB_FILE)


@pytest.mark.parametrize("text", TEXTS)
def test_roundtrip(text):
    tok = get_tokenizer()
    assert tok.decode(tok.encode(text)) == text


def test_native_matches_python(ranks):
    py = BPETokenizer(ranks, use_native=False)
    nat = BPETokenizer(ranks, use_native=True)
    if not nat.native:
        pytest.skip("runtime library not built")
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
    lines = [s["text"] for s in synthetic_transcript(0.3, seed=5)["segments"]] + TEXTS
    for t in lines:
        assert nat.encode(t) == py.encode(t)


def test_rank_merge_is_tiktoken_algorithm():
    ranks = {bytes([i]): i for i in range(256)}
    ranks[b"ab"] = 256
    ranks[b"bc"] = 257
    ranks[b"abc"] = 258
    # "abc": lowest-rank pair is "ab" (256) -> [ab, c] -> "abc" (258)
    assert bpe_merge_py(b"abc", ranks) == [258]
    assert bpe_merge_py(b"bcd", ranks) == [257, ord("d")]


def test_specials_and_folding():
    tok = get_tokenizer()
    ids = tok.encode("<|begin_of_text|>hi<|eot_id|>", allow_special=True)
    assert ids[0] == LLAMA3_SPECIALS["<|begin_of_text|>"] and ids[-1] == LLAMA3_SPECIALS["<|eot_id|>"]
    assert tok.decode(ids) == "hi"
    assert "<|eot_id|>" in tok.decode(ids, skip_special=False)
    # ids above the base vocabulary (random weights) fold back into printable tokens
    assert tok.decode([tok.n_base + 5]) == tok.decode([5])
    assert set(tok.eos_ids) == {128001, 128009}


def test_count_close_to_cl100k_scale(example_transcript):
    """Bundled vocab is calibrated to ~cl100k counts (~100-110k for the example)."""
    from llm_map_reduce_summarizer_amd.pipeline.preprocess import preprocess_transcript, format_timestamp
    tok = get_tokenizer()
    segs = preprocess_transcript(example_transcript["segments"])
    n = sum(tok.count("[%s] %s: %s" % (format_timestamp(s["start"]), s["speaker"], s["text"])) for s in segs)
    assert 90000 < n < 115000


def test_ascii_presplit_matches_the_unicode_pattern():
    """The stdlib-``re`` ASCII fast path of the cl100k pre-split gives the same pieces as the ``regex`` pattern on
    ASCII text, control characters included (engine/tokenizer.py _CL100K_ASCII)."""
    import random

    import regex

    from llm_map_reduce_summarizer_amd.engine.tokenizer import _CL100K_ASCII, CL100K_PATTERN
    full = regex.compile(CL100K_PATTERN)
    rng = random.Random(0)
    alpha = "ab AB zZ09'sStTrRvVmMlLdD.,!?-\t\n\r\x0b\x0c\x1c\x1d\x1e\x1f\x00\x7f'   :;[]()\"#"
    for _ in range(5000):
        s = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 48)))
        assert _CL100K_ASCII.findall(s) == full.findall(s), repr(s)
    text = "[00:14] SPEAKER_00: We'll see--it's 3.14159 o'clock!\n\n  Tabs\tand\r\nlines   end  "
    assert _CL100K_ASCII.findall(text) == full.findall(text)
