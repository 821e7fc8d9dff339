"""Golden numbers from SURVEY.md §4 (exact: preprocessing never tokenizes)."""
import importlib.util
import os

import pytest

from llm_map_reduce_summarizer_amd.pipeline import preprocess as P


@pytest.mark.parametrize("kwargs,n_out,n_chars", [
    ({}, 171, 317891),
    ({"merge_same_speaker": False}, 4778, 262730),
    ({"max_segment_duration": 60}, 353, None),
    ({"max_segment_duration": 300}, 68, None),
    ({"time_interval_seconds": 60}, 442, None),
    ({"time_interval_seconds": 300}, 89, None),
    ({"preserve_timestamps": False}, 171, 267337),
])
def test_golden_counts(example_transcript, kwargs, n_out, n_chars):
    out = P.preprocess_transcript(example_transcript["segments"], **kwargs)
    assert len(out) == n_out
    if n_chars is not None:
        assert sum(len(s["text"]) for s in out) == n_chars


def test_clean_text():
    assert P.clean_text("the the  cat sat.Then   it it left!ok") == "the cat sat. Then it left! ok"


def test_clean_text_changes(example_transcript):
    segs = example_transcript["segments"]
    assert sum(P.clean_text(s["text"]) != s["text"] for s in segs) == 134


def test_format_timestamp():
    assert P.format_timestamp(59.9) == "00:59"
    assert P.format_timestamp(3599) == "59:59"
    assert P.format_timestamp(3600) == "01:00:00"
    assert P.format_timestamp(26561.26) == "07:22:41"


def test_schema_and_defaults():
    segs = [{"start": 0, "end": 1, "text": "hi there", "speaker": "A"},
            {"start": 1, "end": 2, "text": "  ", "speaker": "A"},
            {"start": 2, "end": 3, "text": "again", "speaker": "A"},
            {"text": "no times"}]
    out = P.preprocess_transcript(segs)
    assert len(out) == 2
    assert out[0]["is_combined"] and out[0]["original_segments"] == 2
    assert out[0]["text"] == "[00:00] hi there [00:02] again"
    assert set(out[1]) == {"start", "end", "start_formatted", "end_formatted", "speaker", "text"}
    assert out[1]["speaker"] == "" and out[1]["start"] == 0


def test_single_segment_group_returned_as_is():
    seg = {"start": 0, "end": 200, "text": "long", "speaker": "A"}
    out = P.preprocess_transcript([seg, {"start": 200, "end": 300, "text": "x", "speaker": "A"}])
    assert "is_combined" not in out[0] and out[0]["text"] == "long"


def _load_reference_module():
    path = "/root/reference/preprocessor.py"
    if not os.path.isfile(path):
        pytest.skip("reference sources not mounted")
    spec = importlib.util.spec_from_file_location("ref_preprocessor", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("kwargs", [{}, {"time_interval_seconds": 60}, {"time_interval_seconds": 300},
                                    {"merge_same_speaker": False, "time_interval_seconds": 120},
                                    {"max_segment_duration": 45, "preserve_timestamps": False}])
def test_differential_vs_reference(example_transcript, kwargs, capsys):
    """Bit-identical output to the reference implementation (pure stdlib module)."""
    ref = _load_reference_module()
    segs = example_transcript["segments"][:1500]
    assert P.preprocess_transcript(segs, **kwargs) == ref.preprocess_transcript(segs, **kwargs)


def test_multispeaker_synthetic_differential():
    from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
    ref = _load_reference_module()
    segs = synthetic_transcript(1.0, seed=3, n_speakers=3)["segments"]
    for kw in ({}, {"time_interval_seconds": 90}):
        assert P.preprocess_transcript(segs, **kw) == ref.preprocess_transcript(segs, **kw)
