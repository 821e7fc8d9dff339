"""Build provenance: every in-tree native library carries a stamp (sha256 of the sources + flags it was
built from) and the loader refuses a library whose stamp does not match the tree."""
import pytest

from llm_map_reduce_summarizer_amd import _stamp
from llm_map_reduce_summarizer_amd.ops import _lib


def test_built_libraries_match_tree():
    for kind in _stamp.LIBS:
        assert _stamp.check(kind) is None, _stamp.check(kind)
        rec = _stamp.read_stamp(kind)
        assert rec["flags"] == list(_stamp.LIBS[kind][2])
        assert len(rec["files"]) == len(_stamp.sources(kind)) > 0


def test_stamp_covers_every_source_byte(tmp_path):
    a, b = tmp_path / "a.hip", tmp_path / "b.h"
    a.write_text("kernel A")
    b.write_text("header")
    d0 = _stamp.digest([str(a), str(b)], ["-O3"])
    assert _stamp.digest([str(b), str(a)], ["-O3"]) == d0  # order-independent
    assert _stamp.digest([str(a), str(b)], ["-O2"]) != d0  # flags count
    b.write_text("header ")
    assert _stamp.digest([str(a), str(b)], ["-O3"]) != d0  # one byte of a header counts


def test_loader_refuses_stale_kernels(monkeypatch):
    monkeypatch.setattr(_stamp, "tree_stamp", lambda kind: "0" * 64)
    monkeypatch.setattr(_lib, "_kernels", None)
    monkeypatch.setattr(_lib, "_KERNELS_OVERRIDE", None)
    with pytest.raises(_lib.NativeLibraryMissing, match="stale"):
        _lib.kernels_lib()
    assert _lib.native_stamps()["kernels"]["matches_tree"] is False
