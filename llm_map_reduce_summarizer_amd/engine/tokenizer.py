"""Byte-level BPE tokenizer (tiktoken-file compatible) with a native fast path.

The reference counts tokens with ``tiktoken.get_encoding("cl100k_base")`` in
both the chunker (reference ``big_chunkeroosky.py:43,83``) and the aggregator
(``result_aggregator.py:50,389``).  Neither tiktoken nor its vocabulary files
exist on the target machines, so this module implements the same algorithm:

* pre-tokenisation with the cl100k regular expression (Llama-3 uses the same
  family of pattern);
* per-piece byte-pair merging by *rank* (lowest-rank adjacent pair first),
  exactly tiktoken's ``_byte_pair_merge``;
* ranks loaded from a ``*.tiktoken`` file (``base64(token) rank`` per line).

Vocabularies:

* ``MRSUM_TOKENIZER=/path/to/cl100k_base.tiktoken`` (or any Llama-3
  ``tokenizer.model``, which is the same file format) gives exact token-count
  parity with the reference.
* Otherwise the bundled ``assets/mrsum-bpe.tiktoken`` is used: a byte-level BPE
  trained offline (``tools/train_bpe.py``) whose merge count is calibrated so
  token counts on English talk transcripts are close to cl100k's (chunk counts
  of SURVEY.md §4/§6 are reproduced within a few percent).

Llama-3 special tokens live at their real ids (128000+) regardless of the
base vocabulary size, so prompts built with :mod:`.chat` have the Llama-3 chat
structure.  With random-init weights (the benchmark setting) the sampler can
emit ids above the base vocabulary; :meth:`decode` folds those ids into the
base range (``id % n_base``) so generated text is always printable and
re-tokenisable -- see SURVEY.md §7.4 "Random weights never emit EOS".

The per-piece merge loop runs in C++ (``csrc/runtime/bpe.cpp``) when the
runtime library is built; the pure-Python loop below is the oracle and the
fallback.
"""

from __future__ import annotations

import base64
import ctypes
import logging
import os
from typing import Dict, Iterable, List, Optional, Sequence

import re

import numpy as np
import regex

log = logging.getLogger("mrsum.tokenizer")

# CL100K_PATTERN restricted to ASCII input, for the stdlib ``re`` engine (~1.7x the ``regex`` module's speed on
# transcript text): \p{L} -> [A-Za-z], \p{N} -> [0-9], \s -> Unicode White_Space within ASCII ([\t\n\v\f\r ];
# NOT Python's str.isspace set, which adds \x1c-\x1f).  Same pieces as the full pattern on every ASCII string
# (tests/test_tokenizer.py, differential over random strings incl. control characters).
_WS, _NWS = r"[\t\n\x0b\x0c\r ]", r"[^\t\n\x0b\x0c\r ]"
_CL100K_ASCII = re.compile(r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\nA-Za-z0-9]?[A-Za-z]+|[0-9]{1,3}"
                           r"| ?[^\t\n\x0b\x0c\r A-Za-z0-9]+[\r\n]*|" + _WS + r"*[\r\n]+|" + _WS + r"+(?!" + _NWS + r")|"
                           + _WS + r"+")

CL100K_PATTERN = (
    r"""(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+"""
)

LLAMA3_SPECIALS = {
    "<|begin_of_text|>": 128000,
    "<|end_of_text|>": 128001,
    "<|start_header_id|>": 128006,
    "<|end_header_id|>": 128007,
    "<|eot_id|>": 128009,
}

_ASSETS = os.path.join(os.path.dirname(os.path.dirname(__file__)), "assets")
DEFAULT_VOCAB_FILE = os.path.join(_ASSETS, "mrsum-bpe.tiktoken")


def load_tiktoken_file(path: str) -> Dict[bytes, int]:
    ranks: Dict[bytes, int] = {}
    with open(path, "rb") as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith(b"#"):
                continue
            tok, rank = line.split()
            ranks[base64.b64decode(tok)] = int(rank)
    return ranks


def save_tiktoken_file(path: str, ranks: Dict[bytes, int]) -> None:
    with open(path, "wb") as f:
        for tok, rank in sorted(ranks.items(), key=lambda kv: kv[1]):
            f.write(base64.b64encode(tok) + b" " + str(rank).encode() + b"\n")


def bpe_merge_py(piece: bytes, ranks: Dict[bytes, int]) -> List[int]:
    """tiktoken-style rank merge of one pre-token (pure-Python oracle)."""
    if len(piece) == 1:
        return [ranks[piece]]
    r = ranks.get(piece)
    if r is not None:
        return [r]
    parts = [piece[i:i + 1] for i in range(len(piece))]
    while len(parts) > 1:
        best_rank = None
        best_i = -1
        for i in range(len(parts) - 1):
            rk = ranks.get(parts[i] + parts[i + 1])
            if rk is not None and (best_rank is None or rk < best_rank):
                best_rank, best_i = rk, i
        if best_rank is None:
            break
        parts[best_i:best_i + 2] = [parts[best_i] + parts[best_i + 1]]
    return [ranks[p] for p in parts]


class _NativeBPE:
    """ctypes binding of csrc/runtime/bpe.cpp (rank table lives in C++)."""

    def __init__(self, lib: ctypes.CDLL, ranks: Dict[bytes, int]):
        self._lib = lib
        toks = sorted(ranks.items(), key=lambda kv: kv[1])
        blob = b"".join(t for t, _ in toks)
        lens = (ctypes.c_int32 * len(toks))(*[len(t) for t, _ in toks])
        rks = (ctypes.c_int32 * len(toks))(*[r for _, r in toks])
        lib.mrsum_bpe_create.restype = ctypes.c_void_p
        lib.mrsum_bpe_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32),
                                         ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]
        lib.mrsum_bpe_destroy.argtypes = [ctypes.c_void_p]
        lib.mrsum_bpe_encode_pieces.restype = ctypes.c_int64
        lib.mrsum_bpe_encode_pieces.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32),
                                                ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.c_int64]
        self._h = lib.mrsum_bpe_create(blob, lens, rks, len(toks))

    def encode_pieces(self, pieces: Sequence[bytes]) -> List[int]:
        return self.encode_blob(b"".join(pieces), [len(p) for p in pieces]).tolist()

    def encode_blob(self, blob: bytes, lens) -> "np.ndarray":
        """Token ids (int32 array) of the pre-split pieces laid end to end in ``blob`` (``lens``: their byte
        lengths).  Offsets by one numpy cumsum and one C++ call -- no Python loop per piece (the chunker and
        the prompt builder encode ~0.2 M pieces per 10 h pipeline run)."""
        n = len(lens)
        offs = np.zeros(n + 1, dtype=np.int32)
        if n:
            np.cumsum(np.asarray(lens, dtype=np.int32), out=offs[1:])
        cap = max(1, int(offs[-1]))  # never more tokens than bytes
        out = np.empty(cap, dtype=np.int32)
        m = self._lib.mrsum_bpe_encode_pieces(self._h, blob, offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                              n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), cap)
        if m < 0:
            raise RuntimeError("native BPE failed (unknown byte in vocabulary?)")
        return out[:m]

    def __del__(self):
        try:
            self._lib.mrsum_bpe_destroy(self._h)
        except Exception:
            pass


class BPETokenizer:
    """Encode/decode text; ``count`` is what the chunker/aggregator use."""

    def __init__(self, ranks: Dict[bytes, int], pattern: str = CL100K_PATTERN,
                 special_tokens: Optional[Dict[str, int]] = None, name: str = "bpe",
                 use_native: Optional[bool] = None):
        if len(ranks) < 256:
            raise ValueError("a byte-level BPE needs all 256 single-byte tokens")
        self.name = name
        self.ranks = ranks
        self.n_base = max(ranks.values()) + 1
        self.special_tokens = dict(special_tokens if special_tokens is not None else LLAMA3_SPECIALS)
        self._decoder: Dict[int, bytes] = {r: t for t, r in ranks.items()}
        self._special_decoder = {v: k.encode() for k, v in self.special_tokens.items()}
        self._pat = regex.compile(pattern)
        self._ascii_pat = _CL100K_ASCII if pattern == CL100K_PATTERN else None
        self._special_pat = (regex.compile("|".join(regex.escape(s) for s in sorted(self.special_tokens, key=len,
                                                                                   reverse=True)))
                             if self.special_tokens else None)
        self._cache: Dict[bytes, List[int]] = {}
        self._native: Optional[_NativeBPE] = None
        if use_native is None:
            use_native = os.environ.get("MRSUM_NATIVE_BPE", "1") != "0"
        if use_native:
            from ..ops import _lib
            lib = _lib.runtime_lib(required=False)
            if lib is not None:
                self._native = _NativeBPE(lib, ranks)

    # ------------------------------------------------------------------ encode
    @property
    def native(self) -> bool:
        return self._native is not None

    @property
    def eos_ids(self) -> List[int]:
        return [i for k, i in self.special_tokens.items() if k in ("<|end_of_text|>", "<|eot_id|>")]

    def _encode_ordinary_pieces(self, text: str) -> List[bytes]:
        return [m.encode("utf-8") for m in self._pat.findall(text)]

    def _native_ids(self, text: str) -> "np.ndarray":
        """The native path: pre-split ``text`` with the pattern and BPE-merge every piece in one C++ call.  ASCII
        text (the common case) is encoded once as a whole: piece byte lengths = character lengths."""
        if text.isascii():
            strs = (self._ascii_pat or self._pat).findall(text)
            return self._native.encode_blob("".join(strs).encode("ascii"), [len(x) for x in strs])
        strs = self._pat.findall(text)
        pieces = [x.encode("utf-8") for x in strs]
        return self._native.encode_blob(b"".join(pieces), [len(p) for p in pieces])

    def encode_ordinary(self, text: str) -> List[int]:
        if self._native is not None:
            return self._native_ids(text).tolist()
        pieces = self._encode_ordinary_pieces(text)
        out: List[int] = []
        cache = self._cache
        for p in pieces:
            ids = cache.get(p)
            if ids is None:
                ids = bpe_merge_py(p, self.ranks)
                if len(cache) < 500000:
                    cache[p] = ids
            out.extend(ids)
        return out

    def encode(self, text: str, allow_special: bool = False) -> List[int]:
        if not allow_special or self._special_pat is None:
            return self.encode_ordinary(text)
        out: List[int] = []
        pos = 0
        for m in self._special_pat.finditer(text):
            out.extend(self.encode_ordinary(text[pos:m.start()]))
            out.append(self.special_tokens[m.group(0)])
            pos = m.end()
        out.extend(self.encode_ordinary(text[pos:]))
        return out

    def count(self, text: str) -> int:
        if self._native is not None:
            return int(self._native_ids(text).shape[0])
        return len(self.encode_ordinary(text))

    def encode_batch(self, texts: Iterable[str]) -> List[List[int]]:
        return [self.encode_ordinary(t) for t in texts]

    # ------------------------------------------------------------------ decode
    def decode_bytes(self, ids: Iterable[int], skip_special: bool = True) -> bytes:
        dec = self._decoder
        nb = self.n_base
        parts: List[bytes] = []
        for i in ids:
            i = int(i)
            b = dec.get(i)
            if b is None:
                sp = self._special_decoder.get(i)
                if sp is not None:
                    if not skip_special:
                        parts.append(sp)
                    continue
                b = dec.get(i % nb, b"")  # fold synthetic-vocab ids (random weights)
            parts.append(b)
        return b"".join(parts)

    def decode(self, ids: Iterable[int], skip_special: bool = True) -> str:
        return self.decode_bytes(ids, skip_special).decode("utf-8", errors="replace")


_TOKENIZERS: Dict[str, BPETokenizer] = {}


def get_tokenizer(name: Optional[str] = None) -> BPETokenizer:
    """Return a cached tokenizer.

    ``name`` may be a path to a ``.tiktoken`` file, ``"cl100k_base"`` (looked up
    in ``$TIKTOKEN_CACHE_DIR`` / ``$MRSUM_TOKENIZER_DIR``), or ``None`` /
    ``"mrsum-bpe"`` for the bundled vocabulary.  ``$MRSUM_TOKENIZER`` overrides
    the default.
    """
    if name is None:
        name = os.environ.get("MRSUM_TOKENIZER", "mrsum-bpe")
    if name in _TOKENIZERS:
        return _TOKENIZERS[name]
    path = None
    if name in ("mrsum-bpe", "default"):
        path = DEFAULT_VOCAB_FILE
    elif os.path.isfile(name):
        path = name
    else:
        for d in (os.environ.get("MRSUM_TOKENIZER_DIR"), os.environ.get("TIKTOKEN_CACHE_DIR")):
            if d and os.path.isfile(os.path.join(d, name + ".tiktoken")):
                path = os.path.join(d, name + ".tiktoken")
                break
        if path is None:
            log.warning("tokenizer %r not found; using the bundled mrsum-bpe vocabulary", name)
            path = DEFAULT_VOCAB_FILE
    tok = BPETokenizer(load_tiktoken_file(path), name=os.path.basename(path))
    _TOKENIZERS[name] = tok
    return tok
