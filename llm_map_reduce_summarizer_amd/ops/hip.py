"""ctypes bindings of the gfx950 kernel library (``libmrsum_kernels.so``).

Every wrapper validates shapes, dtypes, devices and strides on the host
BEFORE launching -- a kernel never sees an operand it would index out of
bounds (a GPU fault here can reset the whole node) -- then enqueues on the
current torch stream.  Launchers never synchronise or allocate, so every op
is capturable in a hipGraph (``torch.cuda.CUDAGraph``).
"""

from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from ._lib import kernels_lib
from .reference import Fp8Weight

_c_int, _c_float, _vp = ctypes.c_int, ctypes.c_float, ctypes.c_void_p

_SIGS = {
    "mrsum_rmsnorm": [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_float, _vp],
    "mrsum_add_rmsnorm": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_float, _vp],
    "mrsum_rmsnorm_fp8": [_vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_float, _c_int, _vp],
    "mrsum_rope_kv": [_vp, _c_int, _c_int, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int,
                      _c_int, _c_int, _vp],
    "mrsum_rope_kv_parts": [_vp, _c_int, _vp, _c_int, _c_int, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _c_int,
                            _c_int, _c_int, _c_int, _c_int, _vp],
    "mrsum_swiglu": [_vp, _vp, _c_int, _c_int, _vp],
    "mrsum_kv_scatter": [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _c_int, _vp],
    "mrsum_embed": [_vp, _vp, _vp, _c_int, _c_int, _c_int, _vp],
    "mrsum_attn_prefill": [_vp, _c_int, _vp, _vp, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_float, _vp],
    "mrsum_attn_prefill_paged": [_vp, _c_int, _vp, _vp, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_float,
                                 _vp,
                                 _vp, _vp, _c_int, _vp, _vp, _c_int, _vp],
    "mrsum_attn_decode_mfma": [_vp, _c_int, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int,
                               _c_int, _c_int, _c_int, _c_int, _c_float, _vp, _c_int, _vp],
    "mrsum_attn_decode_rope": [_vp, _c_int, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _c_int, _c_int,
                               _c_int, _c_int, _c_int, _c_int, _c_int, _c_float, _vp, _c_int, _vp],
    "mrsum_skinny_gemm": [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _c_int,
                          _c_float, _vp, _c_int, _vp, _vp, _c_int, _vp],
    "mrsum_skinny_resid_capacity_w": [_c_int],
    "mrsum_skinny_lds": [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp],
    "mrsum_stream_gemm": [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp,
                          _vp, _c_int, _c_float, _vp, _c_int, _vp, _c_int, _vp, _vp],
    "mrsum_stream_fp8": [_vp, _c_int, _vp, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp,
                         _vp, _c_int, _c_float, _vp, _c_int, _vp, _vp, _vp],
    "mrsum_skinny_fp8": [_vp, _c_int, _vp, _vp, _c_int, _c_int, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _vp,
                         _c_int, _c_float, _vp, _c_int, _vp, _vp, _c_int, _vp],
    "mrsum_skinny_fp8_resid_capacity": [],
    "mrsum_quant_fp8_rows": [_vp, _c_int, _vp, _vp, _c_int, _c_int, _vp],
    "mrsum_add_rmsnorm_parts": [_vp, _c_int, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_float, _vp],
    "mrsum_sample_keys": [_vp, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp],
    "mrsum_sample_finish": [_vp, _vp, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _c_int, _vp],
    "mrsum_gemm": [_vp, _c_int, _vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _c_int,
                   _c_int, _vp],
    "mrsum_sample": [_vp, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _vp, _vp,
                     _vp],
}

_fns = {}


def _fn(name: str):
    f = _fns.get(name)
    if f is None:
        lib = kernels_lib()
        f = getattr(lib, name)
        f.argtypes = _SIGS[name]
        f.restype = ctypes.c_int
        _fns[name] = f
    return f


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


DEBUG_SYNC = os.environ.get("MRSUM_DEBUG_SYNC", "0") == "1"


def _check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError("%s launch failed: hipError %d" % (name, rc))
    if DEBUG_SYNC and not torch.cuda.is_current_stream_capturing():
        # debug mode (cli --debug-sync): wait for the kernel so an asynchronous fault is reported here,
        # against the op that caused it, instead of at some later synchronisation point
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError("%s: device error after the launch: %s" % (name, e)) from e


def _req(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def _bf16_cuda(*ts: torch.Tensor) -> None:
    for t in ts:
        _req(t.is_cuda and t.dtype == torch.bfloat16, "expected a bf16 CUDA tensor, got %s %s" % (t.dtype, t.device))


def _i32(*ts: torch.Tensor) -> None:
    for t in ts:
        _req(t.is_cuda and t.dtype == torch.int32 and t.is_contiguous(), "expected a contiguous int32 CUDA tensor")


def _rows_ok(x: torch.Tensor) -> None:
    _req(x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0,
         "expected a 2-D row-major tensor with 16-byte aligned rows")


# ------------------------------------------------------------------ norms
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _bf16_cuda(x, w)
    _rows_ok(x)
    T, D = x.shape
    _req(w.numel() == D and w.is_contiguous() and D % 8 == 0 and D <= 16384, "rmsnorm: bad weight / D")
    if out is None:
        out = torch.empty(T, D, dtype=x.dtype, device=x.device)
    _rows_ok(out)
    _req(out.shape == (T, D), "rmsnorm: bad out shape")
    _check(_fn("mrsum_rmsnorm")(_p(x), _p(w), _p(out), T, D, x.stride(0), out.stride(0), eps, _stream()),
           "rmsnorm")
    return out


def add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _bf16_cuda(x, residual, w)
    _rows_ok(x)
    T, D = x.shape
    _req(residual.shape == (T, D) and residual.is_contiguous(), "add_rmsnorm: residual must be [T, D] contiguous")
    _req(w.numel() == D and D % 8 == 0 and D <= 16384, "add_rmsnorm: bad weight / D")
    if out is None:
        out = torch.empty(T, D, dtype=x.dtype, device=x.device)
    _rows_ok(out)
    _check(_fn("mrsum_add_rmsnorm")(_p(x), _p(residual), _p(w), _p(out), T, D, x.stride(0), out.stride(0), eps,
                                    _stream()), "add_rmsnorm")
    return out


def rmsnorm_fp8(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
                split: bool = False):
    """rmsnorm(x) * w -- or residual += x; rmsnorm(residual) * w -- quantised in the same pass to row-wise
    e4m3fn (the fp8 prefill GEMM's input, as quant_fp8_rows): returns (q [T, D] float8_e4m3fn, scale [T]).
    ``split``: two-term rows q [T, 2 D] = [hi | lo], lo = e4m3(16 (y / s - hi)) (norm.hip Q8 == 2), which
    gemm_fp8 takes as a 2D-deep product with the lo half scaled by 2^-4."""
    _bf16_cuda(x, w)
    _rows_ok(x)
    T, D = x.shape
    _req(w.numel() == D and w.is_contiguous() and D % 16 == 0 and D <= 16384, "rmsnorm_fp8: bad weight / D")
    if residual is not None:
        _bf16_cuda(residual)
        _req(residual.shape == (T, D) and residual.is_contiguous(), "rmsnorm_fp8: residual must be [T, D] contiguous")
    q = torch.empty(T, 2 * D if split else D, dtype=torch.float8_e4m3fn, device=x.device)
    sc = torch.empty(T, dtype=torch.float32, device=x.device)
    _check(_fn("mrsum_rmsnorm_fp8")(_p(x), _p(residual), _p(w), _p(q), _p(sc), T, D, x.stride(0), q.shape[1], eps,
                                    1 if split else 0, _stream()), "rmsnorm_fp8")
    return q, sc


# ------------------------------------------------------------------ kv cache formats
KV8_PAGE, KV8_D = 64, 128
KV8_SLAB = KV8_PAGE * KV8_D + 4 * KV8_PAGE  # csrc/kernels/kv8.h: e4m3 rows then fp32 row scales


def _cache_kind(kcache: torch.Tensor, vcache: torch.Tensor, hkv: int, page: int, d: int, what: str) -> int:
    """The kernels' cache-format bitmask: bit 0 = the K cache, bit 1 = the V cache is the fp8 byte-slab layout
    [pages, hkv, KV8_SLAB] uint8 (kv8.h), else bf16 [pages, hkv, page, d] -- 0 (bf16), 3 (fp8) or 2 (fp8v:
    bf16 K, fp8 V); validates shape / dtype / contiguity of both (an fp8 K with a bf16 V is refused)."""
    _req(kcache is not None and vcache is not None and kcache.is_cuda and vcache.is_cuda
         and kcache.is_contiguous() and vcache.is_contiguous() and kcache.shape[0] == vcache.shape[0],
         "%s: K / V caches must be contiguous CUDA tensors with the same pages" % what)
    kind = 0
    for bit, c in ((1, kcache), (2, vcache)):
        if c.dtype == torch.uint8:
            _req(page == KV8_PAGE and d == KV8_D and tuple(c.shape[1:]) == (hkv, KV8_SLAB),
                 "%s: fp8 cache must be uint8 [pages, Hkv, %d] (page 64, head dim 128)" % (what, KV8_SLAB))
            kind |= bit
        else:
            _req(c.dtype == torch.bfloat16 and tuple(c.shape[1:]) == (hkv, page, d),
                 "%s: cache must be bf16 [pages, Hkv, P, D] (or the fp8 slab layout)" % what)
    _req(kind != 1, "%s: an fp8 K cache needs an fp8 V cache (formats: bf16, fp8, fp8v)" % what)
    return kind


# ------------------------------------------------------------------ rope + kv
def rope_kv(qkv: torch.Tensor, positions: torch.Tensor, seq_idx: torch.Tensor, block_tables: torch.Tensor,
            kcache: Optional[torch.Tensor], vcache: Optional[torch.Tensor], cos_sin: torch.Tensor,
            hq: int, hkv: int, d: int, page: int, write_cache: bool = True, check_bounds: bool = False) -> None:
    _bf16_cuda(qkv)
    _rows_ok(qkv)
    T = qkv.shape[0]
    if T == 0:
        return
    _req(qkv.shape[1] >= (hq + 2 * hkv) * d and d in (64, 128), "rope_kv: qkv too narrow / bad head dim")
    _i32(positions, seq_idx, block_tables)
    _req(positions.numel() >= T and seq_idx.numel() >= T, "rope_kv: positions/seq_idx shorter than T")
    _req(cos_sin.is_cuda and cos_sin.dtype == torch.float32 and cos_sin.is_contiguous()
         and cos_sin.shape[1:] == (d // 2, 2), "rope_kv: cos_sin must be [max_pos, D/2, 2] fp32")
    kv8 = 0
    if write_cache:
        kv8 = _cache_kind(kcache, vcache, hkv, page, d, "rope_kv")
        _req(block_tables.dim() == 2, "rope_kv: block_tables must be 2-D")
    if check_bounds:  # host sync; used by tests and prefill (positions live on the host there anyway)
        pmax = int(positions[:T].max())
        _req(pmax < cos_sin.shape[0], "rope_kv: position %d beyond rope table" % pmax)
        if write_cache:
            _req(pmax // page < block_tables.shape[1], "rope_kv: position beyond block table")
            _req(int(seq_idx[:T].max()) < block_tables.shape[0] and int(seq_idx[:T].min()) >= 0, "rope_kv: seq_idx")
    _check(_fn("mrsum_rope_kv")(_p(qkv), T, qkv.stride(0), _p(positions), _p(seq_idx), _p(block_tables),
                                block_tables.stride(0), _p(kcache) if write_cache else None,
                                _p(vcache) if write_cache else None, _p(cos_sin), hq, hkv, d, page,
                                1 if write_cache else 0, kv8, _stream()), "rope_kv")


def rope_kv_parts(parts: torch.Tensor, positions: torch.Tensor, seq_idx: torch.Tensor, block_tables: torch.Tensor,
                  kcache: torch.Tensor, vcache: torch.Tensor, cos_sin: torch.Tensor, hq: int, hkv: int, d: int,
                  page: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum the QKV GEMM's fp32 split-K slabs [S, T, (hq+2hkv)d], rotate Q/K, write bf16 qkv + paged K/V."""
    _req(parts.is_cuda and parts.dtype == torch.float32 and parts.is_contiguous() and parts.dim() == 3,
         "rope_kv_parts: parts must be fp32 [S, T, W]")
    S, T, W = parts.shape
    _req(W == (hq + 2 * hkv) * d and d in (64, 128), "rope_kv_parts: width")
    _i32(positions, seq_idx, block_tables)
    _req(positions.numel() >= T and seq_idx.numel() >= T and block_tables.dim() == 2, "rope_kv_parts: tables")
    _req(cos_sin.is_cuda and cos_sin.dtype == torch.float32 and cos_sin.shape[1:] == (d // 2, 2), "cos_sin")
    kv8 = _cache_kind(kcache, vcache, hkv, page, d, "rope_kv_parts")
    if out is None:
        out = torch.empty(T, W, dtype=torch.bfloat16, device=parts.device)
    _rows_ok(out)
    _check(_fn("mrsum_rope_kv_parts")(_p(parts), S, _p(out), T, out.stride(0), _p(positions), _p(seq_idx),
                                      _p(block_tables), block_tables.stride(0), _p(kcache), _p(vcache), _p(cos_sin),
                                      hq, hkv, d, page, kv8, _stream()), "rope_kv_parts")
    return out


def kv_scatter(rows: torch.Tensor, page: torch.Tensor, slot: torch.Tensor, kcache: torch.Tensor,
               vcache: torch.Tensor) -> None:
    """kcache / vcache [pages, hkv, P, d] at (page[i], slot[i]) <- rows[i, 0] / rows[i, 1] ([n, 2, hkv, d] bf16;
    page < 0: skipped).  The K/V rows a context-parallel prefill all-gathers from the other ranks (bf16
    caches only: an fp8-KV engine does not run the context-parallel prefill)."""
    _bf16_cuda(rows, kcache, vcache)
    _i32(page, slot)
    n = rows.shape[0]
    _req(rows.is_contiguous() and rows.dim() == 4 and rows.shape[1] == 2 and tuple(rows.shape[2:]) ==
         (kcache.shape[1], kcache.shape[3]), "kv_scatter: rows must be [n, 2, hkv, d]")
    _req(kcache.is_contiguous() and vcache.is_contiguous() and kcache.shape == vcache.shape, "kv_scatter: cache")
    _req(page.numel() >= n and slot.numel() >= n, "kv_scatter: index")
    _check(_fn("mrsum_kv_scatter")(_p(rows), n, kcache.shape[1], kcache.shape[3], _p(page), _p(slot), _p(kcache),
                                   _p(vcache), kcache.shape[2], _stream()), "kv_scatter")


# ------------------------------------------------------------------ activations
def swiglu(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _bf16_cuda(gu)
    _req(gu.dim() == 2 and gu.is_contiguous() and gu.shape[1] % 32 == 0, "swiglu: gu must be [T, 2F], F % 16 == 0")  # noqa
    T, F = gu.shape[0], gu.shape[1] // 2
    if out is None:
        out = torch.empty(T, F, dtype=gu.dtype, device=gu.device)
    _req(out.is_contiguous() and out.shape == (T, F), "swiglu: bad out")
    _check(_fn("mrsum_swiglu")(_p(gu), _p(out), T, F, _stream()), "swiglu")
    return out


def embed(ids: torch.Tensor, table: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _i32(ids)
    _bf16_cuda(table)
    _req(table.is_contiguous() and table.shape[1] % 8 == 0, "embed: table must be [V, D] contiguous")
    T = ids.numel()
    V, D = table.shape
    if out is None:
        out = torch.empty(T, D, dtype=table.dtype, device=table.device)
    _req(out.is_contiguous() and out.shape == (T, D), "embed: bad out")
    _check(_fn("mrsum_embed")(_p(ids), _p(table), _p(out), T, D, V, _stream()), "embed")
    return out


# ------------------------------------------------------------------ attention
def prefill_block_m(group: int) -> int:
    """Query positions per prefill-attention workgroup for ``group`` = Hq / Hkv query heads per kv head
    (attn_prefill.hip: 8 waves x 32 rows cover all ``group`` heads of one kv head; any other ratio, e.g.
    Llama-3.2-3B's 3, runs one query head per workgroup over 256 positions)."""
    _req(1 <= group <= 64, "attn_prefill: GQA ratio %d out of range" % group)
    return 256 // group if group in (1, 2, 4, 8) else 256


def prefill_items(seqlens, group: int) -> torch.Tensor:
    """(sequence, query-block start) work list for GQA ratio ``group`` = Hq / Hkv, heaviest (latest) blocks
    first."""
    block_m = prefill_block_m(group)
    items = []
    for s, n in enumerate(seqlens):
        for qb in range(0, int(n), block_m):
            items.append((qb, s))
    items.sort(key=lambda x: -x[0])
    return torch.tensor([(s, qb) for qb, s in items], dtype=torch.int32).reshape(-1, 2)


def attn_prefill(qkv: torch.Tensor, cu_seqlens: torch.Tensor, hq: int, hkv: int, d: int, scale: float,
                 out: Optional[torch.Tensor] = None, items: Optional[torch.Tensor] = None,
                 seqlens=None, paged=None) -> torch.Tensor:
    """Causal varlen prefill attention.  ``paged`` (ops.PagedPrefill): the packed rows are slices whose
    keys are read from the paged cache for positions [0, prefix + slice length) -- chunked prefill."""
    _bf16_cuda(qkv)
    _rows_ok(qkv)
    _req(d == 128 and hq % hkv == 0 and qkv.shape[1] >= (hq + 2 * hkv) * d, "attn_prefill: bad head config")
    _i32(cu_seqlens)
    T = qkv.shape[0]
    if seqlens is None:
        cu = cu_seqlens.cpu().tolist()
        seqlens = [b - a for a, b in zip(cu[:-1], cu[1:])]
        _req(cu[0] == 0 and cu[-1] <= T and all(n >= 0 for n in seqlens), "attn_prefill: bad cu_seqlens")
    block_m = prefill_block_m(hq // hkv)
    if items is None:
        items = prefill_items(seqlens, hq // hkv).to(qkv.device)
    # a list built for another GQA ratio has another block count (same-count collisions need every
    # sequence shorter than both block sizes, where the blocks cover the same rows anyway)
    _req(items.shape[0] == sum(-(-int(n) // block_m) for n in seqlens),
         "attn_prefill: work list not built for GQA ratio %d (prefill_items(seqlens, %d))" % (hq // hkv, hq // hkv))
    _i32(items)
    if out is None:
        out = torch.empty(T, hq * d, dtype=qkv.dtype, device=qkv.device)
    _rows_ok(out)
    _req(out.shape[0] >= T and out.shape[1] >= hq * d, "attn_prefill: bad out")
    if paged is not None:
        kc, vc, bt = paged.kcache, paged.vcache, paged.block_tables
        kv8 = _cache_kind(kc, vc, hkv, 64, d, "attn_prefill")
        _i32(bt, paged.seq_slot, paged.prefix)
        _req(bt.dim() == 2 and len(paged.prefix_host) == len(seqlens) == paged.seq_slot.numel(),
             "attn_prefill: paged tables")
        for pre, n, slot in zip(paged.prefix_host, seqlens, paged.slot_host):
            _req(0 <= slot < bt.shape[0] and pre >= 0 and pre + n <= bt.shape[1] * 64,
                 "attn_prefill: slice [%d, %d) beyond block table" % (pre, pre + n))
        _check(_fn("mrsum_attn_prefill_paged")(_p(qkv), qkv.stride(0), _p(cu_seqlens), _p(items), items.shape[0],
                                               block_m, _p(out), out.stride(0), hq, hkv, d, scale, _p(kc), _p(vc), _p(bt),
                                               bt.stride(0), _p(paged.seq_slot), _p(paged.prefix), kv8, _stream()),
               "attn_prefill_paged")
        return out
    _check(_fn("mrsum_attn_prefill")(_p(qkv), qkv.stride(0), _p(cu_seqlens), _p(items), items.shape[0], block_m, _p(out),
                                     out.stride(0), hq, hkv, d, scale, _stream()), "attn_prefill")
    return out


def decode_splits(batch: int, hkv: int, max_ctx: int, target_wgs: int = 1024, max_splits: int = 32) -> int:
    """Split-K count for decode attention (measured, MFMA kernel, tools/bench_kernels.py: B=1 ctx 8k: S 16-32
    -> 18 us vs S 4 -> 40 us; B=8 ctx 4k: S 8 -> 27 us (5.0 TB/s); B=39 ctx 4.4k: S 4-8 -> 131-140 us
    (5.0-5.35 TB/s); B=64 ctx 2k: S 2-4 -> 104 us)."""
    s = max(1, -(-target_wgs // max(1, batch * hkv)))
    s = min(s, max_splits, max(1, -(-max_ctx // 64)))
    return s


MAX_SPLITS = 256  # attn_decode.hip MAX_SPLITS: splits of one (sequence, kv head) the merge takes
TP_SHARD_MAX_SPLITS = 128  # decode_attn_plan_bf16: a TP shard's kv head beyond 6k (measured, see there)
ATTN_PAGES_PER_SPLIT = 2  # at least 2 pages per split (1 measured slower at B=1: r1_attn_splits_ab.jsonl)


CTX_CLASSES = (6144, 12288, 32768, 1 << 30)  # decode context classes (tokens): graphs / split plans per class


def ctx_class(ctx: int) -> int:
    """Index of the context class holding ``ctx`` tokens (0: <= 6k, 1: <= 12k, 2: <= 32k, 3: longer)."""
    for i, c in enumerate(CTX_CLASSES):
        if ctx <= c:
            return i
    return len(CTX_CLASSES) - 1


ATTN_SLOTS = 768  # resident decode-attention workgroups (3 per CU, 162 VGPRs; 512 / 1024 measured equal or worse)


# fp8 KV cache: a page is half the bytes, so the same split plan keeps half the bytes in flight per CU.  Whole
# decode steps at 4.4k context with the splits x 1 / 2 / 3 (profiles/r4_kv8_split_sweep.jsonl): B = 10 (80
# groups) 4.036 / 3.901 / 3.996 ms, B = 20 4.469 / 4.705 / 4.639, B = 39 5.649 / 5.942 / 6.187 -- so twice the
# splits up to KV8_SPLIT_GROUPS (sequence, kv head) groups, the bf16 plan above them
KV8_SPLIT_GROUPS = 96


def decode_attn_plan(batch: int, hkv: int, max_ctx: int, kv8=False):
    """(splits, fused) of decode_attn_plan_bf16; with ``kv8`` True / "fp8" (fp8 K and V cache) the measured
    split multiplier (at most one page per split; a fused merge keeps its 16-split cap).  "fp8v" (bf16 K,
    fp8 V: 3/4 of the bf16 bytes per page) keeps the bf16 plan."""
    s, fused = decode_attn_plan_bf16(batch, hkv, max_ctx)
    if kv8 is True or kv8 == "fp8":
        mult = 2.0 if batch * hkv <= KV8_SPLIT_GROUPS else 1.0
        pages = max(1, -(-max_ctx // 64))
        s = max(1, min(int(round(s * mult)), pages, 64, 16 if fused else 64))
    return s, fused


def decode_attn_plan_bf16(batch: int, hkv: int, max_ctx: int):
    """(splits, fused_combine) of the decode attention of ``batch`` sequences x ``hkv`` kv heads whose
    contexts reach ``max_ctx`` tokens (the engine passes its context class's upper bound).

    Splits: as many (sequence, kv head, split) workgroups as fit on the chip AT ONCE (ATTN_SLOTS = 3
    resident workgroups per CU x 256 CUs: the kernel keeps two 32 KiB K+V tiles in flight per
    workgroup in registers, 162 VGPRs) -- never more, so all splits run in one round (at B=39 x 8 kv
    heads the previous ceil(1024 / groups) = 4 splits made 1248 workgroups = two rounds) -- and at
    least ATTN_PAGES_PER_SPLIT pages each, at most 64.  Fused = the split merge runs in the attention
    launch, by the last split of each (sequence, kv head) to arrive, with write-through (sc1) partial
    stores and no release fence; "auto": fused up to 128 (sequence, kv head) groups with at most 16
    splits (<= 16 groups) or 4 splits (the merging workgroup reads every split's partials)."""
    pages = max(1, -(-max_ctx // 64))
    groups = max(1, batch * hkv)
    splits = max(1, min(ATTN_SLOTS // groups, -(-pages // ATTN_PAGES_PER_SPLIT), 64))
    if pages <= 96:
        # the <= 6k context class (profiles/r2_attn_decode_split_sweep_4k.jsonl, B = 2..39 x splits 2..16; TP=4 / 8 shard head counts: r2_attn_decode_split_sweep_tp_shards_4k.jsonl):
        # best at ~one workgroup per CU for small batches (B=5: 6 splits 22.6 us vs 4 25.0; B=10: 3 splits
        # 33.4 vs 4 38.7) and 3 splits from 80 groups up (B=20 60.2 vs 65.3, B=39 111.9 vs 113.9)
        splits = max(1, min(max(3, N_CU // groups), -(-pages // ATTN_PAGES_PER_SPLIT), 64))
        if groups >= 256:
            # B = 39 x 8 kv heads in situ after the sc1 merge loads (profiles/r3_plans_insitu_b39_b10.jsonl):
            # 4 separate splits 6.68 / 6.77 ms per step vs 3 6.86 / 6.86, 2 6.95 / 6.99, 6 6.96 / 6.88
            splits = min(4, -(-pages // ATTN_PAGES_PER_SPLIT))
    # measured (tools/bench_attn_decode.py; profiles/r2_attn_decode_splits_fused_sweep.jsonl at 4k,
    # r2_attn_decode_splits_10k.jsonl, r2_attn_decode_b1_class0.jsonl): B=1 4k fused 16 splits 16.1-18.0 us
    # vs 32-48 unfused 19.0-21.4, 6k fused 16 17.0 vs 47 unfused 19.9, but B=1 10k 64 unfused 19.5 vs 16
    # fused 21.0 (a fused merge caps the splits, and long splits serialise); B=10 fused 4 splits 37.5 us
    # vs 9 unfused 40.1 at 4k, equal at 10k; B=39 unfused 113 vs fused 116-118
    if groups <= 16:
        fused = -(-pages // 16) <= 6  # the <= 6k context class
        if fused and hkv <= 2:
            # a TP shard's one or two kv heads: one workgroup per page (up to one per CU), separate merge --
            # in situ after the sc1 merge loads (TP=8 shard at 4k, whole decode steps, profiles/
            # r3_plans_insitu_sc1.jsonl): B=1 64 separate 1.370 ms vs 32 fused 1.39, 16 fused 1.451;
            # B=10 25 separate 1.600 vs 24 fused 1.615, 16 fused 1.623
            return max(1, min(N_CU // groups, pages, 64)), False
        if not fused and hkv <= 2:
            # a TP shard's one or two kv heads beyond the 6k class (config 5's 32k final reduce at TP=8): the
            # TP=1 rule below leaves B=1 at 32 workgroups.  Up to ATTN_SLOTS workgroups of >= 2 pages, at most
            # TP_SHARD_MAX_SPLITS separate splits.  In situ, whole steps (profiles/r5_attn_plans*.jsonl): 70B fp8
            # TP=8 shard at B=1, 32k -- 32 / 64 / 128 / 250 splits 5.66 / 5.07 / 4.80 / 5.10 ms (the merge of
            # 250 splits costs more than the wider attention gains); 8B TP=8 shard at 13.5k -- 106 splits
            # 1.24 ms vs 64 1.28, 32 1.29
            return max(1, min(ATTN_SLOTS // groups, -(-pages // ATTN_PAGES_PER_SPLIT), TP_SHARD_MAX_SPLITS)), False
        if fused and batch == 1 and hkv >= 8 and pages > 32:
            # one sequence x 8 kv heads: 32 splits with the separate merge beat 16 fused in situ (whole decode
            # steps, 4k context: 3.47 vs 3.55 ms; profiles/r2_attn_plans_insitu_b1_b10.jsonl), as in the
            # <= 12k class below -- the kernel microbench had ranked them the other way
            fused = False
            splits = min(splits, 32)
        elif fused:
            splits = min(splits, 16)
        elif pages <= 512:
            # the <= 12k class at B=1 (profiles/r2_attn_decode_b1_class1.jsonl, 7 rounds x 64 calls): 32 separate
            # splits 18.6 / 17.5 us at 8k / 10k against 64 splits 18.9 / 18.8 and every fused variant >= 19.1;
            # the <= 32k class likewise (r2_attn_decode_b1_class2.jsonl: 16k 22.1 vs 24.1 us, 32k 32.5 vs 33.9)
            splits = min(splits, 32)
    else:
        fused = groups <= 128
        if fused:
            # B=5 at 4k: 6 splits fused 22.6 us, unfused 23.3; a TP shard's one or two kv heads at B=20 (20 groups,
            # 4k) take 12 fused splits: 1.971 / 1.971 ms per TP=8 shard step vs 8 fused 2.020 / 2.016, 12
            # separate 1.984 (in situ, profiles/r3_plans_insitu_tp8_b39_b20.jsonl).  Longer contexts (the <= 12k
            # class: the level-1 reduce) take 6 fused splits -- in situ at ~6k (profiles/
            # r4_attn_plans_insitu_class1.jsonl; ``batch`` here is the graph's bucket): batch 5 in bucket 8
            # 3.92 ms per step vs 4.10 with 4 splits, batch 10 in bucket 16 4.52 vs 4.64 (3 splits tie)
            if pages <= 96:
                splits = min(splits, 12 if hkv <= 2 else 8)
            else:
                splits = min(splits, 4 if hkv <= 2 else 6)
    return splits, fused


def decode_groups(hq: int, hkv: int) -> int:
    """Head groups the decode attention runs (attn_decode.hip mrsum_attn_decode_groups): hkv for GQA ratios
    1/2/4/8/16, hq (one per query head) for any other ratio -- size workspaces / split plans by it."""
    _req(hkv > 0 and hq % hkv == 0 and hq // hkv <= 64, "decode attention: bad head config %d / %d" % (hq, hkv))
    return hkv if hq // hkv in (1, 2, 4, 8, 16) else hq


class DecodeWorkspace:
    """Split-K partial buffers + per-(seq, kv head) arrival counters for attn_decode
    (allocated once per batch bucket; counters start at 0 and every launch re-arms them).
    (A third merge placement -- every workgroup of the o projection merging one row's splits into LDS under
    its weight loads -- measured equal at a TP=8 shard's 4k and 8 % slower at 13.5k, the partials re-read
    by every workgroup costing what the merge launch did: profiles/r5_consumer_merge_ab.jsonl.  Removed.)"""

    def __init__(self, batch: int, hq: int, d: int, splits: int, device, hkv: Optional[int] = None,
                 fused_combine: bool = False):
        # fused_combine (last-arriver merge inside the split kernel) measured SLOWER than the separate
        # merge kernel at every B >= 8 (the per-workgroup drain + agent release costs more than the
        # launch boundary it saves: B=39 238 vs 189 us), so the separate kernel is the default.
        self.splits = splits
        self.part_o = torch.empty(batch * hq * splits * d, dtype=torch.float32, device=device)
        self.part_ml = torch.empty(batch * hq * splits * 2, dtype=torch.float32, device=device)
        self.counters = (torch.zeros(batch * (hkv or hq), dtype=torch.int32, device=device)
                         if fused_combine else None)



def attn_decode_rope(parts: torch.Tensor, cos_sin: torch.Tensor, kcache: torch.Tensor, vcache: torch.Tensor,
                     block_tables: torch.Tensor, positions: torch.Tensor, hq: int, hkv: int, d: int, page: int,
                     scale: float, out: Optional[torch.Tensor] = None,
                     workspace: Optional[DecodeWorkspace] = None) -> torch.Tensor:
    """Decode attention from the QKV GEMM's fp32 split-K slabs ``parts`` [S, B, (hq + 2 hkv) d]: RoPE of
    q and of the new token's k, K/V write into the paged cache and the attention itself in one launch
    (+ the split merge): the rope_kv_parts kernel of the unfused path disappears."""
    _req(parts.is_cuda and parts.dtype == torch.float32 and parts.is_contiguous() and parts.dim() == 3,
         "attn_decode_rope: parts must be fp32 [S, B, width]")
    SP, B, width = parts.shape
    _req(width == (hq + 2 * hkv) * d and d == 128 and page == 64 and hq % hkv == 0 and hq // hkv <= 64,
         "attn_decode_rope: unsupported config")
    ng = decode_groups(hq, hkv)
    kv8 = _cache_kind(kcache, vcache, hkv, page, d, "attn_decode_rope")
    _req(cos_sin.dtype == torch.float32 and cos_sin.is_contiguous() and cos_sin.shape[-2:] == (d // 2, 2),
         "attn_decode_rope: cos_sin [max_pos, d/2, 2] fp32")
    _i32(block_tables, positions)
    _req(block_tables.dim() == 2 and block_tables.shape[0] >= B and positions.numel() >= B, "attn_decode_rope: tables")
    if workspace is None:
        workspace = DecodeWorkspace(B, hq, d, decode_splits(B, ng, block_tables.shape[1] * page), parts.device, ng)
    _req(workspace.part_o.numel() >= B * hq * workspace.splits * d and workspace.part_ml.numel() >=
         B * hq * workspace.splits * 2 and (workspace.counters is None or workspace.counters.numel() >= B * ng),
         "attn_decode_rope: workspace")
    if out is None:
        out = torch.empty(B, hq * d, dtype=torch.bfloat16, device=parts.device)
    _rows_ok(out)
    _check(_fn("mrsum_attn_decode_rope")(_p(parts), SP, _p(cos_sin), _p(kcache), _p(vcache), _p(block_tables),
                                         block_tables.stride(0), _p(positions), _p(workspace.part_o),
                                         _p(workspace.part_ml), _p(out), out.stride(0), B, hq, hkv, d, page,
                                         workspace.splits, scale, _p(workspace.counters), kv8, _stream()),
           "attn_decode_rope")
    return out


def attn_decode(q: torch.Tensor, kcache: torch.Tensor, vcache: torch.Tensor, block_tables: torch.Tensor,
                positions: torch.Tensor, hq: int, hkv: int, d: int, page: int, scale: float,
                out: Optional[torch.Tensor] = None, num_splits: Optional[int] = None,
                workspace: Optional[DecodeWorkspace] = None) -> torch.Tensor:
    """Paged decode attention on MFMA (page 64, G = hq / hkv <= 16): K/V pages staged through LDS,
    QK^T and PV on MFMA, split-K over the context with a fused or separate split merge."""
    _bf16_cuda(q)
    _rows_ok(q)
    B = q.shape[0]
    _req(d == 128 and hq % hkv == 0 and hq // hkv <= 64 and page == 64, "attn_decode: bad config")
    ng = decode_groups(hq, hkv)
    kv8 = _cache_kind(kcache, vcache, hkv, page, d, "attn_decode")
    _i32(block_tables, positions)
    _req(block_tables.dim() == 2 and block_tables.shape[0] >= B and positions.numel() >= B, "attn_decode: tables")
    if workspace is None:
        s = num_splits or decode_splits(B, ng, block_tables.shape[1] * page)
        workspace = DecodeWorkspace(B, hq, d, s, q.device, ng)
    _req(workspace.part_o.numel() >= B * hq * workspace.splits * d, "attn_decode: workspace too small")
    _req(workspace.counters is None or workspace.counters.numel() >= B * ng, "attn_decode: counters too small")
    if out is None:
        out = torch.empty(B, hq * d, dtype=q.dtype, device=q.device)
    _rows_ok(out)
    _check(_fn("mrsum_attn_decode_mfma")(_p(q), q.stride(0), _p(kcache), _p(vcache), _p(block_tables),
                                         block_tables.stride(0), _p(positions), _p(workspace.part_o),
                                         _p(workspace.part_ml), _p(out), out.stride(0), B, hq, hkv, d, page,
                                         workspace.splits, scale, _p(workspace.counters), kv8, _stream()),
           "attn_decode_mfma")
    return out


# ------------------------------------------------------------------ sampler
def _eos_ok(st) -> None:
    # the finish kernel reads EOS_SLOTS (4) stop ids from device memory at every launch (-1 = unused):
    # the stop set is state, never a by-value launch argument a captured graph would freeze
    _req(st.eos.is_cuda and st.eos.dtype == torch.int32 and st.eos.is_contiguous() and st.eos.numel() == 4,
         "sample: eos must be 4 int32 device slots")


def sample(logits: torch.Tensor, st) -> None:
    """Sample one token per row of ``logits`` into decode state ``st`` (see engine.state)."""
    _bf16_cuda(logits)
    _rows_ok(logits)
    B, V = logits.shape
    _req(st.temps.numel() >= B and st.next_ids.numel() >= B and st.out_tokens.shape[0] >= B,
         "sample: state smaller than batch")
    _eos_ok(st)
    _check(_fn("mrsum_sample")(_p(logits), logits.stride(0), B, V, _p(st.temps), _p(st.seeds), _p(st.positions),
                               _p(st.result), _p(st.next_ids), _p(st.positions), _p(st.gen_count), _p(st.max_new),
                               _p(st.out_tokens), st.out_tokens.stride(0), _p(st.done), _p(st.eos),
                               _stream()), "sample")


def sample_tp(logits: torch.Tensor, st, tok_offset: int, max_reduce) -> None:
    """Vocab-parallel sampling: Gumbel-max keys over this rank's logits shard (global token ids =
    tok_offset + column), ``max_reduce(keys)`` across the TP group (in place, unsigned), then the
    usual decode bookkeeping.  Same token as ``sample`` over the gathered row."""
    _bf16_cuda(logits)
    _rows_ok(logits)
    B, V = logits.shape
    _req(st.temps.numel() >= B and st.next_ids.numel() >= B and st.out_tokens.shape[0] >= B,
         "sample_tp: state smaller than batch")
    _eos_ok(st)
    _check(_fn("mrsum_sample_keys")(_p(logits), logits.stride(0), B, V, tok_offset, _p(st.temps), _p(st.seeds),
                                    _p(st.positions), _p(st.result), _stream()), "sample_keys")
    max_reduce(st.result[:B])
    _check(_fn("mrsum_sample_finish")(_p(st.result), _p(st.next_ids), _p(st.positions), _p(st.gen_count),
                                      _p(st.max_new), _p(st.out_tokens), st.out_tokens.stride(0), _p(st.done),
                                      _p(st.eos), B, _stream()), "sample_finish")


# ------------------------------------------------------------------ large-M GEMM (prefill, M > 64)
GEMM_GROUP_M = 4  # tile rows per raster group (4 x 8 tiles per XCD at a time; 8 measured equal)
GEMM_EPI_BF16, GEMM_EPI_SWIGLU = 0, 1
# group_m bit 8: 32x32-MFMA tiles.  Taken by the fp8 gate_up + SwiGLU GEMM only: +1.7..3.8 % at M = 4k-32k on
# the 70B shape on two boxes; the 70B fp8 qkv / o / down and every bf16 projection are equal or slower
# (profiles/r3_gemm_mfma32_experiment.jsonl, r3_gemm_mfma32_fp8_70b.jsonl)
GEMM_MFMA32 = 256


def _gemm(xp, ldx, wp, ldw, out, M, N, K, fp8, epi, sx, sw, group_m, split=0):
    _req(out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 8 == 0, "gemm: bad out layout")
    _check(_fn("mrsum_gemm")(xp, ldx, wp, ldw, _p(out), out.stride(0), M, N, K, fp8, epi, sx, sw,
                             GEMM_GROUP_M if group_m is None else group_m, split, _stream()), "gemm")
    return out


def gemm(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None, swiglu: bool = False,
         group_m: Optional[int] = None) -> torch.Tensor:
    """x [M, K] @ w [N, K]^T in bf16 on the 256 x 256-tile MFMA kernel (csrc/kernels/gemm.hip), any M.
    ``swiglu``: w is the [8 gate | 8 up]-interleaved gate_up weight and the result is silu(gate) * up
    [M, N / 2]."""
    _bf16_cuda(x, w)
    _rows_ok(x)
    _rows_ok(w)
    M, K = x.shape
    N = w.shape[0]
    _req(w.shape[1] == K and K % 64 == 0 and N % (32 if swiglu else 16) == 0,
         "gemm: unsupported shape M=%d N=%d K=%d" % (M, N, K))
    n_out = N // 2 if swiglu else N
    if out is None:
        out = torch.empty(M, n_out, dtype=torch.bfloat16, device=x.device)
    _bf16_cuda(out)
    _req(out.shape == (M, n_out), "gemm: bad out shape")
    if M == 0:
        return out
    return _gemm(_p(x), x.stride(0), _p(w), w.stride(0), out, M, N, K, 0,
                 GEMM_EPI_SWIGLU if swiglu else GEMM_EPI_BF16, None, None, group_m)


# One backend per op: every bf16 prefill product runs on gemm.hip.  The round-4 experiments that lived here
# (gemm4w.hip, a four-wave rebuild 20-25 % slower; the plain products on hipBLASLt, +0.25 % end to end) are
# recorded in profiles/r4_gemm4w_vs_8w_vs_hipblaslt.jsonl and r4_prefill_plain_gemm_blas_ab.jsonl and were
# removed from the library in round 5.


def gemm_fp8(xq: torch.Tensor, xs: torch.Tensor, w, out: Optional[torch.Tensor] = None, swiglu: bool = False,
             group_m: Optional[int] = None) -> torch.Tensor:
    """(xs[:, None] * xq) @ (w.scale[:, None] * w.q)^T on the fp8 MFMA path of the same kernel
    (v_mfma_scale_f32_16x16x128_f8f6f4, OCP e4m3fn operands; the SwiGLU form on the 32x32x64 tiles), bf16 out."""
    _req(xq.is_cuda and xq.dtype == torch.float8_e4m3fn and xq.dim() == 2 and xq.stride(1) == 1
         and xq.stride(0) % 16 == 0 and xq.data_ptr() % 16 == 0, "gemm_fp8: x must be e4m3fn rows, 16-B aligned")
    M, KX = xq.shape
    q, sc = w.q, w.scale
    N, K = q.shape
    split = KX == 2 * K  # two-term activations [hi | lo] (rmsnorm_fp8 split)
    _req(q.is_cuda and q.dtype == torch.float8_e4m3fn and q.is_contiguous() and (KX == K or split),
         "gemm_fp8: weight must be e4m3fn [N, K] contiguous, x [M, K] or two-term [M, 2K]")
    _req(xs.dtype == torch.float32 and xs.is_contiguous() and xs.numel() >= M and sc.dtype == torch.float32
         and sc.is_contiguous() and sc.numel() == N, "gemm_fp8: scales")
    _req(K % 128 == 0 and N % (32 if swiglu else 16) == 0, "gemm_fp8: unsupported shape M=%d N=%d K=%d" % (M, N, K))
    n_out = N // 2 if swiglu else N
    if out is None:
        out = torch.empty(M, n_out, dtype=torch.bfloat16, device=xq.device)
    _bf16_cuda(out)
    _req(out.shape == (M, n_out), "gemm_fp8: bad out shape")
    if M == 0:
        return out
    if group_m is None and swiglu:
        group_m = GEMM_GROUP_M | GEMM_MFMA32
    return _gemm(_p(xq), xq.stride(0), _p(q), K, out, M, N, K, 1, GEMM_EPI_SWIGLU if swiglu else GEMM_EPI_BF16,
                 _p(xs), _p(sc), group_m, 1 if split else 0)


# ------------------------------------------------------------------ decode GEMMs (M <= 64)
SKINNY_MAX_M = 64
# decode batches above 64 rows (e.g. the 92-chunk map of a 24 h transcript, bucket 96) run the stream GEMM
# over 64-row chunks -- the weights are streamed once per chunk, still far cheaper than the 256 x 256-tile
# GEMM, whose grid at M <= 256 is only N / 256 workgroups (16 for the 4096-wide o / down projections).
# gate_up (+ SwiGLU, 112 tiles) switches back to the tile GEMM above 128 rows.
STREAM_MAX_M = 256
STREAM_MAX_M_SWIGLU = 128
EPI_BF16, EPI_F32_PARTIAL, EPI_SWIGLU, EPI_SWIGLU_SPLIT, EPI_RESID_SPLIT = 0, 1, 2, 3, 4
EPI_SKINNY_RESID = 3  # skinny_gemm.hip's residual-update epilogue


def choose_splits(N: int, K: int, nt: int, target_wgs: int = 512, max_splits: int = 8) -> int:
    """Smallest split-K (dividing K/128) that gives >= target_wgs workgroups."""
    blocks = K // 128
    base = N // (16 * nt)
    for s in range(1, max_splits + 1):
        if blocks % s == 0 and base * s >= target_wgs:
            return s
    best = 1
    for s in range(1, max_splits + 1):
        if blocks % s == 0:
            best = s
    return best


# Register-streaming kernels (skinny_gemm.hip) run 8-wave workgroups for one decode row when the grid is at
# most SKINNY_WAVES8_MAX_WGS workgroups (about one per CU or less: a TP shard's N / 16 tiles), so twice the
# weight bytes are in flight per CU; larger grids already hold several 4-wave workgroups per CU.  In situ,
# whole decode steps (profiles/r5_skinny_waves_insitu.jsonl): Llama-3-8B TP=8 shard B=1 at 4k 1.374 -> 1.219
# ms, TP=1 B=1 at 13.5k 3.539 -> 3.522, 70B fp8 TP=8 shard B=1 at 32k 5.122 -> 5.105; at B=10 8 waves lose
# 0.3-1 % (TP=8 shard 1.449 vs 1.465, TP=1 4.527 vs 4.541), so more rows keep 4.
# ``SKINNY_WAVES_FORCE`` (4 / 8) overrides the choice for in-situ A/Bs (tools/exp_plans_insitu.py "waves:W");
# $MRSUM_SKINNY_WAVES sets it at import (multi-process rehearsals: the 4-wave summation order reproduces round
# 4's token streams bit for bit, git show 96648c3:tools/gpu_r5_q.sh).
SKINNY_WAVES8_MAX_WGS = 2 * 256
SKINNY_WAVES8_MAX_M = 1
SKINNY_WAVES_FORCE = int(os.environ["MRSUM_SKINNY_WAVES"]) if os.environ.get("MRSUM_SKINNY_WAVES") else None


def skinny_waves(N: int, nt: int, splits: int, M: int = 1) -> int:
    """Waves per workgroup (4 or 8) of a register-streaming launch of N / (16 nt) x splits workgroups over M
    rows."""
    if SKINNY_WAVES_FORCE in (4, 8):
        return SKINNY_WAVES_FORCE
    return 8 if M <= SKINNY_WAVES8_MAX_M and (N // (16 * nt)) * splits <= SKINNY_WAVES8_MAX_WGS else 4


def _skinny(x, w, out, epi, nt, splits, ldo, norm=None, resid=None, ssp=None, ar=None):
    """Register-streaming decode GEMM (skinny_gemm.hip).  ``norm``: deferred-RMSNorm input of the SwiGLU
    epilogue; EPI_SKINNY_RESID: residual += x @ w^T (TP push over ``ar`` when given), ``ssp`` [M, N / 16]."""
    _bf16_cuda(x, w)
    _rows_ok(x)
    M, K = x.shape
    N = w.shape[0]
    _req(w.is_contiguous() and w.shape[1] == K, "skinny_gemm: weight must be [N, K] contiguous")
    _req(1 <= M <= SKINNY_MAX_M and K % 128 == 0 and N % (16 * nt) == 0 and (K // 128) % splits == 0,
         "skinny_gemm: unsupported shape M=%d N=%d K=%d nt=%d S=%d" % (M, N, K, nt, splits))
    sq, tiles, eps = _norm_args(x, norm)
    rp, ldr, sp = None, 0, None
    if epi == EPI_SKINNY_RESID:
        _req(nt == 1 and splits == 1 and M <= 16, "skinny resid: one 16-row tile per workgroup, M <= 16")
        _bf16_cuda(resid)
        _rows_ok(resid)
        _req(resid.shape == (M, N) and ssp is not None and ssp.dtype == torch.float32 and ssp.is_contiguous()
             and ssp.shape == (M, N // 16), "skinny resid: residual [M, N] bf16 and ssp fp32 [M, N / 16]")
        rp, ldr, sp = _p(resid), resid.stride(0), _p(ssp)
    _check(_fn("mrsum_skinny_gemm")(_p(x), x.stride(0), _p(w), N, K, M, _p(out), ldo, epi, nt, splits, sq, tiles, eps,
                                    rp, ldr, sp, ar, skinny_waves(N, nt, splits, M), _stream()), "skinny_gemm")
    return out


def _skinny_lds(x, w, out, epi, splits, ldo, wpb=4):
    """Medium-M (x staged in LDS) variant; same contract as _skinny, 16*wpb-row tiles (wpb waves)."""
    _bf16_cuda(x, w)
    _rows_ok(x)
    M, K = x.shape
    N = w.shape[0]
    _req(w.is_contiguous() and w.shape[1] == K, "skinny_lds: weight must be [N, K] contiguous")
    _req(1 <= M <= SKINNY_MAX_M and K % 128 == 0 and 4 <= wpb <= 8 and N % (16 * wpb) == 0
         and (K // 128) % splits == 0, "skinny_lds: unsupported shape M=%d N=%d K=%d S=%d wpb=%d" % (M, N, K, splits, wpb))
    _check(_fn("mrsum_skinny_lds")(_p(x), x.stride(0), _p(w), N, K, M, _p(out), ldo, epi, splits, wpb, _stream()),
           "skinny_lds")
    return out


def _norm_args(x, norm):
    """(ssq ptr, tiles, eps) of a deferred-RMSNorm input (``norm`` = (ssq [M, tiles] fp32, eps)) or nulls."""
    if norm is None:
        return None, 0, 0.0
    ssq, eps = norm
    _req(ssq.is_cuda and ssq.dtype == torch.float32 and ssq.is_contiguous() and ssq.dim() == 2
         and ssq.shape[0] == x.shape[0] and ssq.shape[1] % 32 == 0, "deferred norm: ssq must be fp32 [M, 32k]")
    return _p(ssq), ssq.shape[1], float(eps)


def _resid_args(x, N, epi, resid, ssp):
    if epi != EPI_RESID_SPLIT:
        return None, 0, None
    M = x.shape[0]
    _bf16_cuda(resid)
    _rows_ok(resid)
    _req(resid.shape == (M, N) and ssp is not None and ssp.dtype == torch.float32 and ssp.is_contiguous()
         and ssp.dim() == 2 and ssp.shape[0] == M, "resid split: residual [M, N] bf16 and ssp fp32 [M, tiles]")
    return _p(resid), resid.stride(0), _p(ssp)


def _stream_gemm(x, w, out, epi, splits, ldo, wpb, parts=None, counters=None, norm=None, resid=None, ssp=None,
                 ar=None):
    """LDS-DMA weight-ring decode GEMM (csrc/kernels/stream_gemm.hip); same contract as _skinny_lds,
    one 16*wpb-row tile per workgroup, ~one workgroup per CU.  ``norm``: deferred-RMSNorm input
    (ssq, eps); EPI_RESID_SPLIT: residual += x @ w^T with per-tile row sums of squares into ``ssp``."""
    _bf16_cuda(x, w)
    _rows_ok(x)
    M, K = x.shape
    N = w.shape[0]
    if M > SKINNY_MAX_M and epi in (EPI_BF16, EPI_F32_PARTIAL, EPI_SWIGLU) and norm is None:
        # up to STREAM_TALL_M rows in one pass over the weights (96- / 128-row x tiles, a workgroup width that
        # keeps a 3-slot ring); above that, row chunks of that height: row slices of the bf16 output, or of
        # every fp32 slab (slab row stride = M)
        ch = STREAM_TALL_M  # the kernel's tallest x tile
        for r0 in range(0, M, ch):
            r1 = min(M, r0 + ch)
            if r1 - r0 > SKINNY_MAX_M:
                tw = tall_wpb(N, r1 - r0, splits)
                if tw is not None:
                    o = out[:, r0:r1] if epi == EPI_F32_PARTIAL else out[r0:r1]
                    _stream_launch(x[r0:r1], w, o, epi, splits, ldo, tw, None, None, None, None, None,
                                   M if epi == EPI_F32_PARTIAL else 0)
                    continue
            for c0 in range(r0, r1, SKINNY_MAX_M):
                c1 = min(r1, c0 + SKINNY_MAX_M)
                o = out[:, c0:c1] if epi == EPI_F32_PARTIAL else out[c0:c1]
                _stream_launch(x[c0:c1], w, o, epi, splits, ldo, wpb, None, None, None, None, None,
                               M if epi == EPI_F32_PARTIAL else 0)
        return out
    return _stream_launch(x, w, out, epi, splits, ldo, wpb, parts, counters, norm, resid, ssp, 0, ar)


# Decode batches of 65-128 rows run the stream GEMM on 96- / 128-row x tiles in ONE pass over the weights
# (stream_gemm.hip); before, each 64-row chunk re-streamed every weight byte (profiles/r4_stream_tall_tiles_24h_ab.jsonl).
STREAM_TALL_M = 128
# widths whose slot (16 wpb W rows + 16 MT x rows) x 256 B leaves a ring of >= 3 slots in the 157 KiB budget
# (mrsum_stream_gemm refuses the others): MT 6 -> wpb 4-6, MT 8 -> wpb 4-5
_TALL_WPB = {6: (4, 5, 6), 8: (4, 5)}


def tall_wpb(N: int, M: int, splits: int) -> Optional[int]:
    """Workgroup width (waves) of the tall-tile stream GEMM for M in (64, 128] rows: among the widths that
    keep a 3-slot LDS ring at that tile height, the one whose grid (N / (16 wpb) x splits) best fills whole
    rounds of one workgroup per CU; None if no width divides N."""
    mt = 6 if M <= 96 else 8
    best, key = None, None
    for wpb in _TALL_WPB[mt]:
        if N % (16 * wpb):
            continue
        grid = N // (16 * wpb) * splits
        k = (round(grid / (-(-grid // N_CU) * N_CU), 3), wpb)
        if key is None or k > key:
            best, key = wpb, k
    return best


def _stream_launch(x, w, out, epi, splits, ldo, wpb, parts, counters, norm, resid, ssp, slab_m, ar=None):
    M, K = x.shape
    N = w.shape[0]
    _req(w.is_contiguous() and w.shape[1] == K, "stream_gemm: weight must be [N, K] contiguous")
    tall_ok = M <= 128 and epi in (EPI_BF16, EPI_F32_PARTIAL, EPI_SWIGLU) and norm is None
    _req(1 <= M and (M <= SKINNY_MAX_M or tall_ok) and K % 128 == 0 and 4 <= wpb <= 8 and N % (16 * wpb) == 0
         and (K // 128) % splits == 0, "stream_gemm: unsupported shape M=%d N=%d K=%d S=%d wpb=%d"
         % (M, N, K, splits, wpb))
    if epi in (EPI_SWIGLU_SPLIT, EPI_RESID_SPLIT):
        _req(parts is not None and parts.shape == (splits, M, N) and parts.dtype == torch.float32
             and counters is not None and counters.numel() >= N // (16 * wpb), "stream_gemm: split-K scratch")
    if epi == EPI_RESID_SPLIT:
        _req(ssp.shape[1] == N // (16 * wpb), "stream_gemm: ssp tiles")
    sq, tiles, eps = _norm_args(x, norm)
    rp, ldr, sp = _resid_args(x, N, epi, resid, ssp)
    _check(_fn("mrsum_stream_gemm")(_p(x), x.stride(0), _p(w), N, K, M, _p(out), ldo, epi, splits, wpb, _p(parts),
                                    _p(counters), sq, tiles, eps, rp, ldr, sp, slab_m, ar, _stream()), "stream_gemm")
    return out


def linear_takes_norm(M: int, N: int, K: int) -> bool:
    """Whether ``linear`` of this shape runs on the stream kernel (the one that takes a deferred norm)."""
    return 1 <= M <= SKINNY_MAX_M and K % 128 == 0 and stream_config(N, K, splits=1) is not None


def linear(x: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None, norm=None) -> torch.Tensor:
    """x @ w^T, bf16 out: the 256 x 256-tile MFMA GEMM for M > 64 (or shapes the decode kernels do not
    take; up to 128 rows of a stream shape take the tall-tile stream GEMM), else the LDS-DMA weight-ring
    stream GEMM when it fills the chip (the LM head), else the
    register-streaming skinny kernel.  ``norm`` (stream shapes only, see linear_takes_norm): x holds
    un-normalised residual rows, scaled by their deferred RMSNorm factor in the epilogue."""
    M, K = x.shape
    N = w.shape[0]
    _req(norm is None or linear_takes_norm(M, N, K), "linear: a deferred norm needs a stream-GEMM shape")
    tall = (SKINNY_MAX_M < M <= STREAM_TALL_M and K % 128 == 0 and norm is None
            and stream_config(N, K, splits=1) is not None and tall_wpb(N, M, 1) is not None)
    if (M > SKINNY_MAX_M and not tall) or M == 0 or K % 128:
        return gemm(x, w, out=out)
    if out is None:
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    _req(out.is_contiguous() and out.shape == (M, N), "linear: bad out")
    if tall:  # a decode LM head of 65-128 rows: one pass over the weights on the tall-tile stream GEMM
        return _stream_gemm(x, w, out, EPI_BF16, 1, N, tall_wpb(N, M, 1))
    cfg = stream_config(N, K, splits=1)
    if cfg is not None:
        return _stream_gemm(x, w, out, EPI_BF16, 1, N, cfg[0], norm=norm)
    nt = 2 if N % 32 == 0 and N >= 16384 else 1
    if N % (16 * nt):
        return gemm(x, w, out=out)
    return _skinny(x, w, out, EPI_BF16, nt, 1, N)


def linear_parts(x: torch.Tensor, w: torch.Tensor, splits: Optional[int] = None,
                 out: Optional[torch.Tensor] = None, nt: int = 1, kernel: str = "skinny", norm=None) -> torch.Tensor:
    """fp32 split-K slabs [S, M, N] of x @ w^T (summed by add_rmsnorm_parts / rope_kv_parts).
    kernel "skinny" (waves split k, nt 16-row tiles), "lds" (x staged in LDS, 64-row tiles) or "stream"
    (LDS-DMA weight ring; nt = waves per workgroup, 16 * nt-row tiles)."""
    M, K = x.shape
    N = w.shape[0]
    if splits is None:
        splits = choose_splits(N, K, nt if kernel == "skinny" else 4)
    if out is None:
        out = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
    _req(out.is_contiguous() and out.shape == (splits, M, N) and out.dtype == torch.float32, "linear_parts: bad out")
    if kernel == "stream":
        return _stream_gemm(x, w, out, EPI_F32_PARTIAL, splits, N, nt, norm=norm)
    _req(norm is None, "linear_parts: a deferred norm needs the stream kernel")
    if kernel == "lds":
        return _skinny_lds(x, w, out, EPI_F32_PARTIAL, splits, N)
    return _skinny(x, w, out, EPI_F32_PARTIAL, nt, splits, N)


_TILE_COUNTERS = {}


def _tile_counters(device, n: int) -> torch.Tensor:
    """Per-device arrival tickets of the split-K SwiGLU GEMM (one per column tile, zero between
    launches: the last arriver of every tile re-arms its ticket).  One buffer serves every launch on
    the device's decode stream -- launches on one stream never overlap."""
    key = (str(device), n)
    t = _TILE_COUNTERS.get(key)
    if t is None:
        # must outlive any graph: never allocate inside a capture (the engine's eager warm-up step
        # before every capture allocates it)
        _req(not torch.cuda.is_current_stream_capturing(), "split-K SwiGLU tickets first used inside a capture")
        t = _TILE_COUNTERS[key] = torch.zeros(max(n, 1024), dtype=torch.int32, device=device)
    return t


def stream_swiglu_split(x: torch.Tensor, w_gu: torch.Tensor, out: torch.Tensor, wpb: int, splits: int,
                        norm=None) -> torch.Tensor:
    """SwiGLU of the gate_up GEMM split-K over ``splits`` workgroups per column tile; the last split
    of a tile to finish sums the fp32 partial tiles and applies silu(gate) * up (stream_gemm.hip)."""
    M, K = x.shape
    N = w_gu.shape[0]
    _req(out.is_contiguous() and out.shape == (M, N // 2), "stream_swiglu_split: bad out")
    parts = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
    cnt = _tile_counters(x.device, N // (16 * wpb))
    return _stream_gemm(x, w_gu, out, EPI_SWIGLU_SPLIT, splits, out.stride(0), wpb, parts=parts, counters=cnt,
                        norm=norm)


def stream_resid(x: torch.Tensor, w, residual: torch.Tensor, wpb: int, splits: int, tp=None) -> torch.Tensor:
    """Deferred-RMSNorm producer: residual += x @ w^T (bf16 or Fp8Weight ``w``), split-K over ``splits``
    workgroups per column tile, summed by the last to arrive; returns the fp32 [M, N / (16 wpb)] per-tile
    row sums of squares of the new residual (the consumers' ``norm`` input).  ``tp``: a custom all-reduce
    handle (parallel/custom_ar.py ``push_handle``): x @ w^T is this rank's share of a row-parallel
    projection and the last arriver all-reduces its tile over the TP group before the residual update
    (stream_gemm.hip "TP push") -- no separate all-reduce launch."""
    M = x.shape[0]
    fp8 = isinstance(w, Fp8Weight)
    N = (w.q if fp8 else w).shape[0]
    tiles = N // (16 * wpb)
    if tp is not None:
        STATS["tp_push"] += 1
    parts = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
    ssp = torch.empty(M, tiles, dtype=torch.float32, device=x.device)
    cnt = _tile_counters(x.device, tiles)
    if fp8:
        _stream_fp8(x, w, None, EPI_RESID_SPLIT, splits, 0, wpb, parts=parts, counters=cnt, resid=residual, ssp=ssp,
                    ar=tp)
    else:
        _stream_gemm(x, w, None, EPI_RESID_SPLIT, splits, 0, wpb, parts=parts, counters=cnt, resid=residual, ssp=ssp,
                     ar=tp)
    return ssp


_RESID_CAP = {}


def skinny_resid_capacity(N: Optional[int] = None) -> int:
    """Workgroups of the register-streaming residual producer resident at once on this device (a TP-push
    grid of N / 16 workgroups must fit: every one spins on its peers' copies of its tile) -- the smaller
    of the 4- and 8-wave forms (skinny_waves picks either by the row count).  ``N`` is accepted for the
    callers' readability; the bound does not depend on it."""
    for waves in (4, 8):
        if waves not in _RESID_CAP:
            _RESID_CAP[waves] = int(_fn("mrsum_skinny_resid_capacity_w")(waves))
    return min(_RESID_CAP[4], _RESID_CAP[8])


def skinny_resid(x: torch.Tensor, w, residual: torch.Tensor, tp=None) -> torch.Tensor:
    """Deferred-RMSNorm producer on the register-streaming kernel (one 16-row tile per workgroup, no
    split-K, M <= 16): residual += x @ w^T (bf16 or Fp8Weight ``w``) -- all-reduced over the custom
    all-reduce group ``tp`` first (TP push) when given; returns the fp32 [M, N / 16] per-tile row sums of
    squares of the new residual."""
    N = w.shape[0]
    fp8 = isinstance(w, Fp8Weight)
    M = x.shape[0]
    ssp = torch.empty(M, N // 16, dtype=torch.float32, device=x.device)
    if tp is not None:
        cap = skinny_fp8_resid_capacity() if fp8 else skinny_resid_capacity(N)
        _req(N // 16 <= cap, "skinny_resid: TP-push grid of %d workgroups is not fully resident (capacity %d)"
             % (N // 16, cap))
        STATS["tp_push"] += 1
    if fp8:
        _skinny_fp8(x, w, None, EPI_SKINNY_RESID, 1, 1, 0, resid=residual, ssp=ssp, ar=tp)
    else:
        _skinny(x, w, None, EPI_SKINNY_RESID, 1, 1, 0, resid=residual, ssp=ssp, ar=tp)
    return ssp


def skinny_fp8_resid_capacity() -> int:
    """skinny_resid_capacity of the fp8-weight residual producer."""
    if "fp8" not in _RESID_CAP:
        _RESID_CAP["fp8"] = int(_fn("mrsum_skinny_fp8_resid_capacity")())
    return _RESID_CAP["fp8"]


def linear_swiglu(x: torch.Tensor, w_gu: torch.Tensor, out: Optional[torch.Tensor] = None,
                  kernel: str = "skinny", wpb: int = 4, splits: int = 1, norm=None) -> torch.Tensor:
    """silu(gate) * up straight out of the gate_up GEMM (blocked [8 gate | 8 up] weight rows);
    ``norm``: deferred-RMSNorm input (stream kernels only)."""
    M = x.shape[0]
    F2 = w_gu.shape[0]
    _req(norm is None or kernel in ("stream", "stream_split", "skinny"),
         "linear_swiglu: a deferred norm needs the stream or register-streaming kernel")
    if kernel == "gemm" or M > (STREAM_MAX_M_SWIGLU if kernel == "stream" else SKINNY_MAX_M):
        return gemm(x, w_gu, out=out, swiglu=True)
    if out is None:
        out = torch.empty(M, F2 // 2, dtype=x.dtype, device=x.device)
    _req(out.is_contiguous() and out.shape == (M, F2 // 2), "linear_swiglu: bad out")
    if kernel == "stream":
        return _stream_gemm(x, w_gu, out, EPI_SWIGLU, 1, F2 // 2, wpb, norm=norm)
    if kernel == "stream_split":
        return stream_swiglu_split(x, w_gu, out, wpb, splits, norm=norm)
    if kernel == "lds":
        return _skinny_lds(x, w_gu, out, EPI_SWIGLU, 1, F2 // 2)
    return _skinny(x, w_gu, out, EPI_SWIGLU, 1, 1, F2 // 2, norm=norm)


def add_rmsnorm_parts(parts: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _req(parts.is_cuda and parts.dtype == torch.float32 and parts.is_contiguous() and parts.dim() == 3,
         "add_rmsnorm_parts: parts must be fp32 [S, T, D]")
    _bf16_cuda(residual, w)
    S, T, D = parts.shape
    _req(residual.shape == (T, D) and residual.is_contiguous() and w.numel() == D and D % 8 == 0,
         "add_rmsnorm_parts: shapes")
    if out is None:
        out = torch.empty(T, D, dtype=residual.dtype, device=residual.device)
    _rows_ok(out)
    _check(_fn("mrsum_add_rmsnorm_parts")(_p(parts), S, _p(residual), _p(w), _p(out), T, D, out.stride(0), eps,
                                          _stream()), "add_rmsnorm_parts")
    return out


# ------------------------------------------------------------------ per-role GEMM plans
# Measured on MI355X (tools/exp_lds_wpb.py, back-to-back launches, weights beyond the 256 MiB
# Infinity Cache, Llama-3-8B shapes, us per call; profiles/r1_decode_gemm_sweep.txt):
#   stream (LDS-DMA ring, one WG per CU)   M=1  qkv 10.7 | o 10.2 | gate_up+SwiGLU 44.3 | down 22.0
#                                          M=39 qkv 11.7 | o 10.2 | gate_up+SwiGLU 44.1 | down 23.2
#   register-streaming skinny / LDS-x      M=1  qkv 12.1 | o  9.9 | gate_up+SwiGLU 44.6 | down 24.2
#                                          M=39 qkv 15.8 | o 11.7 | gate_up+SwiGLU 60.7 | down 30.7
#   hipBLASLt                              M=39 qkv 19.9 | o 19.7 | gate_up 49.8 (+SwiGLU) | down 36.3
# The stream kernel is flat in M up to 64 and best on grids of exactly one workgroup per CU.
# Streaming floor (probe): qkv 9.5, o 7.6, down 20.1, gate_up 39.1.
# Plan = ("stream", wpb, S) | ("skinny", nt, S) | ("lds", S) | ("gemm",) (the 256 x 256-tile kernel)
N_CU = 256
STATS = {"tp_push": 0}  # host-side launch counts of selected paths (tests check which path ran)


def stream_config(N: int, K: int, swiglu: bool = False, splits: Optional[int] = None, max_splits: int = 16):
    """(wpb, S) for the stream GEMM whose grid N/(16 wpb) * S best fills one workgroup per CU, or None
    when no configuration fills >= 70 % of the CUs (then the register-streaming kernels win)."""
    if K % 128:
        return None
    nkb = K // 128
    best, best_key = None, None
    for wpb in (4, 5, 6, 7, 8):
        if N % (16 * wpb):
            continue
        tiles = N // (16 * wpb)
        cands = [1] if swiglu else ([splits] if splits else range(1, max_splits + 1))
        for S in cands:
            if nkb % S:
                continue
            grid = tiles * S
            eff = grid / (-(-grid // N_CU) * N_CU)
            # ties: wider tiles for grids of <= 2 rounds; narrower (finer-grained, better balanced rounds)
            # for long multi-round grids -- the LM head (128256 rows): wpb 4 vs 8 at M = 1 / 10 / 39
            # 179.8 / 179.6 / 202.3 vs 194.1 / 196.8 / 205.9 us (profiles/r2_lm_head_cfg_sweep.jsonl)
            key = (round(eff, 3), -S, wpb if grid <= 2 * N_CU else -wpb)
            if best_key is None or key > best_key:
                best, best_key = (wpb, S), key
    if best is None or best_key[0] < 0.7:
        return None
    return best


def tp_resid_config(N: int, K: int):
    """(wpb, S) of the TP-push residual producer (a row-parallel shard projection on the stream kernel)
    where the bare-GEMM plan picks the register-streaming kernel: the best-filling stream grid, with
    N / (16 wpb) a multiple of 32 (the consumers' deferred-norm tile count)."""
    best, best_key = None, None
    for wpb in (4, 8):
        if N % (16 * wpb) or (N // (16 * wpb)) % 32:
            continue
        tiles = N // (16 * wpb)
        for S in range(1, 17):
            if (K // 128) % S:
                continue
            grid = tiles * S
            eff = grid / (-(-grid // N_CU) * N_CU)
            key = (round(eff, 3), -S, wpb)
            if best_key is None or key > best_key:
                best, best_key = (wpb, S), key
    return best


def swiglu_split_config(N: int, K: int):
    """(wpb, S) of the split-K SwiGLU stream kernel that best fills the chip (a narrow gate_up shard taking
    a deferred norm), or None."""
    best, best_key = None, None
    for wpb in (4, 7, 8):
        if N % (16 * wpb):
            continue
        tiles = N // (16 * wpb)
        for S in (1, 2, 4, 8, 16):
            if (K // 128) % S or tiles * S > 2 * N_CU:
                continue
            grid = tiles * S
            key = (round(grid / (-(-grid // N_CU) * N_CU), 3), -S, wpb)
            if best_key is None or key > best_key:
                best, best_key = (wpb, S), key
    return best if best_key is not None and best_key[0] >= 0.7 else None


def plan(role: str, M: int, N: int, K: int, splits: Optional[int] = None, stream: bool = True):
    if M > (STREAM_MAX_M_SWIGLU if role == "gate_up" else STREAM_MAX_M) or K % 128:
        return ("gemm",)
    if role in ("o", "down") and M <= 16 and K <= 2048 and stream:
        # TP shard row-parallel projections (K = hidden / TP of the heads or the FFN): the register-
        # streaming kernel, no split-K beyond 2 -- in situ, TP=8 shard B=1 (profiles/
        # r3_plans_insitu_sc1.jsonl): down (K 1792) skinny S=2 1.394 ms vs stream (8, 7) 1.451; o (K 512)
        # skinny S=1 1.43 vs stream (4, 4) 1.451
        s = splits or (2 if (K // 128) % 2 == 0 and K >= 1024 else 1)
        return ("skinny", 1, s)
    cfg = stream_config(N, K, swiglu=(role == "gate_up"), splits=splits) if stream else None
    if cfg is not None:
        return ("stream",) + cfg
    if M > SKINNY_MAX_M:
        return ("gemm",)
    if role == "gate_up" and stream and (K // 128) % 4 == 0:
        # narrow gate_up (TP shards) that the one-tile-per-CU stream kernel cannot fill: split-K over the
        # column tiles, SwiGLU by the last split to arrive -- where it beats the register-streaming kernel
        # (tools/bench_tp_shard.py with write-through partials, us: TP=4 N=7168 M=10 15.7 vs 17.0, M=39
        # 21.2 vs 29.4 (M=1 14.9 vs 14.4: skinny); TP=8 N=3584 M=39 15.2 vs 15.8, M <= 10 12.2-12.8 vs
        # 10.3: skinny)
        if N >= 7168 and N % 112 == 0 and (M > 8 or N // 112 * 4 <= N_CU):
            # (a TP=4 shard's 7168 rows at one row too, where the 4-split grid is one round: in situ 8B TP=4
            # B=1 1.634 / 1.636 ms vs 1.669 / 1.662 on the register-streaming kernel; a TP=8 shard's 3584 rows
            # stay there, every split grid measured slower: profiles/r6_bf16_swiglu_split_insitu.jsonl)
            return ("stream_split", 7, 4)
        if N % 64 == 0 and M > 16:
            # (> 32 rows measured as above; 17..32 rows fell through to the 256 x 256 prefill GEMM: 81 us per
            # layer at a TP=8 shard, profiles/r3_tp8shard_b20_gaps.txt)
            return ("stream_split", 4, 4)
    blocks = K // 128

    def div(s):
        while blocks % s:
            s -= 1
        return s

    if role == "qkv":
        if M <= 8:
            return ("skinny", 1, splits or div(2))
        if M <= 16:
            return ("skinny", 2, splits or div(4)) if N % 32 == 0 else ("skinny", 1, splits or div(2))
        return ("lds", splits or div(8)) if N % 64 == 0 else ("gemm",)
    if role in ("o", "down"):
        if M <= 16:
            return ("skinny", 2, splits or div(2)) if N % 32 == 0 else ("skinny", 1, splits or div(4))
        if N % 64:
            return ("gemm",)
        return ("lds", splits or div(8))
    if role == "gate_up":
        if M <= 16:
            return ("skinny", 1, 1)
        return ("gemm",)
    return ("gemm",)




# ------------------------------------------------------------------ FP8 (e4m3fn) weights
def quant_fp8_rows(x: torch.Tensor):
    """Row-wise dynamic e4m3fn quantisation: returns (q [T, K] float8_e4m3fn, scale [T] fp32)."""
    _bf16_cuda(x)
    _rows_ok(x)
    T, K = x.shape
    _req(K % 8 == 0 and K <= 32768, "quant_fp8_rows: K")
    q = torch.empty(T, K, dtype=torch.float8_e4m3fn, device=x.device)
    sc = torch.empty(T, dtype=torch.float32, device=x.device)
    _check(_fn("mrsum_quant_fp8_rows")(_p(x), x.stride(0), _p(q), _p(sc), T, K, _stream()), "quant_fp8_rows")
    return q, sc


def skinny_fp8_takes_norm(M: int, K: int, splits: int = 1) -> bool:
    """Does the register-streaming fp8 kernel take a deferred-RMSNorm input (one row, x slice in LDS)?"""
    return M == 1 and K % 128 == 0 and (K // 128) % splits == 0 and (K // splits) * 2 <= 56 * 1024


def _skinny_fp8(x, w, out, epi, nt, splits, ldo, norm=None, resid=None, ssp=None, ar=None):
    _bf16_cuda(x)
    _rows_ok(x)
    M, K = x.shape
    N = w.q.shape[0]
    _req(w.q.is_cuda and w.q.dtype == torch.float8_e4m3fn and w.q.is_contiguous() and w.q.shape[1] == K,
         "skinny_fp8: weight must be e4m3fn [N, K] contiguous")
    _req(w.scale.dtype == torch.float32 and w.scale.numel() == N, "skinny_fp8: scale")
    _req(1 <= M <= SKINNY_MAX_M and K % 128 == 0 and N % (16 * nt) == 0 and (K // 128) % splits == 0,
         "skinny_fp8: unsupported shape M=%d N=%d K=%d nt=%d S=%d" % (M, N, K, nt, splits))
    _req(norm is None or skinny_fp8_takes_norm(M, K, splits), "skinny_fp8: a deferred norm needs M = 1")
    sq, tiles, eps = _norm_args(x, norm)
    rp, ldr, sp = None, 0, None
    if epi == EPI_SKINNY_RESID:
        _req(nt == 1 and splits == 1 and M <= 16 and norm is None, "skinny_fp8 resid: one 16-row tile, M <= 16")
        _bf16_cuda(resid)
        _rows_ok(resid)
        _req(resid.shape == (M, N) and ssp is not None and ssp.dtype == torch.float32 and ssp.is_contiguous()
             and ssp.shape == (M, N // 16), "skinny_fp8 resid: residual [M, N] bf16 and ssp fp32 [M, N / 16]")
        rp, ldr, sp = _p(resid), resid.stride(0), _p(ssp)
    _check(_fn("mrsum_skinny_fp8")(_p(x), x.stride(0), _p(w.q), _p(w.scale), N, K, M, _p(out), ldo, epi, nt, splits,
                                   sq, tiles, eps, rp, ldr, sp, ar, skinny_waves(N, nt, splits, M), _stream()),
           "skinny_fp8")
    return out


def stream_config_fp8(N: int, K: int, swiglu: bool = False, splits: Optional[int] = None, M: int = 1):
    """(wpb, S) for the fp8 stream GEMM (256-wide k slots), or None (register-streaming skinny_fp8).

    Measured (tools/bench_fp8_gemm.py, us, stream vs skinny): Llama-3-70B TP=1 at M=1 the skinny kernel
    wins (gate_up 103 vs 92, down 66 vs 51, qkv 24 vs 20) -- at M=16/40 the stream kernel does (gate_up
    110 / 138 vs 158 / 312, down 67 / 88 vs 66 / 161); TP=8 shards (< 64 M weights) the stream kernel at
    every M (o 12.9 vs 22.7, qkv 13.4 vs 18.1, down 13.7 vs 15.3 at M=1)."""
    if K % 256 or (M <= 8 and N * K >= (64 << 20)):
        return None
    cfg = stream_config(N, K // 2, swiglu=swiglu, splits=splits)  # K/256 slots == (K/2)/128 blocks
    if cfg is None and swiglu and splits is None and N >= 4096:
        cfg = fp8_swiglu_split_cfg(N, K)
    return cfg


def fp8_swiglu_split_cfg(N: int, K: int):
    """(wpb, S > 1) of the split-K SwiGLU on the fp8 stream kernel for a gate_up too narrow to fill the chip
    with one workgroup per column tile, or None.  The best-filling grid of 2 / 4 / 8 splits.  In situ,
    Llama-3-70B fp8 TP=8 shard (N 7168, K 8192; profiles/r6_fp8_swiglu_split_insitu.jsonl), ms per step vs
    the register-streaming kernel: B=1 at 32k 4.40 (wpb 7, S 4) / 4.37 (8, 4) vs 4.44, B=10 at 4k 4.75 /
    4.76 vs 5.55; two splits lose (4.53-4.58 at B=1)."""
    best, best_key = None, None
    for wpb in (8, 7, 6, 5, 4):
        if N % (16 * wpb):
            continue
        tiles = N // (16 * wpb)
        for S in (4, 8, 2):
            if (K // 256) % S or K // S < 1024:
                continue
            grid = tiles * S
            key = (round(grid / (-(-grid // N_CU) * N_CU), 3), S == 4, wpb)
            if best_key is None or key > best_key:
                best, best_key = (wpb, S), key
    return best if best_key is not None and best_key[0] >= 0.7 else None


def _stream_fp8(x, w, out, epi, splits, ldo, wpb, parts=None, counters=None, norm=None, resid=None, ssp=None,
                ar=None):
    """fp8 (e4m3fn, per-row scale) LDS-DMA weight-ring decode GEMM (stream_gemm.hip stream_fp8_kernel);
    the epilogues / deferred-RMSNorm operands of _stream_gemm."""
    _bf16_cuda(x)
    _rows_ok(x)
    M, K = x.shape
    N = w.q.shape[0]
    _req(w.q.is_cuda and w.q.dtype == torch.float8_e4m3fn and w.q.is_contiguous() and w.q.shape[1] == K,
         "stream_fp8: weight must be e4m3fn [N, K] contiguous")
    _req(w.scale.dtype == torch.float32 and w.scale.numel() == N and w.scale.is_contiguous(), "stream_fp8: scale")
    _req(1 <= M <= SKINNY_MAX_M and K % 256 == 0 and 4 <= wpb <= 8 and N % (16 * wpb) == 0
         and (K // 256) % splits == 0, "stream_fp8: unsupported shape M=%d N=%d K=%d S=%d "
         "wpb=%d" % (M, N, K, splits, wpb))
    if epi in (EPI_RESID_SPLIT, EPI_SWIGLU_SPLIT):
        _req(parts is not None and parts.shape == (splits, M, N) and parts.dtype == torch.float32
             and counters is not None and counters.numel() >= N // (16 * wpb)
             and (epi == EPI_SWIGLU_SPLIT or ssp.shape[1] == N // (16 * wpb)), "stream_fp8: split-K scratch")
    sq, tiles, eps = _norm_args(x, norm)
    rp, ldr, sp = _resid_args(x, N, epi, resid, ssp)
    _check(_fn("mrsum_stream_fp8")(_p(x), x.stride(0), _p(w.q), _p(w.scale), N, K, M, _p(out), ldo, epi, splits, wpb,
                                   _p(parts), _p(counters), sq, tiles, eps, rp, ldr, sp, ar, _stream()), "stream_fp8")
    return out


def fp8_stream_cfg(M: int, N: int, K: int, swiglu: bool = False, splits: Optional[int] = None):
    """(wpb, S) of the fp8 stream kernel for a decode shape, or None (register-streaming / fp8 GEMM)."""
    if not 1 <= M <= SKINNY_MAX_M:
        return None
    return stream_config_fp8(N, K, swiglu=swiglu, splits=splits, M=M)


def fp8_linear(x: torch.Tensor, w, swiglu: bool = False, norm=None) -> torch.Tensor:
    """x @ (scale * W8)^T for any M: MFMA W8A16 weight-streaming kernel at decode sizes; at prefill sizes
    row-wise e4m3fn activation quantisation + the fp8 MFMA GEMM (gemm.hip, per-row activation x
    per-row weight scales in the epilogue)."""
    M = x[0].shape[0] if isinstance(x, tuple) else x.shape[0]
    N = w.q.shape[0]
    _req(norm is None or (not swiglu and fp8_stream_cfg(M, N, x.shape[1], splits=1) is not None),
         "fp8_linear: a deferred norm needs the stream kernel")
    if isinstance(x, tuple):  # (q, scale): prefill rows quantised by their producer (rmsnorm_fp8)
        _req(norm is None and M > max(STREAM_MAX_M, STREAM_MAX_M_SWIGLU), "fp8_linear: pre-quantised rows are "
             "prefill rows")
        return gemm_fp8(x[0], x[1], w, swiglu=swiglu)
    if SKINNY_MAX_M < M <= (STREAM_MAX_M_SWIGLU if swiglu else STREAM_MAX_M) and norm is None:
        # decode batches of 65-256 rows: the weight-streaming kernels over 64-row chunks (the fp8 tile
        # GEMM's grid at M <= 256 is only N / 256 workgroups)
        out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=x.device)
        for r0 in range(0, M, SKINNY_MAX_M):
            r1 = min(M, r0 + SKINNY_MAX_M)
            out[r0:r1] = fp8_linear_swiglu(x[r0:r1], w) if swiglu else fp8_linear(x[r0:r1], w)
        return out
    if M <= SKINNY_MAX_M:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        cfg = stream_config_fp8(N, x.shape[1], splits=1, M=M)
        if cfg is not None:
            return _stream_fp8(x, w, out, EPI_BF16, 1, N, cfg[0], norm=norm)
        nt = 2 if N % 32 == 0 and N >= 16384 else 1
        return _skinny_fp8(x, w, out, EPI_BF16, nt, 1, N)
    xq, xs = quant_fp8_rows(x)
    return gemm_fp8(xq, xs, w, swiglu=swiglu)


def fp8_linear_parts(x: torch.Tensor, w, splits: int, nt: int = 1, stream_wpb: Optional[int] = None,
                     norm=None) -> torch.Tensor:
    """fp32 split-K slabs [splits, M, N] of x @ (scale * W8)^T: the fp8 stream GEMM when ``stream_wpb`` is
    given (its own split count), else the register-streaming kernel; ``norm``: deferred-RMSNorm input (the
    stream kernel at any M, the register-streaming one at M = 1)."""
    M, K = x.shape
    N = w.q.shape[0]
    out = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
    if stream_wpb is not None:
        return _stream_fp8(x, w, out, EPI_F32_PARTIAL, splits, N, stream_wpb, norm=norm)
    return _skinny_fp8(x, w, out, EPI_F32_PARTIAL, nt, splits, N, norm=norm)


def fp8_swiglu_takes_norm(M: int, F2: int, K: int) -> bool:
    """Does the decode gate_up + SwiGLU of this shape consume a deferred RMSNorm (no materialised rows)?"""
    return fp8_stream_cfg(M, F2, K, swiglu=True) is not None or skinny_fp8_takes_norm(M, K)


def fp8_linear_swiglu(x: torch.Tensor, w, norm=None) -> torch.Tensor:
    if isinstance(x, tuple):
        return fp8_linear(x, w, swiglu=True)
    M = x.shape[0]
    F2 = w.q.shape[0]
    cfg = fp8_stream_cfg(M, F2, x.shape[1], swiglu=True)
    _req(norm is None or fp8_swiglu_takes_norm(M, F2, x.shape[1]),
         "fp8_linear_swiglu: a deferred norm needs the stream kernel or one row")
    if M > SKINNY_MAX_M:
        return fp8_linear(x, w, swiglu=True)  # 64-row chunks up to STREAM_MAX_M_SWIGLU, else the fp8 GEMM
    out = torch.empty(M, F2 // 2, dtype=torch.bfloat16, device=x.device)
    if cfg is not None and cfg[1] > 1:
        # split-K over cfg[1] workgroups per column tile, silu(gate) * up by the last split to arrive (the
        # bf16 stream_swiglu_split of a narrow gate_up, e.g. a Llama-3-70B TP=8 shard's 7168 rows)
        parts = torch.empty(cfg[1], M, F2, dtype=torch.float32, device=x.device)
        cnt = _tile_counters(x.device, F2 // (16 * cfg[0]))
        return _stream_fp8(x, w, out, EPI_SWIGLU_SPLIT, cfg[1], F2 // 2, cfg[0], parts=parts, counters=cnt, norm=norm)
    if cfg is not None:
        return _stream_fp8(x, w, out, EPI_SWIGLU, 1, F2 // 2, cfg[0], norm=norm)
    return _skinny_fp8(x, w, out, EPI_SWIGLU, 1, 1, F2 // 2, norm=norm)


def fp8_resid_cfg(M: int, N: int, K: int):
    """(wpb, S) of the fp8 deferred-RMSNorm producer (stream kernel, split-K residual update), or None.
    Where the plan streams M <= 8 rows through the register-streaming kernel (large N K), one row still
    goes through the stream kernel with the x row resident in LDS: measured at Llama-3-70B o / down
    (profiles/r2_fp8_stream_xres_sweep.jsonl, us) wpb 8 S 4: o 16.7 vs 15.7 register-streaming, down 49.5
    vs 50.5 -- and it removes the separate add + RMSNorm launch (6.9 us) behind each of them."""
    cfg = fp8_stream_cfg(M, N, K)
    if cfg is not None or M != 1 or K % 256:
        return cfg
    for wpb in (8, 4):
        if N % (16 * wpb):
            continue
        tiles = N // (16 * wpb)
        for S in range(1, 17):
            if (K // 256) % S == 0 and tiles * S >= N_CU and K // S <= 8192 and (K // S) % 512 == 0:
                return (wpb, S)
    return None
