"""Engine ops: HIP/CDNA4 kernels on the GPU, PyTorch reference on the CPU.

There is exactly one implementation per device: tensors on a ROCm device go
to the hand-written gfx950 kernels in ``ops.hip`` (and fail loudly if
``libmrsum_kernels.so`` is missing -- no silent fallback), CPU tensors go to
``ops.reference`` (the numerics oracle, also what CPU-only tests run).
``MRSUM_OPS=torch`` forces the reference on the GPU for debugging only.

Plain dense GEMMs (projections, LM head) are ``torch.matmul`` -> hipBLASLt;
every fused / non-GEMM hot op (norms, RoPE + KV write, SwiGLU, embedding,
flash prefill attention, paged decode attention, sampling) is ours.
"""

from __future__ import annotations

import os

from . import reference

_FORCE_TORCH = os.environ.get("MRSUM_OPS", "").lower() == "torch"


def _use_hip(t) -> bool:
    return t.is_cuda and not _FORCE_TORCH


def _impl(t):
    if _use_hip(t):
        from . import hip
        return hip
    return reference


def rmsnorm(x, w, eps, out=None):
    return _impl(x).rmsnorm(x, w, eps, out)


def add_rmsnorm(x, residual, w, eps, out=None):
    return _impl(x).add_rmsnorm(x, residual, w, eps, out)


def rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page, write_cache=True):
    return _impl(qkv).rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page,
                              write_cache)


def rope_kv_parts(parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page):
    """Sum split-K fp32 QKV slabs + RoPE + paged KV write; returns the bf16 qkv rows."""
    return _impl(parts).rope_kv_parts(parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d,
                                      page)


def swiglu(gu, out=None):
    return _impl(gu).swiglu(gu, out)


def linear(x, w):
    """x @ w^T (bf16).  GPU: MFMA weight-streaming kernel for decode shapes, hipBLASLt otherwise."""
    return _impl(x).linear(x, w)


def linear_parts(x, w, splits=None):
    """fp32 split-K partial slabs [S, M, N] of x @ w^T, consumed by add_rmsnorm_parts."""
    if _use_hip(x):
        from . import hip
        return hip.linear_parts(x, w, splits)
    return reference.linear_parts(x, w, splits or 1)


def linear_swiglu(x, w_gu):
    return _impl(x).linear_swiglu(x, w_gu)


def add_rmsnorm_parts(parts, residual, w, eps, out=None):
    return _impl(residual).add_rmsnorm_parts(parts, residual, w, eps, out)


def embed(ids, table, out=None):
    return _impl(table).embed(ids, table, out)


def attn_prefill(qkv, cu_seqlens, hq, hkv, d, scale, out=None, **kw):
    if _use_hip(qkv):
        from . import hip
        return hip.attn_prefill(qkv, cu_seqlens, hq, hkv, d, scale, out, **kw)
    return reference.attn_prefill(qkv, cu_seqlens, hq, hkv, d, scale, out)


def attn_decode(q, kcache, vcache, block_tables, positions, hq, hkv, d, page, scale, out=None, workspace=None):
    if _use_hip(q):
        from . import hip
        return hip.attn_decode(q, kcache, vcache, block_tables, positions, hq, hkv, d, page, scale, out,
                               workspace=workspace)
    return reference.attn_decode(q, kcache, vcache, block_tables, positions, hq, hkv, d, page, scale, out)


def sample(logits, st):
    if _use_hip(logits):
        from . import hip
        return hip.sample(logits, st)
    n = logits.shape[0]
    toks = reference.sample_tokens(logits, st.temps[:n], st.seeds[:n], st.positions[:n])
    reference.sample_finish(toks, st)
