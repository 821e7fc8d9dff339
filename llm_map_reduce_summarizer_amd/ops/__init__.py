"""Engine ops: HIP/CDNA4 kernels on the GPU, PyTorch reference on the CPU.

There is exactly one implementation per device: tensors on a ROCm device go
to the hand-written gfx950 kernels in ``ops.hip`` (and fail loudly if
``libmrsum_kernels.so`` is missing -- no silent fallback), CPU tensors go to
``ops.reference`` (the numerics oracle, also what CPU-only tests run).
There is no switch that sends GPU tensors to the reference.

Every GPU op is a hand-written gfx950 kernel, GEMMs included: decode-shaped
projections on the weight-streaming MFMA kernels (stream_gemm.hip /
skinny_gemm.hip, fused split-K / SwiGLU / RoPE epilogues), everything with
more rows (prefill projections, the LM head over many rows) on the 256 x 256
MFMA GEMM (gemm.hip; bf16 or OCP fp8).  No vendor BLAS on the hot path.
"""

from __future__ import annotations

import torch

from . import reference
from .reference import Fp8Weight

def _use_hip(t) -> bool:
    return t.is_cuda


def _impl(t):
    if _use_hip(t):
        from . import hip
        return hip
    return reference


_UNIT = {}


def unit_gain(hidden, device):
    """A cached all-ones RMSNorm gain: the model folds its norm gains into the consumer projections
    (engine/model.py), so every norm the forward pass runs is unit-gain."""
    key = (hidden, str(device))
    t = _UNIT.get(key)
    if t is None:
        t = _UNIT[key] = torch.ones(hidden, dtype=torch.bfloat16, device=device)
    return t


def rmsnorm(x, w, eps, out=None, quant=False):
    """``w`` None: unit gain.  ``quant`` (the consumer is an fp8 GEMM): on the GPU at prefill sizes the
    rows come back quantised (QuantRows); ``quant="split"``: as two-term fp8 rows (ops.hip.rmsnorm_fp8)."""
    if w is None:
        w = unit_gain(x.shape[-1], x.device)
    if quant and out is None and _quant_ok(x):
        from . import hip
        return QuantRows(*hip.rmsnorm_fp8(x, w, eps, split=quant == "split"))
    return _impl(x).rmsnorm(x, w, eps, out)


class NormRows:
    """Deferred RMSNorm of decode rows (GPU): ``h`` = the residual rows (bf16 [M, hidden], not normalised)
    and ``ssq`` = fp32 [M, tiles] per-column-tile sums of squares of h written by the producing GEMM
    (ops.hip.stream_resid).  A consumer GEMM on the stream kernel takes h as its input and scales its
    product rows by rsqrt(mean(h^2) + eps) in the epilogue -- exact because the norm gains are folded
    into the consumer weights (engine/model.py).  ``materialize`` runs the unit-gain RMSNorm instead
    (consumers on other kernels).  Valid until the next producer updates the residual in place."""

    def __init__(self, h, ssq, eps):
        self.h, self.ssq, self.eps = h, ssq, eps

    @property
    def shape(self):
        return self.h.shape

    @property
    def norm(self):
        return (self.ssq, self.eps)

    def materialize(self):
        from . import hip
        return hip.rmsnorm(self.h, unit_gain(self.h.shape[1], self.h.device), self.eps)


class QuantRows:
    """Normalised prefill rows already quantised to row-wise e4m3fn by their producer (ops.hip.rmsnorm_fp8:
    the norm and the quantisation in one pass) for an fp8-weight GEMM: ``q`` [T, K] float8_e4m3fn (or
    two-term [T, 2K] = [hi | lo]), ``scale`` [T] fp32."""

    def __init__(self, q, scale):
        self.q, self.scale = q, scale

    @property
    def shape(self):
        return self.q.shape

    @property
    def pair(self):
        return (self.q, self.scale)


def rows(x):
    """Plain normalised rows of ``x`` (a tensor or a NormRows)."""
    if isinstance(x, QuantRows):
        raise TypeError("QuantRows feed fp8 GEMMs only")
    return x.materialize() if isinstance(x, NormRows) else x


def _quant_ok(x) -> bool:
    """Prefill rows that every fp8 consumer sends to the fp8 MFMA GEMM (above the stream kernels' rows)."""
    if not _use_hip(x):
        return False
    from . import hip
    return x.shape[0] > max(hip.STREAM_MAX_M, hip.STREAM_MAX_M_SWIGLU) and x.shape[1] % 16 == 0


def add_rmsnorm(x, residual, w, eps, out=None):
    """residual += x; returns rmsnorm(residual) * w (``w`` None: unit gain)."""
    if w is None:
        w = unit_gain(residual.shape[-1], residual.device)
    return _impl(x).add_rmsnorm(x, residual, w, eps, out)


def rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page, write_cache=True):
    return _impl(qkv).rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page,
                              write_cache)


def rope_kv_parts(parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page):
    """Sum split-K fp32 QKV slabs + RoPE + paged KV write; returns the bf16 qkv rows."""
    return _impl(parts).rope_kv_parts(parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d,
                                      page)


def kv_scatter(rows, page, slot, kcache, vcache):
    """Scatter all-gathered K/V rows [n, 2, hkv, d] into one layer's paged cache (see ops.hip.kv_scatter)."""
    return _impl(rows).kv_scatter(rows, page, slot, kcache, vcache)


def swiglu(gu, out=None):
    return _impl(gu).swiglu(gu, out)


def linear(x, w):
    """x @ w^T (bf16).  GPU: MFMA weight-streaming kernels for decode shapes, the 256 x 256 MFMA GEMM
    otherwise; ``w`` may be an Fp8Weight (W8A16 decode kernel / fp8 MFMA GEMM at prefill sizes).
    ``x`` may be a NormRows (the LM head after the last layer)."""
    if isinstance(x, NormRows):
        from . import hip
        M, K = x.shape
        if isinstance(w, Fp8Weight):
            if hip.fp8_stream_cfg(M, w.shape[0], K, splits=1) is not None:
                return hip.fp8_linear(x.h, w, norm=x.norm)
        elif hip.linear_takes_norm(M, w.shape[0], K):
            return hip.linear(x.h, w, norm=x.norm)
        x = x.materialize()
    if isinstance(w, Fp8Weight):
        if _use_hip(x):
            from . import hip
            return hip.fp8_linear(x, w)
        return reference.linear(x, w)
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


class PagedPrefill:
    """Chunked-prefill context of a packed batch of prompt slices: sequence i's slice starts at absolute
    position ``prefix[i]`` of the sequence in decode slot ``seq_slot[i]`` (block-table row); its keys
    are read from the paged cache (``kcache`` / ``vcache`` of one layer) -- see ops.hip.attn_prefill."""

    def __init__(self, block_tables, seq_slot, prefix, slot_host, prefix_host, kcache=None, vcache=None):
        self.block_tables, self.seq_slot, self.prefix = block_tables, seq_slot, prefix
        self.slot_host, self.prefix_host = list(slot_host), list(prefix_host)
        self.kcache, self.vcache = kcache, vcache

    def layer(self, kcache, vcache) -> "PagedPrefill":
        return PagedPrefill(self.block_tables, self.seq_slot, self.prefix, self.slot_host, self.prefix_host,
                            kcache, vcache)


def attn_prefill(qkv, cu_seqlens, hq, hkv, d, scale, out=None, paged=None, **kw):
    if _use_hip(qkv):
        from . import hip
        return hip.attn_prefill(qkv, cu_seqlens, hq, hkv, d, scale, out, paged=paged, **kw)
    if paged is not None:
        return reference.attn_prefill_paged(qkv, cu_seqlens, hq, hkv, d, scale, paged, out)
    return reference.attn_prefill(qkv, cu_seqlens, hq, hkv, d, scale, out)


def attn_decode(q, kcache, vcache, block_tables, positions, hq, hkv, d, page, scale, out=None, workspace=None):
    """``q``: bf16 rows [B, hq * d] (already rotated, K/V already in the cache) or a QKVParts."""
    if isinstance(q, QKVParts):
        from . import hip
        return hip.attn_decode_rope(q.parts, q.cos_sin, kcache, vcache, block_tables, positions, hq, hkv, d,
                                    page, scale, out, workspace=workspace)
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


def sample_tp(logits, st, tok_offset, max_reduce):
    """Vocab-parallel sampling over this rank's logits shard (GPU only; see hip.sample_tp)."""
    from . import hip
    return hip.sample_tp(logits, st, tok_offset, max_reduce)


# ---------------------------------------------------------------- fused projection blocks
# The model calls these; each picks (on the GPU) between our MFMA weight-streaming kernels
# with a fused epilogue (decode rows) and the 256 x 256 MFMA GEMM + a separate HIP kernel
# (prefill rows), per the measured plan table (ops.hip.plan).  On the CPU they are the
# reference composition.

def _plan_parts(hip, p, x, w, splits):
    if p[0] == "stream":
        if isinstance(x, NormRows):
            return hip.linear_parts(x.h, w, p[2], nt=p[1], kernel="stream", norm=x.norm)
        return hip.linear_parts(x, w, p[2], nt=p[1], kernel="stream")
    x = rows(x)
    if p[0] == "lds":
        return hip.linear_parts(x, w, splits or p[1], kernel="lds")
    return hip.linear_parts(x, w, splits or p[2], nt=p[1])


def _fp8_parts(hip, x, w, role, splits):
    """Split-K fp32 slabs from an fp8 weight-streaming kernel (decode): the LDS-DMA stream kernel when
    it fills the chip, else the register-streaming kernel with the bf16 plan shapes."""
    cfg = hip.stream_config_fp8(w.shape[0], w.shape[1], splits=splits, M=x.shape[0])
    if cfg is not None:
        if isinstance(x, NormRows):
            return hip.fp8_linear_parts(x.h, w, cfg[1], stream_wpb=cfg[0], norm=x.norm)
        return hip.fp8_linear_parts(x, w, cfg[1], stream_wpb=cfg[0])
    if x.shape[0] == 1 and splits is None:
        # one row: the x slice sits in LDS (skinny_fp8 XL), one 16-row tile per wave group and the
        # largest split-K that keeps >= 2048 k per workgroup and <= 4096 workgroups -- measured best at
        # Llama-3-70B shapes (profiles/r2_fp8_decode_x_in_lds_sweep.jsonl: qkv S=4, o S=4, down S=8;
        # TP=8 shards sit at the ~9 us launch floor whatever the split); a deferred norm is applied in
        # its epilogue
        N, K = w.shape
        s = next(s for s in (8, 4, 2, 1) if (K // 128) % s == 0 and (K // s >= 2048 or s == 1)
                 and N // 16 * s <= 4096)
        if isinstance(x, NormRows) and hip.skinny_fp8_takes_norm(1, K, s):
            return hip.fp8_linear_parts(x.h, w, s, 1, norm=x.norm)
        return hip.fp8_linear_parts(rows(x), w, s, 1)
    x = rows(x)
    p = hip.plan(role, x.shape[0], w.shape[0], w.shape[1], stream=False)
    nt = p[1] if p[0] == "skinny" else 1
    s = splits or (p[2] if p[0] == "skinny" else (p[1] if p[0] == "lds" else 1))
    if w.shape[0] % (16 * nt):
        nt = 1
    return hip.fp8_linear_parts(x, w, s, nt)


class QKVParts:
    """Deferred decode QKV: the QKV GEMM's fp32 split-K slabs [S, B, (hq + 2 hkv) d], not yet rotated nor
    written to the cache.  ``attn_decode`` consumes it with the fused RoPE + KV-write attention kernel
    (ops.hip.attn_decode_rope); ``materialize`` runs the separate rope_kv_parts pass instead."""

    def __init__(self, parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page):
        self.parts, self.positions, self.seq_idx, self.block_tables = parts, positions, seq_idx, block_tables
        self.kcache, self.vcache, self.cos_sin = kcache, vcache, cos_sin
        self.hq, self.hkv, self.d, self.page = hq, hkv, d, page

    def materialize(self):
        from . import hip
        return hip.rope_kv_parts(self.parts, self.positions, self.seq_idx, self.block_tables, self.kcache,
                                 self.vcache, self.cos_sin, self.hq, self.hkv, self.d, self.page)


def _defer_ok(hip, defer, x, hq, hkv, d, page):
    return defer and d == 128 and page == 64 and hq % hkv == 0 and hq // hkv <= 16


def qkv_rope(x, wqkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page, defer=False):
    """qkv = x @ wqkv^T, RoPE on Q/K, K/V into the paged cache; returns bf16 qkv rows -- or, with
    ``defer`` on the GPU decode path, a QKVParts for attn_decode's fused RoPE + KV write.  ``x`` may
    be a NormRows (deferred RMSNorm of the previous layer's down projection)."""
    if isinstance(x, QuantRows):
        from . import hip
        qkv = hip.fp8_linear(x.pair, wqkv)
        hip.rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page)
        return qkv
    xt = x.h if isinstance(x, NormRows) else x
    if _use_hip(xt) and isinstance(wqkv, Fp8Weight):
        from . import hip
        if x.shape[0] <= hip.SKINNY_MAX_M:
            parts = _fp8_parts(hip, x, wqkv, "qkv", None)
            if _defer_ok(hip, defer, x, hq, hkv, d, page):
                return QKVParts(parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page)
            return hip.rope_kv_parts(parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d,
                                     page)
        qkv = hip.fp8_linear(rows(x), wqkv)
        hip.rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page)
        return qkv
    if _use_hip(xt):
        from . import hip
        p = hip.plan("qkv", x.shape[0], wqkv.shape[0], wqkv.shape[1])
        if p[0] != "gemm":
            parts = _plan_parts(hip, p, x, wqkv, None)
            if _defer_ok(hip, defer, x, hq, hkv, d, page):
                return QKVParts(parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page)
            return hip.rope_kv_parts(parts, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv,
                                     d, page)
        qkv = hip.gemm(rows(x), wqkv)
        hip.rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page)
        return qkv
    qkv = reference.linear(x, wqkv)
    reference.rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page)
    return qkv


def _fused_ar(all_reduce, rows, hidden):
    """The fused all-reduce + add + RMSNorm of ``all_reduce`` (``all_reduce.add_rmsnorm(parts, residual,
    ln, eps)``, parallel/custom_ar.py) when it exists and takes ``rows`` x ``hidden``, else None."""
    f = getattr(all_reduce, "add_rmsnorm", None)
    if f is None or not all_reduce.fused_ok(rows, hidden):
        return None
    return f


# The deferred norm trades a separate add + RMSNorm launch for a split-K last-arriver tail in the
# producer: measured on one box (tools/ab_decode_old_new.sh, profiles/r2_deferred_norm_ab.jsonl) decode
# steps at B=1 -1.5 %, B=10 -0.5 %, B=39 +1 % -- so it runs up to 16 rows.
DEFER_NORM_MAX_M = 16
# Under TP the producer's tail replaces the all-reduce + add + RMSNorm launch (7.8 us at B=1, 14 us at B=20
# on a TP=8 shard: profiles/r3_tp8shard_b20_gaps.txt), so the TP push runs at every decode batch the
# stream kernel takes.
TP_PUSH_MAX_M = 64
# fp8 weights: the TP-push producer of a row-parallel shard projection runs on the fp8 register-streaming
# kernel (skinny_gemm.hip skinny_fp8_kernel EPI_RESID, no split-K tail) instead of the split-K stream kernel
# for K <= FP8_SKINNY_PUSH_MAX_K, and at one row for K <= FP8_SKINNY_PUSH_MAX_K_M1.  In situ, Llama-3-70B fp8
# TP=8 shard (profiles/r5_fp8_skinny_push_ab.jsonl): B=1 at 32k 4.77 ms -> o 4.64, down 4.62; B=10 at 4k
# 5.74 -> o 5.58, but down (K 3584) 5.87
FP8_SKINNY_PUSH_MAX_K = 1024
FP8_SKINNY_PUSH_MAX_K_M1 = 4096


RESID_FORCE = {}  # role -> "skinny" | "stream": measurement override of _resid_plan (tools only)


def _resid_plan(hip, a, w, role, tp=False, force=None):
    """The deferred-RMSNorm producer of this decode projection: ("stream", wpb, S) (stream kernel, split-K
    last-arriver residual update), ("skinny",) (register-streaming kernel, one tile per workgroup, no
    split-K) or None.  ``tp``: the TP-push producer of a row-parallel shard, which runs whatever the plan
    for its bare GEMM (the all-reduce launch it saves outweighs the kernel choice): on the register-
    streaming kernel where that is the plan (TP-shard o / down at K <= 2048), else the stream kernel.
    ``RESID_FORCE[role]`` ("skinny" / "stream") overrides the choice for in-situ measurements
    (tools/exp_plans_insitu.py sets it; nothing in the package does); ``force`` likewise, per call (the
    custom all-reduce's self-test of each producer kind, and the fallback when one kind failed it)."""
    M = a.shape[0]
    force = force or RESID_FORCE.get(role)
    if M > (TP_PUSH_MAX_M if tp else DEFER_NORM_MAX_M):
        return None
    N, K = w.shape
    if tp and M > 16:  # the register-streaming producer takes one 16-row tile
        if force == "skinny":
            return None
        cfg = (hip.fp8_resid_cfg(M, N, K) if isinstance(w, Fp8Weight) else
               (hip.plan(role, M, N, K)[1:] if hip.plan(role, M, N, K)[0] == "stream" else hip.tp_resid_config(N, K)))
        return None if cfg is None or (N // (16 * cfg[0])) % 32 else ("stream",) + tuple(cfg)
    if isinstance(w, Fp8Weight):
        if force == "skinny" or (force is None and tp and (K <= FP8_SKINNY_PUSH_MAX_K or
                                                           (M == 1 and K <= FP8_SKINNY_PUSH_MAX_K_M1))):
            # the fp8 register-streaming producer (one 16-row tile per workgroup, no split-K tail)
            ok = M <= 16 and N % 512 == 0 and N // 16 <= hip.skinny_fp8_resid_capacity()
            if ok or force == "skinny":
                return ("skinny",) if ok else None
        cfg = hip.fp8_resid_cfg(M, N, K)
    else:
        p = hip.plan(role, M, N, K)
        cfg = p[1:] if p[0] == "stream" else None
        if not tp and M <= 16 and N % 512 == 0 and (force == "skinny" or (force is None and role == "o" and K <= 4096)):
            # TP=1 o projection on the register-streaming producer (no split-K tail), in situ 4k context
            # (profiles/r3_tp1_resid_skinny_insitu.jsonl): B=1 3.336 vs 3.380 ms per step, B=10 4.078 vs 4.087;
            # down (K 14336) loses (3.50 / 4.32)
            return ("skinny",)
        if tp:
            if (force == "skinny" or (force is None and p[0] == "skinny")) and N % 512 == 0 \
                    and N // 16 <= hip.skinny_resid_capacity(N):  # every pushing workgroup resident at once
                return ("skinny",)
            if force == "skinny":
                return None
            if cfg is None or force == "stream":
                cfg = hip.tp_resid_config(N, K)
    if cfg is None or (N // (16 * cfg[0])) % 32:
        return None
    return ("stream",) + tuple(cfg)


def proj_add_rmsnorm(a, w, residual, ln, eps, role="o", all_reduce=None, quant=False):
    """residual += a @ w^T (TP-all-reduced when ``all_reduce``); returns rmsnorm(residual) * ln (``ln``
    None: unit gain, the model's folded-gain form).

    GPU decode rows with a unit gain: the projection itself updates the residual (split-K last-arriver
    epilogue) and the result is a NormRows -- the RMSNorm is deferred into the consumer GEMM, so no
    separate add + RMSNorm kernel runs; under TP (``all_reduce.push_ok``) that last arriver also
    all-reduces its tile over the group first (TP push), so no all-reduce kernel runs either.  ``all_reduce`` is a callable summing a tensor over
    the TP group in place; when it also offers ``add_rmsnorm``/``fused_ok`` (the model's P2P
    all-reduce) the decode path runs the projection's split-K slabs straight into one fused
    all-reduce + residual add + RMSNorm kernel."""
    if _use_hip(a):
        from . import hip
        if ln is None and a.shape[0] <= hip.SKINNY_MAX_M:
            # TP: the producer all-reduces its own tiles (TP push) when the group's buffers take the rows
            ok = getattr(all_reduce, "push_ok", None)
            push = all_reduce.push_handle() if ok is not None and ok(a.shape[0], residual.shape[1]) else None
            if all_reduce is None or push is not None:
                rp = _resid_plan(hip, a, w, role, tp=push is not None)
                kinds = getattr(all_reduce, "push_kinds", None)
                if push is not None and rp is not None and kinds is not None and rp[0] not in kinds():
                    # that producer failed the start-up self-test: the other kind if it takes the shape
                    # and passed, else the fused all-reduce path below
                    other = ({"stream", "skinny"} - {rp[0]}) & kinds()
                    # (_resid_plan's forced "skinny" checks the capacity of the kernel the weight runs on:
                    # skinny_fp8_resid_capacity for an Fp8Weight, skinny_resid_capacity for bf16)
                    rp = _resid_plan(hip, a, w, role, tp=True, force=other.pop()) if other else None
                if rp is not None and rp[0] == "skinny":
                    return NormRows(residual, hip.skinny_resid(a, w, residual, tp=push), eps)
                if rp is not None:
                    return NormRows(residual, hip.stream_resid(a, w, residual, rp[1], rp[2], tp=push), eps)
    if ln is None:
        ln = unit_gain(residual.shape[1], residual.device)
    if _use_hip(a) and isinstance(w, Fp8Weight):
        from . import hip
        if a.shape[0] <= hip.SKINNY_MAX_M:
            fused = _fused_ar(all_reduce, a.shape[0], residual.shape[1])
            parts = _fp8_parts(hip, a, w, role, 1 if (all_reduce and not fused) else None)
            if fused:
                return fused(parts, residual, ln, eps)
            if all_reduce:
                all_reduce(parts)
            return hip.add_rmsnorm_parts(parts, residual, ln, eps)
        o = hip.fp8_linear(a, w)
        if all_reduce:
            all_reduce(o)
        if quant and _quant_ok(o):
            return QuantRows(*hip.rmsnorm_fp8(o, ln, eps, residual=residual, split=quant == "split"))
        return hip.add_rmsnorm(o, residual, ln, eps)
    if _use_hip(a):
        from . import hip
        fused = _fused_ar(all_reduce, a.shape[0], residual.shape[1])
        one = 1 if (all_reduce and not fused) else None  # a plain all-reduce takes one slab
        p = hip.plan(role, a.shape[0], w.shape[0], w.shape[1], splits=one)
        if p[0] != "gemm":
            parts = _plan_parts(hip, p, a, w, one)
            if fused:
                return fused(parts, residual, ln, eps)
            if all_reduce:
                all_reduce(parts)
            return hip.add_rmsnorm_parts(parts, residual, ln, eps)
        o = hip.gemm(a, w)
        if all_reduce:
            all_reduce(o)
        if quant and _quant_ok(o):
            return QuantRows(*hip.rmsnorm_fp8(o, ln, eps, residual=residual, split=quant == "split"))
        return hip.add_rmsnorm(o, residual, ln, eps)
    o = reference.linear(a, w)
    if all_reduce:
        all_reduce(o)
    return reference.add_rmsnorm(o, residual, ln, eps)


def mlp(x, wgu, wdown, residual, eps, all_reduce=None, quant=False):
    """The decode/prefill MLP block: residual += swiglu(x wgu^T) wdown^T (TP-all-reduced when
    ``all_reduce``); returns the next layer's normed input as proj_add_rmsnorm does: gate_up_swiglu then
    proj_add_rmsnorm.  (A one-launch fused MLP of a TP shard was built in round 4, bit-exact and 1-5 %
    slower per TP=8 shard step -- profiles/r4_mlp_fused_tp8_shard_ab.jsonl, docs/decode_latency.md -- and
    removed from the library in round 5.)"""
    act = gate_up_swiglu(x, wgu)
    return proj_add_rmsnorm(act, wdown, residual, None, eps, "down", all_reduce, quant=quant)


def gate_up_swiglu(x, wgu):
    """silu(gate) * up of the fused, [8 gate | 8 up]-blocked gate_up projection; ``x`` may be a
    NormRows (deferred RMSNorm) or QuantRows (fp8 prefill rows quantised by the norm)."""
    if isinstance(x, QuantRows):
        from . import hip
        return hip.fp8_linear_swiglu(x.pair, wgu)
    xt = x.h if isinstance(x, NormRows) else x
    if _use_hip(xt) and isinstance(wgu, Fp8Weight):
        from . import hip
        if isinstance(x, NormRows) and hip.fp8_swiglu_takes_norm(x.shape[0], wgu.shape[0], x.shape[1]):
            return hip.fp8_linear_swiglu(x.h, wgu, norm=x.norm)
        return hip.fp8_linear_swiglu(rows(x), wgu)
    if _use_hip(xt):
        from . import hip
        p = hip.plan("gate_up", x.shape[0], wgu.shape[0], wgu.shape[1])
        nr = isinstance(x, NormRows) and p[0] in ("stream", "stream_split", "skinny")
        xin, norm = (x.h, x.norm) if nr else (rows(x), None)
        if p[0] == "stream":
            return hip.linear_swiglu(xin, wgu, kernel="stream", wpb=p[1], norm=norm)
        if p[0] == "stream_split":
            return hip.linear_swiglu(xin, wgu, kernel="stream_split", wpb=p[1], splits=p[2], norm=norm)
        return hip.linear_swiglu(xin, wgu, kernel=p[0], norm=norm)
    return reference.swiglu(reference.linear(x, wgu))
