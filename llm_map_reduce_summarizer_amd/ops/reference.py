"""Plain-PyTorch reference implementations of every engine op.

These are (1) the numerics oracle the HIP kernels are tested against
(fp32 math, same data layouts, same masking rules) and (2) the compute path
on CPU-only hosts, where the tiny test models run.  On a GPU the engine uses
``ops.hip`` exclusively (see ``ops/__init__.py``).

Layouts shared with the kernels (``csrc/kernels/*.hip``):

* ``qkv`` [T, (Hq + 2 Hkv) * D]: Q heads, then K heads, then V heads.
* KV cache per layer: ``kcache``/``vcache`` [num_pages, Hkv, P, D];
  token at position ``p`` of a sequence lives in page
  ``block_tables[row, p // P]`` at offset ``p % P``.
* ``cos_sin`` [max_pos, D/2, 2] fp32 (cos, sin), HF rotate-half pairing.
* fp8 KV cache (``--kv-dtype fp8``: K and V; ``fp8v``: V only, K stays bf16; csrc/kernels/kv8.h): per layer uint8 [num_pages, Hkv, SLAB],
  SLAB = P * D + 4 * P -- a (page, head) slab holds P rows of D e4m3fn bytes, then P fp32 row scales;
  a row is quantised whole with the power-of-two scale >= max|x| / 448.
"""

from __future__ import annotations

import math
from typing import Optional

import torch

LOG2E = 1.4426950408889634


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    y = y.to(x.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    residual.copy_((x.float() + residual.float()).to(residual.dtype))
    return rmsnorm(residual, w, eps, out)


def rope_inv_freq(head_dim: int, theta: float, scaling=None) -> torch.Tensor:
    """RoPE inverse frequencies (float64); ``scaling`` = (factor, low_freq_factor, high_freq_factor,
    original_max_position) applies Llama-3.1's "llama3" rule: wavelengths longer than
    orig / low_freq_factor are divided by ``factor``, shorter than orig / high_freq_factor kept, and the
    band between interpolated smoothly."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling is None:
        return inv
    factor, low, high, orig = scaling
    wavelen = 2 * math.pi / inv
    low_wl, high_wl = orig / low, orig / high
    smooth = ((orig / wavelen) - low) / (high - low)
    mid = (1 - smooth) * inv / factor + smooth * inv
    out = torch.where(wavelen > low_wl, inv / factor, inv)
    band = (wavelen <= low_wl) & (wavelen >= high_wl)
    return torch.where(band, mid, out)


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None, scaling=None) -> torch.Tensor:
    inv = rope_inv_freq(head_dim, theta, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return torch.stack([ang.cos(), ang.sin()], dim=-1).float().contiguous().to(device)


def kv8_slab(page: int, d: int) -> int:
    return page * d + 4 * page


def kv8_quant_rows(x: torch.Tensor):
    """Rows [..., d] -> (e4m3fn bytes [..., d] uint8, fp32 scales [...]): scale = the power of two >= max|x| / 448
    (1 for a zero row) and at least 2^-126 (a normal number: 1 / scale stays finite), q = RNE e4m3(x / scale) --
    kv8.h's row rule."""
    xf = x.float()
    amax = xf.abs().amax(-1)
    m, e = torch.frexp(amax / 448.0)
    e = torch.clamp(torch.where(m == 0.5, e - 1, e), min=-126)
    sc = torch.where(amax > 0, torch.ldexp(torch.ones_like(amax), e), torch.ones_like(amax))
    q = (xf / sc[..., None]).to(torch.float8_e4m3fn).view(torch.uint8)
    return q, sc


def kv8_from_bf16(cache: torch.Tensor) -> torch.Tensor:
    """A bf16 cache [pages, Hkv, P, d] in the fp8 slab layout [pages, Hkv, P * d + 4 P] (every row quantised)."""
    n, hkv, page, d = cache.shape
    q, sc = kv8_quant_rows(cache)
    return torch.cat([q.reshape(n, hkv, page * d), sc.contiguous().view(torch.uint8).reshape(n, hkv, 4 * page)], -1)


def cache_pages(cache: torch.Tensor, pages: torch.Tensor, page: int, d: int) -> torch.Tensor:
    """fp32 [len(pages), Hkv, P, d] of a bf16 or fp8-slab cache."""
    c = cache.index_select(0, pages)
    if cache.dtype != torch.uint8:
        return c.float()
    q = c[..., : page * d].reshape(*c.shape[:2], page, d).contiguous().view(torch.float8_e4m3fn).float()
    sc = c[..., page * d:].contiguous().view(torch.float32)
    return q * sc[..., None]


def cache_write(cache: torch.Tensor, pages: torch.Tensor, offs: torch.Tensor, rows: torch.Tensor, page: int,
                d: int) -> None:
    """cache[pages[i], :, offs[i]] = rows[i] ([n, Hkv, d]) for a bf16 or fp8-slab cache."""
    if cache.dtype != torch.uint8:
        cache[pages, :, offs] = rows.to(cache.dtype)
        return
    q, sc = kv8_quant_rows(rows)  # [n, Hkv, d] bytes, [n, Hkv]
    n, hkv = rows.shape[0], rows.shape[1]
    col = offs[:, None] * d + torch.arange(d, device=offs.device)[None, :]  # [n, d] byte columns
    for h in range(hkv):
        cache[pages[:, None], h, col] = q[:, h]
        sb = page * d + 4 * offs[:, None] + torch.arange(4, device=offs.device)[None, :]
        cache[pages[:, None], h, sb] = sc[:, h].contiguous().view(torch.uint8).view(n, 4)


def rope_kv(qkv: torch.Tensor, positions: torch.Tensor, seq_idx: torch.Tensor, block_tables: torch.Tensor,
            kcache: Optional[torch.Tensor], vcache: Optional[torch.Tensor], cos_sin: torch.Tensor,
            hq: int, hkv: int, d: int, page: int, write_cache: bool = True) -> None:
    T = qkv.shape[0]
    if T == 0:
        return
    half = d // 2
    pos = positions[:T].long()
    cs = cos_sin[pos]  # [T, half, 2]
    cos, sin = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    qk = qkv[:, : (hq + hkv) * d].view(T, hq + hkv, d).float()
    a, b = qk[..., :half], qk[..., half:]
    ra = a * cos - b * sin
    rb = b * cos + a * sin
    rot = torch.cat([ra, rb], dim=-1).to(qkv.dtype)
    qkv[:, : (hq + hkv) * d] = rot.reshape(T, -1)
    if write_cache:
        rows = seq_idx[:T].long()
        keep = rows >= 0  # seq_idx < 0: prefill padding token, never cached
        rows, p_, k = rows[keep], pos[keep], rot[:, hq:][keep]
        pages = block_tables[rows, p_ // page].long()
        offs = p_ % page
        v = qkv[:, (hq + hkv) * d: (hq + 2 * hkv) * d].view(T, hkv, d)[keep]
        cache_write(kcache, pages, offs, k, page, d)
        cache_write(vcache, pages, offs, v, page, d)


def rope_kv_parts(parts: torch.Tensor, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    qkv = parts.float().sum(0).to(torch.bfloat16)
    rope_kv(qkv, positions, seq_idx, block_tables, kcache, vcache, cos_sin, hq, hkv, d, page)
    if out is not None:
        out.copy_(qkv)
        return out
    return qkv


def kv_scatter(rows: torch.Tensor, page: torch.Tensor, slot: torch.Tensor, kcache: torch.Tensor,
               vcache: torch.Tensor) -> None:
    """Reference of ops.hip.kv_scatter: cache[page[i], :, slot[i], :] = rows[i, 0 | 1] (page < 0 skipped)."""
    if kcache.dtype == torch.uint8 or vcache.dtype == torch.uint8:
        raise ValueError("kv_scatter: the context-parallel K/V exchange takes bf16 caches only")
    keep = page[: rows.shape[0]].long() >= 0
    pg, sl, r = page[: rows.shape[0]].long()[keep], slot[: rows.shape[0]].long()[keep], rows[keep]
    kcache[pg, :, sl, :] = r[:, 0].to(kcache.dtype)
    vcache[pg, :, sl, :] = r[:, 1].to(vcache.dtype)


def interleave_gate_up(wg: torch.Tensor, wu: torch.Tensor) -> torch.Tensor:
    """[F, H] gate + [F, H] up -> [2F, H] rows in blocks of 16 = [8 gate | 8 up]."""
    f, h = wg.shape
    return torch.stack([wg.reshape(f // 8, 8, h), wu.reshape(f // 8, 8, h)], dim=1).reshape(2 * f, h)


def split_gate_up(gu: torch.Tensor):
    """Inverse of the blocked column layout of a gate_up GEMM output."""
    f = gu.shape[-1] // 2
    v = gu.reshape(*gu.shape[:-1], f // 8, 2, 8)
    return v[..., 0, :].reshape(*gu.shape[:-1], f), v[..., 1, :].reshape(*gu.shape[:-1], f)


def swiglu(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    g, u = split_gate_up(gu)
    g, u = g.float(), u.float()
    y = (g * torch.sigmoid(g) * u).to(gu.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


class Fp8Weight:
    """OCP e4m3fn weight [N, K] with one fp32 scale per output row (W = scale[:, None] * float(q))."""

    def __init__(self, q: torch.Tensor, scale: torch.Tensor):
        self.q, self.scale = q, scale

    @property
    def shape(self):
        return self.q.shape

    def numel(self) -> int:
        return self.q.numel()

    def nbytes(self) -> int:
        return self.q.numel() + 4 * self.scale.numel()

    def dequant(self, dtype=torch.float32) -> torch.Tensor:
        return (self.q.float() * self.scale.float()[:, None]).to(dtype)

    @staticmethod
    def quantize(w: torch.Tensor) -> "Fp8Weight":
        wf = w.float()
        scale = wf.abs().amax(dim=1).clamp_min(1e-12) / 448.0
        q = (wf / scale[:, None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
        return Fp8Weight(q.contiguous(), scale.contiguous())


def _w(w):
    return w.dequant(torch.bfloat16) if isinstance(w, Fp8Weight) else w


def linear(x: torch.Tensor, w) -> torch.Tensor:
    if isinstance(w, Fp8Weight):
        return (x.float() @ w.dequant().t()).to(x.dtype)
    return torch.nn.functional.linear(x, w)


def linear_parts(x: torch.Tensor, w: torch.Tensor, splits: int = 1) -> torch.Tensor:
    """fp32 split-K partial slabs [S, M, N] of x @ w^T (what skinny_gemm EPI_F32_PARTIAL emits)."""
    K = x.shape[1]
    ks = K // splits
    wf = w.dequant() if isinstance(w, Fp8Weight) else w.float()
    return torch.stack([x[:, i * ks:(i + 1) * ks].float() @ wf[:, i * ks:(i + 1) * ks].t()
                        for i in range(splits)])


def linear_swiglu(x: torch.Tensor, w_gu) -> torch.Tensor:
    return swiglu(linear(x, w_gu))


def add_rmsnorm_parts(parts: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    residual.copy_((parts.float().sum(0) + residual.float()).to(residual.dtype))
    return rmsnorm(residual, w, eps, out)


def embed(ids: torch.Tensor, table: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    y = table[ids.long().clamp(0, table.shape[0] - 1)]
    if out is not None:
        out.copy_(y)
        return out
    return y


def attn_prefill(qkv: torch.Tensor, cu_seqlens: torch.Tensor, hq: int, hkv: int, d: int, scale: float,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    T = qkv.shape[0]
    if out is None:
        out = torch.empty(T, hq * d, dtype=qkv.dtype, device=qkv.device)
    cu = cu_seqlens.tolist()
    g = hq // hkv
    for i in range(len(cu) - 1):
        s, e = cu[i], cu[i + 1]
        if e <= s:
            continue
        n = e - s
        q = qkv[s:e, : hq * d].view(n, hq, d).float().transpose(0, 1)
        k = qkv[s:e, hq * d: (hq + hkv) * d].view(n, hkv, d).float().transpose(0, 1)
        v = qkv[s:e, (hq + hkv) * d: (hq + 2 * hkv) * d].view(n, hkv, d).float().transpose(0, 1)
        k = k.repeat_interleave(g, dim=0)
        v = v.repeat_interleave(g, dim=0)
        sc = torch.matmul(q, k.transpose(1, 2)) * scale
        mask = torch.ones(n, n, dtype=torch.bool, device=qkv.device).triu(1)
        sc.masked_fill_(mask, float("-inf"))
        p = torch.softmax(sc, dim=-1)
        o = torch.matmul(p, v).transpose(0, 1).reshape(n, hq * d)
        out[s:e] = o.to(out.dtype)
    return out


def attn_prefill_paged(qkv: torch.Tensor, cu_seqlens: torch.Tensor, hq: int, hkv: int, d: int, scale: float,
                       paged, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Chunked prefill: slice rows of every packed sequence attend to the cached positions
    [0, prefix) of that sequence (paged cache, already holding this slice's K/V too) and causally
    within the slice."""
    T = qkv.shape[0]
    if out is None:
        out = torch.empty(T, hq * d, dtype=qkv.dtype, device=qkv.device)
    cu = cu_seqlens.tolist()
    g = hq // hkv
    P = 64 if paged.kcache.dtype == torch.uint8 else paged.kcache.shape[2]
    for i in range(len(cu) - 1):
        s, e = cu[i], cu[i + 1]
        if e <= s:
            continue
        n, pre, slot = e - s, paged.prefix_host[i], paged.slot_host[i]
        tot = pre + n
        pages = paged.block_tables[slot, : -(-tot // P)].long()
        k = cache_pages(paged.kcache, pages, P, d).permute(1, 0, 2, 3).reshape(hkv, -1, d)[:, :tot]
        v = cache_pages(paged.vcache, pages, P, d).permute(1, 0, 2, 3).reshape(hkv, -1, d)[:, :tot]
        q = qkv[s:e, : hq * d].view(n, hq, d).float().transpose(0, 1)
        k = k.repeat_interleave(g, dim=0)
        v = v.repeat_interleave(g, dim=0)
        sc = torch.matmul(q, k.transpose(1, 2)) * scale
        qpos = torch.arange(pre, tot, device=qkv.device)[:, None]
        kpos = torch.arange(tot, device=qkv.device)[None, :]
        sc.masked_fill_(kpos > qpos, float("-inf"))
        p = torch.softmax(sc, dim=-1)
        out[s:e] = torch.matmul(p, v).transpose(0, 1).reshape(n, hq * d).to(out.dtype)
    return out


def attn_decode(q: torch.Tensor, kcache: torch.Tensor, vcache: torch.Tensor, block_tables: torch.Tensor,
                positions: torch.Tensor, hq: int, hkv: int, d: int, page: int, scale: float,
                out: Optional[torch.Tensor] = None, num_splits: int = 1) -> torch.Tensor:
    """q: [B, >= hq*d] (rows of the qkv buffer); context = positions + 1."""
    B = q.shape[0]
    if out is None:
        out = torch.empty(B, hq * d, dtype=q.dtype, device=q.device)
    g = hq // hkv
    for b in range(B):
        ctx = int(positions[b]) + 1
        npg = (ctx + page - 1) // page
        pages = block_tables[b, :npg].long()
        k = cache_pages(kcache, pages, page, d).permute(1, 0, 2, 3).reshape(hkv, npg * page, d)[:, :ctx]
        v = cache_pages(vcache, pages, page, d).permute(1, 0, 2, 3).reshape(hkv, npg * page, d)[:, :ctx]
        qq = q[b, : hq * d].view(hkv, g, d).float()
        sc = torch.matmul(qq, k.transpose(1, 2)) * scale
        p = torch.softmax(sc, dim=-1)
        o = torch.matmul(p, v).reshape(hq * d)
        out[b] = o.to(out.dtype)
    return out


# ----------------------------------------------------------------- sampler
_M1 = 0xbf58476d1ce4e5b9
_M2 = 0x94d049bb133111eb
_GOLD = 0x9E3779B97F4A7C15
_TOKMUL = 0xD1B54A32D192ED03
_U64 = (1 << 64) - 1


def _s64(x: int) -> int:
    x &= _U64
    return x - (1 << 64) if x >= (1 << 63) else x


def _lsr(x: torch.Tensor, n: int) -> torch.Tensor:
    return (x >> n) & ((1 << (64 - n)) - 1)


def _mix64_t(x: torch.Tensor) -> torch.Tensor:
    x = x ^ _lsr(x, 30)
    x = x * _s64(_M1)
    x = x ^ _lsr(x, 27)
    x = x * _s64(_M2)
    x = x ^ _lsr(x, 31)
    return x


def gumbel_noise(seed: int, position: int, vocab: int, device=None) -> torch.Tensor:
    """The sampler kernel's counter-based Gumbel noise for one row (fp32)."""
    k0 = _mix64_t(torch.tensor([_s64(seed * _GOLD + position + 1)], dtype=torch.int64))
    tok = torch.arange(vocab, dtype=torch.int64)
    h = _mix64_t(k0 ^ (tok * _s64(_TOKMUL)))
    u = (_lsr(h, 40).double() + 0.5) / 16777216.0
    return (-torch.log(-torch.log(u))).float().to(device)


def sample_tokens(logits: torch.Tensor, temps: torch.Tensor, seeds: torch.Tensor,
                  positions: torch.Tensor) -> torch.Tensor:
    """Gumbel-max sampling (argmax when temperature <= 0); ties -> lowest id."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32)
    for b in range(B):
        row = logits[b].float().cpu()
        t = float(temps[b])
        if t > 0:
            row = row / t + gumbel_noise(int(seeds[b]), int(positions[b]), V)
        out[b] = int(torch.argmax(row))
    return out.to(logits.device)


def sample_finish(tokens: torch.Tensor, st) -> None:
    """Bookkeeping identical to the finish kernel (st = engine DecodeState)."""
    B = tokens.shape[0]
    eos = set(int(x) for x in st.eos.tolist() if int(x) >= 0)
    for b in range(B):
        if int(st.done[b]):
            continue
        tok = int(tokens[b])
        g = int(st.gen_count[b])
        st.out_tokens[b, g] = tok
        st.gen_count[b] = g + 1
        st.next_ids[b] = tok
        if g + 1 >= int(st.max_new[b]) or tok in eos:
            st.done[b] = 1
        else:
            st.positions[b] += 1


def attention_scale(d: int) -> float:
    return 1.0 / math.sqrt(d)
