"""Llama-3 forward pass for the on-node engine (prefill and decode).

Weights are random-init and seeded per tensor (the benchmark setting: no
checkpoints offline), generated full-size and then sliced for tensor
parallelism so a model is bit-identical for every TP degree.  Fused layouts:

* ``wqkv`` [(Hq + 2 Hkv) * hd / tp, hidden]: this rank's Q heads, K heads, V heads
* ``wo``   [hidden, Hq * hd / tp]           (row-parallel, all-reduced)
* ``wgu``  [2 * ffn / tp, hidden]            (gate/up shards interleaved in blocks of
                                             8 rows, one GEMM; see ops.reference.swiglu)
* ``wdown``[hidden, ffn / tp]                (row-parallel, all-reduced)
* ``lm_head`` [vocab / tp, hidden]           (vocab-parallel, logits all-gathered)

One residual block (both phases)::

    qkv = x @ wqkv^T                 HIP MFMA GEMM (stream / skinny decode kernels, 256^2 prefill)
    rope_kv(qkv -> Q,K rotated; K,V -> paged cache)     HIP
    a   = attention(qkv)             HIP: flash prefill | paged split-K decode
    o   = a @ wo^T  (+ TP all-reduce over RCCL)
    x   = add_rmsnorm(o, residual)   HIP (residual += o, fused)
    gu  = x @ wgu^T ; act = swiglu(gu) (HIP) ; dn = act @ wdown^T (+ all-reduce)
    x   = add_rmsnorm(dn, residual)  HIP

RMSNorm gains are folded into the projection that consumes the normalised rows (``wqkv`` <- ln1,
``wgu`` <- ln2, ``lm_head`` <- the final norm: W' = W diag(g), at load time, before any fp8
quantisation), so every norm in the forward pass is unit-gain -- which lets decode defer the norm
into the consumer GEMM's epilogue (ops.NormRows): on one GPU the o / down projections update the
residual themselves and no separate add + RMSNorm kernel runs.  ``ln1`` / ``ln2`` / ``final_norm``
keep the checkpoint's gains for export (engine/weights.save_hf un-folds them).
"""

from __future__ import annotations

import hashlib
import math
import os
from dataclasses import dataclass
from typing import Callable, List, Optional

import torch

from .. import ops
from ..ops.reference import Fp8Weight, interleave_gate_up, rope_cos_sin
from ..parallel.dist import AsyncWorks
from .config import ModelConfig


def _seed_for(seed: int, name: str) -> int:
    return int.from_bytes(hashlib.sha1(("%d:%s" % (seed, name)).encode()).digest()[:8], "little") & ((1 << 63) - 1)


def _randn(shape, std: float, seed: int, name: str, device, dtype) -> torch.Tensor:
    g = torch.Generator(device=device)
    g.manual_seed(_seed_for(seed, name))
    t = torch.randn(*shape, generator=g, device=device, dtype=torch.float32 if device.type == "cpu" else dtype)
    t.mul_(std)
    return t.to(dtype)


class _TPReduce:
    """The all-reduce handed to ops.proj_add_rmsnorm: RCCL / one-shot P2P sum (``__call__``) plus, on
    GPUs with the P2P buffers, the fused all-reduce + residual add + RMSNorm kernel for decode rows."""

    def __init__(self, model: "LlamaModel"):
        self.model = model
        ar = model.custom_ar
        self.fused = ar is not None and os.environ.get("MRSUM_FUSED_AR", "1") == "1"

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return self.model._all_reduce(t)

    def fused_ok(self, rows: int, hidden: int) -> bool:
        ar = self.model.custom_ar
        return self.fused and ar is not None and ar.paths["fused_norm"] and rows <= ar.MAX_ROWS and \
            hidden % 4 == 0 and hidden <= 8192 and rows * hidden * 2 <= ar.max_bytes

    def add_rmsnorm(self, parts, residual, ln, eps):
        return self.model.custom_ar.add_rmsnorm(parts, residual, ln, eps)

    def push_ok(self, rows: int, hidden: int) -> bool:
        """TP push (ops.proj_add_rmsnorm): the row-parallel GEMM all-reduces its own tiles."""
        ar = self.model.custom_ar
        return ar is not None and _tp_push_enabled() and ar.push_ok(rows, hidden)

    def push_handle(self) -> int:
        return self.model.custom_ar.push_handle()

    def push_kinds(self) -> set:
        """TP-push producers that passed the custom all-reduce's start-up self-test."""
        return self.model.custom_ar.push_kinds()


def _page_of(kcache: torch.Tensor, head_dim: int) -> int:
    """Page size (tokens) of a whole-model cache: bf16 [L, pages, hkv, P, D] or the fp8 byte slabs
    [L, pages, hkv, P * D + 4 P] (engine/kv_cache.py)."""
    if kcache.dtype == torch.uint8:
        return kcache.shape[3] // (head_dim + 4)
    return kcache.shape[3]


# fp8 prefill: the QKV projection's input as two-term fp8 ([hi | lo], ops.hip.rmsnorm_fp8 split) -- the
# attention scores computed from q / k amplify e4m3's 2-3 % row rounding into ~24 % relative logit error on
# the parity checkpoint; two-term QKV input brings it to ~10 % for ~1.1x the QKV GEMM's cost (the o / gate_up /
# down inputs stay single-term)  (CPU emulation: profiles/r4_fp8_activation_emulation.txt)
_QKV_SPLIT = os.environ.get("MRSUM_FP8_QKV_SPLIT", "1") == "1"


def _hip():
    from ..ops import hip
    return hip


def _tp_push_enabled() -> bool:
    return os.environ.get("MRSUM_TP_PUSH", "1") == "1"


class LocalReduce:
    """Single-GPU stand-in for _TPReduce when measuring ONE rank's TP shard of the decode step
    (tools/bench_decode.py --tp-shard K): the sum over ranks is the identity and the fused all-reduce +
    residual add + RMSNorm kernel and the TP push run over a group of one (parallel/custom_ar.py
    LocalPush) -- the same kernels per layer as a real TP rank (the deferred norm of TP=1 is off), minus
    the cross-GPU hop."""
    fused = True

    def __init__(self, model: "LlamaModel"):
        self.model = model

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def fused_ok(self, rows: int, hidden: int) -> bool:
        return rows <= 64

    def add_rmsnorm(self, parts, residual, ln, eps):
        lp = self.model.local_push()
        if lp.fits_rows(parts):
            return lp.add_rmsnorm(parts, residual, ln, eps)
        return ops.add_rmsnorm_parts(parts, residual, ln, eps)

    def push_ok(self, rows: int, hidden: int) -> bool:
        return _tp_push_enabled() and self.model.local_push().push_ok(rows, hidden)

    def push_handle(self) -> int:
        return self.model.local_push().push_handle()


@dataclass
class LayerWeights:
    ln1: torch.Tensor
    wqkv: torch.Tensor
    wo: torch.Tensor
    ln2: torch.Tensor
    wgu: torch.Tensor
    wdown: torch.Tensor


class LlamaModel:
    def __init__(self, cfg: ModelConfig, device: torch.device, dtype: torch.dtype = torch.bfloat16, seed: int = 0,
                 tp_rank: int = 0, tp_size: int = 1, tp_group=None, weight_dtype: str = "bf16",
                 weights_path: Optional[str] = None):
        """``weights_path``: a Hugging Face Llama safetensors checkpoint (file or directory) loaded by
        engine.weights.load_hf instead of the seeded random init.

        ``weight_dtype="fp8"``: the four projection matrices of every layer are stored as OCP e4m3fn
        with per-output-row fp32 scales (ops.Fp8Weight) -- W8A16 MFMA kernels at decode sizes, the
        fp8 MFMA GEMM (dynamic per-token activation scales) at prefill sizes; the LM head likewise.
        Embedding and norms stay bf16."""
        if weight_dtype not in ("bf16", "fp8"):
            raise ValueError("weight_dtype must be bf16 or fp8")
        self.weight_dtype = weight_dtype
        if cfg.n_heads % tp_size or cfg.n_kv_heads % tp_size or cfg.ffn % tp_size or cfg.vocab_size % tp_size:
            raise ValueError("%s does not shard over tp=%d" % (cfg.name, tp_size))
        self.cfg, self.device, self.dtype = cfg, torch.device(device), dtype
        self.tp_rank, self.tp_size, self.tp_group = tp_rank, tp_size, tp_group
        self.hq, self.hkv, self.hd = cfg.n_heads // tp_size, cfg.n_kv_heads // tp_size, cfg.head_dim
        self.ffn_local = cfg.ffn // tp_size
        self.vocab_local = cfg.vocab_size // tp_size
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        if weights_path:
            from .weights import load_hf
            self.layers = [LayerWeights(None, None, None, None, None, None) for _ in range(cfg.n_layers)]
            load_hf(self, weights_path)
        else:
            self._init_weights(seed)
        self.cos_sin = rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta, self.device,
                                    scaling=cfg.rope_scaling)
        self.vocab_offset = tp_rank * self.vocab_local
        self.emulate_tp_reduce = False  # LocalReduce in place of the TP all-reduce (shard measurements)
        self._local_push = None
        # TP prefill with sequence parallelism (prefill_passes; MRSUM_SP=0: all-reduces)
        self.sequence_parallel = os.environ.get("MRSUM_SP", "1") == "1"
        # TP on GPUs: decode all-reduces (fp32 split-K slabs, <= 1 MiB) and the sampler's key max go
        # through the one-shot P2P kernel (parallel/custom_ar.py); larger messages through RCCL
        self.custom_ar = None
        if tp_size > 1 and self.device.type == "cuda" and os.environ.get("MRSUM_CUSTOM_AR", "1") == "1":
            from ..parallel.custom_ar import maybe_custom_all_reduce
            # self-tested at THIS model's decode shapes: hidden size, the shard K of the row-parallel
            # projections (o: the local heads, down: the local ffn), the weight format, decode rows 1-64
            self.custom_ar = maybe_custom_all_reduce(tp_group, shapes=dict(
                hidden=cfg.hidden, k={"o": self.hq * self.hd, "down": self.ffn_local},
                fp8=weight_dtype == "fp8", rows=(1, 16, 64)))

    # ------------------------------------------------------------------ weights
    def _init_weights(self, seed: int) -> None:
        c, dev, dt = self.cfg, self.device, self.dtype
        std = c.init_std
        r, tp, hd = self.tp_rank, self.tp_size, c.head_dim
        ones = lambda: torch.ones(c.hidden, device=dev, dtype=dt)  # noqa: E731
        self.embed = _randn((c.vocab_size, c.hidden), std, seed, "embed", dev, dt)
        self.layers: List[LayerWeights] = []
        for i in range(c.n_layers):
            wq = _randn((c.n_heads * hd, c.hidden), std, seed, "l%d.wq" % i, dev, dt)
            wk = _randn((c.n_kv_heads * hd, c.hidden), std, seed, "l%d.wk" % i, dev, dt)
            wv = _randn((c.n_kv_heads * hd, c.hidden), std, seed, "l%d.wv" % i, dev, dt)
            qs, ks = self.hq * hd, self.hkv * hd
            wqkv = torch.cat([wq[r * qs:(r + 1) * qs], wk[r * ks:(r + 1) * ks], wv[r * ks:(r + 1) * ks]]).contiguous()
            del wq, wk, wv
            wo = _randn((c.hidden, c.n_heads * hd), std, seed, "l%d.wo" % i, dev, dt)
            wo = wo[:, r * qs:(r + 1) * qs].contiguous()
            f = self.ffn_local
            wg = _randn((c.ffn, c.hidden), std, seed, "l%d.wg" % i, dev, dt)
            wu = _randn((c.ffn, c.hidden), std, seed, "l%d.wu" % i, dev, dt)
            wgu = interleave_gate_up(wg[r * f:(r + 1) * f], wu[r * f:(r + 1) * f]).contiguous()
            del wg, wu
            wd = _randn((c.hidden, c.ffn), std, seed, "l%d.wd" % i, dev, dt)
            wd = wd[:, r * f:(r + 1) * f].contiguous()
            if self.weight_dtype == "fp8":
                wqkv, wo, wgu, wd = (Fp8Weight.quantize(t) for t in (wqkv, wo, wgu, wd))
            self.layers.append(LayerWeights(ones(), wqkv, wo, ones(), wgu, wd))
        self.final_norm = ones()  # unit gains: nothing to fold into the consumers
        lm = _randn((c.vocab_size, c.hidden), std, seed, "lm_head", dev, dt)
        v = self.vocab_local
        self.lm_head = lm[r * v:(r + 1) * v].contiguous()
        del lm
        self._quantize_lm_head()

    def _quantize_lm_head(self) -> None:
        """fp8 models: the LM head is an fp8 weight too (per-row scales, W8A16 at decode).  In bf16 it was
        2.1 GB of the 70B model's 81 GB read per token at 32k -- 409 us of a 15.7 ms step
        (docs/decode_latency.md); the embedding stays bf16 (a row gather)."""
        if self.weight_dtype == "fp8" and not isinstance(self.lm_head, Fp8Weight):
            self.lm_head = Fp8Weight.quantize(self.lm_head)

    def weight_bytes(self) -> int:
        def nb(t):
            return t.nbytes() if isinstance(t, Fp8Weight) else t.numel() * t.element_size()
        n = nb(self.embed) + nb(self.lm_head) + nb(self.final_norm)
        for lw in self.layers:
            n += sum(nb(t) for t in (lw.ln1, lw.wqkv, lw.wo, lw.ln2, lw.wgu, lw.wdown))
        return n

    # ------------------------------------------------------------------ comm
    def local_push(self):
        """The one-rank TP-push handle of a TP-shard measurement (created on first use: outside a capture,
        the engine's eager step before every capture gets here first)."""
        if self._local_push is None:
            from ..parallel.custom_ar import LocalPush
            self._local_push = LocalPush()
        return self._local_push

    def _all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp_size > 1:
            if self.custom_ar is not None and self.custom_ar.fits(t):
                self.custom_ar.all_reduce(t)
            else:
                if t.is_cuda and torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("TP all-reduce of %s does not fit the P2P buffers inside a hipGraph "
                                       "capture (lower the decode batch or raise max_bytes)" % (tuple(t.shape),))
                torch.distributed.all_reduce(t, group=self.tp_group)
        return t

    def _all_reduce_async(self, t: torch.Tensor):
        """Start the TP sum of ``t``; returns a handle whose ``wait()`` orders later work on the current stream
        after it (RCCL runs on its own stream, so compute issued before the wait overlaps it), or None when
        the sum already happened (the P2P kernel for small messages, runs in stream order)."""
        if self.tp_size == 1:
            return None
        if self.custom_ar is not None and self.custom_ar.fits(t):
            self.custom_ar.all_reduce(t)
            return None
        return torch.distributed.all_reduce(t, group=self.tp_group, async_op=True)

    # ---- sequence parallelism (Megatron SP) of the TP prefill: the residual stream is split over the TP
    # ranks by token rows; a projection's partial sums are REDUCE-SCATTERED to the row shards (instead of
    # all-reduced), add + RMSNorm run on 1 / TP of the rows, and the normed rows are ALL-GATHERED for the
    # next column-parallel GEMM -- the same bytes on the links as the all-reduce, 1 / TP of the norm work
    # and residual memory.  Rows are padded to a multiple of TP.
    def _sp_backend_ok(self) -> bool:
        """Sequence parallelism runs on every backend: RCCL natively, gloo on CPU tensors, and gloo over GPU
        tensors (ranks sharing one GPU: rehearsals, the TP parity test) through host-staged collectives
        (_sp_host)."""
        return True

    def _sp_host(self) -> bool:
        """Device tensors over a non-RCCL group (gloo): stage the SP collectives through host memory."""
        return self.device.type == "cuda" and torch.distributed.get_backend(self.tp_group) != "nccl"

    def _sp_rows(self, T: int):
        Tp = -(-T // self.tp_size) * self.tp_size
        return Tp, Tp // self.tp_size

    def _sp_shard(self, t: torch.Tensor) -> torch.Tensor:
        """This rank's row shard of a replicated [T, H] tensor (padded rows are zero)."""
        T = t.shape[0]
        Tp, Ts = self._sp_rows(T)
        out = torch.zeros(Ts, t.shape[1], dtype=t.dtype, device=t.device)
        lo = self.tp_rank * Ts
        n = max(0, min(T, lo + Ts) - lo)
        if n:
            out[:n] = t[lo:lo + n]
        return out

    def _sp_reduce_scatter_async(self, t: torch.Tensor):
        """Start the TP sum of partial rows ``t`` [T, H], scattered by row shards: (shard, handle)."""
        T = t.shape[0]
        Tp, Ts = self._sp_rows(T)
        if Tp != T:
            t = torch.cat([t, torch.zeros(Tp - T, t.shape[1], dtype=t.dtype, device=t.device)])
        if self._sp_host():  # gloo: synchronous, through host memory
            cpu = torch.empty(Ts, t.shape[1], dtype=t.dtype)
            torch.distributed.reduce_scatter_tensor(cpu, t.contiguous().cpu(), group=self.tp_group)
            return cpu.to(t.device), None
        out = torch.empty(Ts, t.shape[1], dtype=t.dtype, device=t.device)
        h = torch.distributed.reduce_scatter_tensor(out, t.contiguous(), group=self.tp_group, async_op=True)
        return out, h

    def _sp_all_gather(self, shard: torch.Tensor, T: int) -> torch.Tensor:
        if self._sp_host():
            cpu = torch.empty(shard.shape[0] * self.tp_size, shard.shape[1], dtype=shard.dtype)
            torch.distributed.all_gather_into_tensor(cpu, shard.contiguous().cpu(), group=self.tp_group)
            return cpu.to(shard.device)[:T]
        out = torch.empty(shard.shape[0] * self.tp_size, shard.shape[1], dtype=shard.dtype, device=shard.device)
        torch.distributed.all_gather_into_tensor(out, shard.contiguous(), group=self.tp_group)
        return out[:T]

    def _prefill_quant(self, T: int):
        """(o / gate_up input quant, QKV input quant) of an fp8 prefill of T rows, as run_layers picks them:
        row-wise e4m3 rows made by the norm (single-term for gate_up, two-term for QKV), decided on the FULL
        row count the consumer GEMMs see (ops._quant_ok: above the decode kernels' rows); (False, False) for
        bf16 weights."""
        if self.weight_dtype != "fp8" or not self.device.type == "cuda" or T <= max(_hip().STREAM_MAX_M,
                                                                                    _hip().STREAM_MAX_M_SWIGLU):
            return False, False
        return True, ("split" if _QKV_SPLIT else True)

    def _add_norm_q(self, x: torch.Tensor, residual: torch.Tensor, eps: float, quant):
        """residual += x; the normed rows -- as ops.QuantRows (fp8 prefill: the norm quantises in the same
        pass, ``quant`` True / "split") or bf16."""
        if quant:
            return ops.QuantRows(*_hip().rmsnorm_fp8(x, ops.unit_gain(residual.shape[1], residual.device), eps,
                                                     residual=residual, split=quant == "split"))
        return ops.add_rmsnorm(x, residual, None, eps)

    def _sp_gather_rows(self, x, T: int):
        """All-gather of this rank's normed row shard (bf16 rows or fp8 QuantRows: e4m3 bytes + fp32 row
        scales -- the same bytes on the link as the bf16 rows for two-term, half for single-term)."""
        if isinstance(x, ops.QuantRows):
            q = self._sp_all_gather(x.q.view(torch.uint8), T).view(torch.float8_e4m3fn)
            sc = self._sp_all_gather(x.scale.view(-1, 1), T).view(-1)
            return ops.QuantRows(q.contiguous(), sc.contiguous())
        return self._sp_all_gather(ops.rows(x), T)

    @property
    def tp_sampling(self) -> bool:
        """Sample from the local vocab shard + 8-byte key max instead of gathering the logits."""
        return self.tp_size > 1 and self.custom_ar is not None

    def _gather_vocab(self, logits: torch.Tensor) -> torch.Tensor:
        if self.tp_size == 1:
            return logits
        B, vl = logits.shape
        if logits.is_cuda and torch.distributed.get_backend(self.tp_group) != "nccl":
            # gloo group over GPU tensors (ranks sharing one GPU: the rehearsals, the custom all-reduce
            # recovery test): gather through host memory
            cpu = torch.empty(self.tp_size * B, vl, dtype=logits.dtype)
            torch.distributed.all_gather_into_tensor(cpu, logits.cpu().contiguous(), group=self.tp_group)
            out = cpu.to(logits.device)
            return out.view(self.tp_size, B, vl).permute(1, 0, 2).reshape(B, self.tp_size * vl)
        out = torch.empty(self.tp_size * B, vl, dtype=logits.dtype, device=logits.device)
        torch.distributed.all_gather_into_tensor(out, logits.contiguous(), group=self.tp_group)
        return out.view(self.tp_size, B, vl).permute(1, 0, 2).reshape(B, self.tp_size * vl)

    # ------------------------------------------------------------------ forward
    def run_layers(self, ids: torch.Tensor, positions: torch.Tensor, seq_idx: torch.Tensor,
                   block_tables: torch.Tensor, kcache: torch.Tensor, vcache: torch.Tensor,
                   attention: Callable[[int, torch.Tensor], torch.Tensor], decode: bool = False) -> torch.Tensor:
        """Embedding -> all layers -> final (unit-gain) norm; returns the normed hidden rows [T, hidden]
        -- a tensor, or on the GPU decode path an ops.NormRows (the deferred norm of the last residual).

        Projections go through the fused blocks of ``ops`` (qkv_rope, proj_add_rmsnorm,
        gate_up_swiglu): at decode row counts they run on the MFMA weight-streaming kernels
        with fused epilogues (split-K residual update + deferred RMSNorm, SwiGLU inside the gate_up
        GEMM, RoPE + KV write inside decode attention), at prefill sizes on the 256 x 256 MFMA GEMM.
        """
        c = self.cfg
        residual = ops.embed(ids, self.embed)
        # fp8 prefill: the norms feeding the fp8 GEMMs quantise their rows in the same pass (ops.QuantRows)
        q8 = not decode and self.weight_dtype == "fp8"
        q8qkv = ("split" if _QKV_SPLIT else True) if q8 else False  # the QKV projection's input
        x = ops.rmsnorm(residual, None, c.rms_eps, quant=q8qkv)  # gains folded into the consumer weights
        page = _page_of(kcache, self.hd)
        ar = _TPReduce(self) if self.tp_size > 1 else (LocalReduce(self) if self.emulate_tp_reduce else None)
        last = len(self.layers) - 1
        for i, lw in enumerate(self.layers):
            qkv = ops.qkv_rope(x, lw.wqkv, positions, seq_idx, block_tables, kcache[i], vcache[i], self.cos_sin,
                               self.hq, self.hkv, self.hd, page, defer=decode)
            a = attention(i, qkv)
            x = ops.proj_add_rmsnorm(a, lw.wo, residual, None, c.rms_eps, "o", ar, quant=q8)
            x = ops.mlp(x, lw.wgu, lw.wdown, residual, c.rms_eps, ar,
                        quant=q8qkv if i < last else False)  # the last one feeds the bf16 LM head
        return x

    def logits(self, x: torch.Tensor, gather: bool = True) -> torch.Tensor:
        # decode rows: the LDS-DMA weight-ring stream GEMM (the 1 GB head read once); more rows: the
        # 256 x 256 MFMA GEMM (ops.linear -> ops.hip.linear)
        local = ops.linear(x, self.lm_head)
        return self._gather_vocab(local) if gather else local

    def prefill(self, ids: torch.Tensor, positions: torch.Tensor, seq_idx: torch.Tensor, cu_seqlens: torch.Tensor,
                last_rows: torch.Tensor, block_tables: torch.Tensor, kcache: torch.Tensor, vcache: torch.Tensor,
                seqlens: Optional[List[int]] = None, items: Optional[torch.Tensor] = None,
                gather: bool = True, paged=None, logits: bool = True) -> Optional[torch.Tensor]:
        """Packed varlen prefill; returns logits of each sequence's last token [nseq, vocab]
        (this rank's vocab shard [nseq, vocab / tp] when ``gather`` is False).  ``paged``
        (ops.PagedPrefill): the rows are prompt SLICES that attend to their sequence's cached prefix
        (chunked prefill); ``logits=False`` skips the LM head (a non-final slice)."""
        kw = {}
        if ids.is_cuda:
            kw = {"seqlens": seqlens, "items": items}

        def attention(i, qkv):
            pp = paged.layer(kcache[i], vcache[i]) if paged is not None else None
            return ops.attn_prefill(qkv, cu_seqlens, self.hq, self.hkv, self.hd, self.scale, paged=pp, **kw)

        x = self.run_layers(ids, positions, seq_idx, block_tables, kcache, vcache, attention)
        if not logits:
            return None
        return self.logits(ops.rows(x).index_select(0, last_rows), gather)

    def prefill_passes(self, passes, block_tables: torch.Tensor, kcache: torch.Tensor, vcache: torch.Tensor,
                       gather: bool = True) -> torch.Tensor:
        """Chunked prefill of a tensor-parallel engine with the all-reduces under compute: the packed passes
        (``passes``: objects with ids, positions, seq_idx, cu_seqlens, last_rows, seqlens, items, paged --
        the slices of the same prompts, in order) run LAYER-MAJOR: at every layer each pass's attention
        block is issued, its o-projection all-reduce started on the RCCL stream, and the next pass's
        attention block issued before the first pass waits for its sum; the MLP half likewise.  Pass p+1's
        attention reads pass p's K/V of the same layer, which its QKV stage wrote earlier in stream order.
        All but the last pass's all-reduces overlap another pass's GEMMs (reference
        result_aggregator.py:346-355 is the single long final-reduce call this serves).  Returns the logits
        of the last pass's last rows."""
        c = self.cfg
        eps = c.rms_eps
        page = _page_of(kcache, self.hd)
        sp = self.sequence_parallel and self.tp_size > 1 and self._sp_backend_ok()
        st = []
        for p in passes:
            res = ops.embed(p.ids, self.embed)
            T = int(res.shape[0])
            q8, q8qkv = self._prefill_quant(T)  # fp8: the norms quantise for the fp8 GEMMs (as run_layers)
            x = ops.rmsnorm(res, None, eps, quant=q8qkv)
            # SP: the residual is kept as this rank's row shard (see _sp_rows)
            st.append({"res": self._sp_shard(res) if sp else res, "x": x, "T": T, "q": (q8, q8qkv)})

        def wait(h):  # a waited handle is dropped from the scope at once (AsyncWorks.wait)
            works.wait(h)

        def reduce_async(s, t, key):  # the TP sum of a projection's partial rows
            if sp:
                s[key], s["w"] = self._sp_reduce_scatter_async(t)
            else:
                s[key], s["w"] = t, self._all_reduce_async(t)
            works.add(s["w"])

        def add_norm(s, key, last=False):  # residual += the summed projection; the normed rows for the next GEMM
            wait(s.pop("w"))
            # fp8: the o sum feeds gate_up (single-term rows), the down sum the next QKV (two-term), the last
            # one the bf16 LM head
            quant = False if last else s["q"][0 if key == "o" else 1]
            x = self._add_norm_q(s.pop(key), s["res"], eps, quant)
            return self._sp_gather_rows(x, s["T"]) if sp else x

        # every async collective started below is waited before this frame is left, also when an op raises
        # (parallel/dist.py AsyncWorks): no work handle outlives the prefill
        with AsyncWorks() as works:
            for i, lw in enumerate(self.layers):
                for p, s in zip(passes, st):
                    if "d" in s:  # previous layer's down-projection sum (overlapped with the other passes' MLPs)
                        s["x"] = add_norm(s, "d")
                    qkv = ops.qkv_rope(s["x"], lw.wqkv, p.positions, p.seq_idx, block_tables, kcache[i],
                                       vcache[i], self.cos_sin, self.hq, self.hkv, self.hd, page)
                    kw = {"seqlens": p.seqlens, "items": p.items} if qkv.is_cuda else {}
                    pp = p.paged.layer(kcache[i], vcache[i]) if p.paged is not None else None
                    a = ops.attn_prefill(qkv, p.cu_seqlens, self.hq, self.hkv, self.hd, self.scale, paged=pp, **kw)
                    reduce_async(s, ops.linear(a, lw.wo), "o")
                for s in st:
                    x = add_norm(s, "o")
                    act = ops.gate_up_swiglu(x, lw.wgu)
                    reduce_async(s, ops.linear(act, lw.wdown), "d")
            last, s = passes[-1], st[-1]
            for t in st[:-1]:
                wait(t.pop("w"))
            x = add_norm(s, "d", last=True)
        return self.logits(x.index_select(0, last.last_rows), gather)

    def prefill_cp(self, passes, block_tables: torch.Tensor, kcache: torch.Tensor, vcache: torch.Tensor,
                   exchange, logits_pass: Optional[int] = None) -> Optional[torch.Tensor]:
        """Context-parallel prefill (SURVEY §2.5 CP): ``passes`` are THIS rank's slices of one prompt (full
        weights on every rank, no activation all-reduces), run layer-major.  Slice k of every rank is
        exchanged on its own: right after pass k's QKV stage has written its K/V rows into the local paged
        cache, ``exchange.start(layer, k)`` starts the all-gather of every rank's slice-k rows (RCCL's
        stream), and ``exchange.finish(handle)`` -- just before pass k's attention -- waits for it and
        scatters the rows into the cache.  With the zigzag split (slice 0 early, slice 1 late) pass k's
        causal prefix lies in slices <= k of the ranks, so exchange 0 overlaps pass 1's QKV and exchange 1
        overlaps pass 0's attention + MLP.  Returns the logits of ``passes[logits_pass]``'s last row (the
        rank holding the prompt's end), else None."""
        c = self.cfg
        eps = c.rms_eps
        page = _page_of(kcache, self.hd)
        st = []
        for p in passes:
            res = ops.embed(p.ids, self.embed)
            q8, q8qkv = self._prefill_quant(int(res.shape[0]))  # fp8 weights: quantising norms (run_layers)
            st.append({"res": res, "x": ops.rmsnorm(res, None, eps, quant=q8qkv), "q": (q8, q8qkv)})
        last_layer = len(self.layers) - 1
        with AsyncWorks() as works:  # every started exchange is waited, also when an op raises
            for i, lw in enumerate(self.layers):
                qkvs, handles = [], []
                for k, (p, s) in enumerate(zip(passes, st)):
                    qkvs.append(ops.qkv_rope(s["x"], lw.wqkv, p.positions, p.seq_idx, block_tables, kcache[i],
                                             vcache[i], self.cos_sin, self.hq, self.hkv, self.hd, page))
                    handles.append(exchange.start(i, k))
                    works.add(handles[-1][2])
                for p, s, qkv, h in zip(passes, st, qkvs, handles):
                    exchange.finish(h, works)
                    kw = {"seqlens": p.seqlens, "items": p.items} if qkv.is_cuda else {}
                    a = ops.attn_prefill(qkv, p.cu_seqlens, self.hq, self.hkv, self.hd, self.scale,
                                         paged=p.paged.layer(kcache[i], vcache[i]), **kw)
                    q8, q8qkv = s["q"]
                    x = ops.proj_add_rmsnorm(a, lw.wo, s["res"], None, eps, "o", None, quant=q8)
                    act = ops.gate_up_swiglu(x, lw.wgu)
                    s["x"] = ops.proj_add_rmsnorm(act, lw.wdown, s["res"], None, eps, "down", None,
                                                  quant=q8qkv if i < last_layer else False)
        if logits_pass is None:
            return None
        p, s = passes[logits_pass], st[logits_pass]
        return self.logits(ops.rows(s["x"]).index_select(0, p.last_rows))

    def decode(self, ids: torch.Tensor, positions: torch.Tensor, seq_idx: torch.Tensor, block_tables: torch.Tensor,
               kcache: torch.Tensor, vcache: torch.Tensor, workspace=None, gather: bool = True) -> torch.Tensor:
        """One token per sequence; context = positions + 1.  Returns logits [B, vocab] (or the local
        vocab shard when ``gather`` is False)."""
        page = _page_of(kcache, self.hd)

        def attention(i, qkv):
            return ops.attn_decode(qkv, kcache[i], vcache[i], block_tables, positions, self.hq, self.hkv, self.hd,
                                   page, self.scale, workspace=workspace)

        x = self.run_layers(ids, positions, seq_idx, block_tables, kcache, vcache, attention, decode=True)
        return self.logits(x, gather)
