"""The on-node batched generation engine (replaces the reference's remote
LLM call, ``llm_executor.py:232-409``).

Scheduling model (continuous batching, offline batch):

* A request reserves KV pages for ``prompt + max_new`` tokens at admission.
* Prefill: waiting requests are packed (varlen, no padding) into forward
  passes of up to ``max_prefill_tokens`` tokens; each sequence's first
  token is sampled straight into its decode slot.
* Decode: the active sequences occupy decode slots ``[0, n)``; a step runs
  the model over the smallest captured batch bucket >= n.  All per-step
  state (next ids, positions, generated tokens, stop flags) lives on the
  device and is advanced by the sampler's finish kernel, so the host only
  replays a captured hipGraph (``torch.cuda.CUDAGraph``) ``sync_every``
  times, then reads the stop flags, retires finished sequences (freeing
  their pages and compacting slots) and admits waiting ones.

This is the "semaphore fan-out" of the reference re-thought for one GPU:
every chunk of a rank is in flight at once, bounded only by HBM.
"""

from __future__ import annotations

import logging
import os
import time
from dataclasses import dataclass, field
from types import SimpleNamespace
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from .config import PREFILL_CHUNK, ModelConfig
from .kv_cache import PagedKVCache
from .model import LlamaModel

log = logging.getLogger("mrsum.engine")

BUCKETS = (1, 2, 4, 8, 16, 24, 32, 40, 48, 64, 80, 96, 128, 160, 192, 224, 256)
MAX_WINDOW = 256  # decode steps between host syncs when no row can stop early (LLMEngine._window)


def _always() -> bool:
    return True


@dataclass
class SamplingParams:
    max_new_tokens: int = 1000
    temperature: float = 0.3
    seed: int = 0


@dataclass
class GenOutput:
    token_ids: List[int]
    prompt_len: int
    finish_reason: str  # "stop" | "length"


@dataclass
class _Seq:
    rid: int
    prompt: List[int]
    params: SamplingParams
    pages: List[int] = field(default_factory=list)
    slot: int = -1
    imported: Optional["ImportedPrefill"] = None
    spans: List[Tuple[int, int]] = field(default_factory=list)  # interleaved prefill: slices still to run
    pf_slot: int = -1  # interleaved prefill: row of LLMEngine.pf_tables


@dataclass
class ImportedPrefill:
    """A prompt prefilled ELSEWHERE (another engine / rank): its first sampled token and this engine's
    share of its KV, ``kv`` [2, n_layers, ceil(prompt / page), hkv_local, page, head_dim] (K then V,
    whole pages; rows past the prompt are ignored).  See LLMEngine.prefill_export."""
    first_token: int
    kv: Optional[torch.Tensor]


class DecodeState:
    """Device-resident per-slot decode state (one row per decode slot)."""

    def __init__(self, max_seqs: int, max_pages: int, max_new_cap: int, device, eos: Sequence[int]):
        i32 = dict(dtype=torch.int32, device=device)
        self.max_seqs = max_seqs
        self.next_ids = torch.zeros(max_seqs, **i32)
        self.positions = torch.zeros(max_seqs, **i32)
        self.seq_idx = torch.arange(max_seqs, **i32)
        self.block_tables = torch.zeros(max_seqs, max_pages, **i32)
        self.gen_count = torch.zeros(max_seqs, **i32)
        self.max_new = torch.ones(max_seqs, **i32)
        self.out_tokens = torch.zeros(max_seqs, max_new_cap, **i32)
        self.done = torch.ones(max_seqs, **i32)
        self.result = torch.zeros(max_seqs, dtype=torch.int64, device=device)
        self.temps = torch.zeros(max_seqs, dtype=torch.float32, device=device)
        self.seeds = torch.zeros(max_seqs, dtype=torch.int64, device=device)
        # the sampler's finish kernel reads these 4 stop ids from device memory at every launch (-1 =
        # unused slot), so captured decode graphs follow the stop set at REPLAY time (set_eos)
        self.eos = torch.full((4,), -1, **i32)
        self.eos_ids: List[int] = []
        self.set_eos(eos)

    def set_eos(self, ids: Sequence[int]) -> None:
        """Stop ids of every later sampler launch, captured graphs included (at most 4; [] = none)."""
        ids = [int(x) for x in ids]
        if len(ids) > 4 or any(x < 0 for x in ids):
            raise ValueError("at most 4 non-negative EOS ids, got %s" % ids)
        self.eos.copy_(torch.tensor(ids + [-1] * (4 - len(ids)), dtype=torch.int32), non_blocking=False)
        self.eos_ids = ids

    _ROW_FIELDS = ("next_ids", "positions", "block_tables", "gen_count", "max_new", "out_tokens", "done", "result",
                   "temps", "seeds")

    def view(self, start: int, n: int) -> "DecodeState":
        v = object.__new__(DecodeState)
        v.max_seqs = n
        for f in self._ROW_FIELDS:
            setattr(v, f, getattr(self, f)[start:start + n])
        v.seq_idx = self.seq_idx[:n]
        v.eos, v.eos_ids = self.eos, self.eos_ids
        return v

    def move_row(self, src: int, dst: int) -> None:
        for f in self._ROW_FIELDS:
            t = getattr(self, f)
            t[dst].copy_(t[src])

    def park_row(self, i: int) -> None:
        """Idle slot: stopped, position 0, all pages -> scratch page 0."""
        self.done[i] = 1
        self.positions[i] = 0
        self.block_tables[i].zero_()
        self.gen_count[i] = 0


class _CPExchange:
    """Per-slice K/V all-gather of a context-parallel prefill (LLMEngine.prefill_export_cp /
    LlamaModel.prefill_cp): slice k of every rank's zigzag split is exchanged on its own, asynchronously
    (RCCL on its own stream; gloo async on CPU ranks), and the received rows land in the paged cache in ONE
    kv_scatter kernel per slice (own and padding rows carry page -1)."""

    def __init__(self, eng: "LLMEngine", pages: List[int], slices, rank: int, world: int, group):
        import torch.distributed as dist
        self.eng, self.rank, self.world, self.group = eng, rank, world, group
        self.nccl = dist.get_backend(group) == "nccl"
        dev, P = eng.device, eng.page
        pg = torch.tensor(pages, dtype=torch.long)
        self.mine, self.width, self.dst = [], [], []
        for k in range(len(slices[rank])):
            rows = [torch.arange(b, e) for b, e in (slices[q][k] for q in range(world))]
            width = max(1, max(int(r.numel()) for r in rows))
            b, e = slices[rank][k]
            own = torch.arange(b, e)
            self.mine.append(((pg[own // P]).to(dev), (own % P).to(dev), int(own.numel())))
            # destination (page, slot) of every gathered row, rank-major with padding; own rows -> -1
            page_d = torch.full((world, width), -1, dtype=torch.int32)
            slot_d = torch.zeros((world, width), dtype=torch.int32)
            for q, r in enumerate(rows):
                if q != rank and r.numel():
                    page_d[q, :r.numel()] = pg[r // P].to(torch.int32)
                    slot_d[q, :r.numel()] = (r % P).to(torch.int32)
            self.width.append(width)
            self.dst.append((page_d.reshape(-1).to(dev), slot_d.reshape(-1).to(dev)))

    def start(self, layer: int, k: int):
        """Gather this rank's slice-k K/V rows of ``layer`` and start the all-gather (returns a handle)."""
        import torch.distributed as dist
        e = self.eng
        kc, vc = e.kv.k[layer], e.kv.v[layer]
        p0, r0, n0 = self.mine[k]
        mine = torch.zeros(self.width[k], 2, e.model.hkv, e.cfg.head_dim, dtype=kc.dtype, device=e.device)
        mine[:n0, 0] = kc[p0, :, r0, :]
        mine[:n0, 1] = vc[p0, :, r0, :]
        if self.nccl:
            out = torch.empty((self.world,) + tuple(mine.shape), dtype=kc.dtype, device=e.device)
            work = dist.all_gather_into_tensor(out, mine, group=self.group, async_op=True)
        else:
            out = [torch.empty_like(mine, device="cpu") for _ in range(self.world)]
            work = dist.all_gather(out, mine.cpu(), group=self.group, async_op=True)
        return (layer, k, work, out, mine)

    def finish(self, h, works=None) -> None:
        """Wait for a started exchange and scatter the other ranks' rows into the paged cache; ``works``
        (parallel/dist.py AsyncWorks) stops tracking the handle once waited, so its buffers can go."""
        layer, k, work, out, _mine = h
        if works is not None:
            works.wait(work)
        else:
            work.wait()
        e = self.eng
        rows = out if self.nccl else torch.stack(out).to(e.device)
        page_d, slot_d = self.dst[k]
        ops.kv_scatter(rows.reshape(-1, 2, e.model.hkv, e.cfg.head_dim).contiguous(), page_d, slot_d,
                       e.kv.k[layer], e.kv.v[layer])


class LLMEngine:
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 max_num_seqs: int = 256, max_model_len: int = 16384, max_new_cap: int = 2048,
                 kv_pages: Optional[int] = None, kv_fraction: float = 0.6, page_size: int = 64,
                 max_prefill_tokens: int = 32768, use_graphs: bool = True, sync_every: int = 16,
                 eos_ids: Sequence[int] = (128001, 128009), tp_rank: int = 0, tp_size: int = 1, tp_group=None,
                 weight_dtype: str = "bf16", weights_path: Optional[str] = None, prefill_chunk: int = PREFILL_CHUNK,
                 kv_dtype: Optional[str] = None):
        """``kv_dtype``: "bf16" (default, $MRSUM_KV_DTYPE), "fp8v" (V rows fp8, K bf16) or "fp8" -- e4m3fn K/V rows with power-of-two
        row scales (engine/kv_cache.py): half the KV bytes per decode step; no context-parallel prefill.

        ``max_prefill_tokens``: rows of one packed prefill pass (whole prompts up to it; longer prompts are sliced
        by ``prefill_chunk``).  32768: the headline's 39 map prompts of ~4k in 5 passes instead of 10 and its 10
        level-1 prompts of ~5.4k in 2 instead of 4 -- 10 h bench 18.10 / 18.10 -> 18.06 / 18.01 s, A/B/A/B on one
        box (profiles/r6_prefill_budget_ab.jsonl).

        ``prefill_chunk``: cut prompts longer than this many tokens into slices prefilled one pass
        after the other through the paged cache (chunked prefill; 0 = one pass per prompt).  At 32k
        tokens on Llama-3-8B 4096-token slices took 0.669 s vs 0.701 s in one pass (profiles/
        r2_chunked_prefill_32k_ab.jsonl); 8192-token slices keep every GEMM's 256-row tile grid whole waves on
        256 CUs (4096 rows left the QKV projections at 1.5 / 2.5 waves): Llama-3-70B fp8 at 32k 3.21 s vs
        3.27 with 4096 and 3.23 with 16384, Llama-3-8B at 13.5k / 32k 0.203 / 0.607 s vs 0.207 / 0.610
        (profiles/r5_prefill_chunk_{70b,8b}_ab.jsonl)."""
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.kv_dtype = kv_dtype or os.environ.get("MRSUM_KV_DTYPE", "bf16")
        t0 = time.perf_counter()
        self.model = LlamaModel(cfg, self.device, dtype, seed, tp_rank, tp_size, tp_group, weight_dtype=weight_dtype,
                                 weights_path=weights_path)
        self.init_seconds = time.perf_counter() - t0
        self.page = page_size
        self.max_model_len = min(max_model_len, cfg.max_position)
        self.max_num_seqs = min(max_num_seqs, BUCKETS[-1])
        self.max_new_cap = max_new_cap
        self.max_prefill_tokens = int(os.environ.get("MRSUM_MAX_PREFILL_TOKENS", max_prefill_tokens))
        self.prefill_chunk = int(os.environ.get("MRSUM_PREFILL_CHUNK", prefill_chunk))
        # one-pass prefill attention reads the packed qkv rows (the paged-cache path measured equal:
        # profiles/r2_chunked_prefill_32k_ab.jsonl); tools/bench_prefill.py flips this for the A/B
        self.paged_prefill = False
        if self.prefill_chunk and self.prefill_chunk % page_size:
            raise ValueError("prefill_chunk must be a multiple of the page size (%d)" % page_size)
        self.sync_every = max(1, sync_every)
        if kv_pages is None:
            if self.device.type == "cuda":
                free, _total = torch.cuda.mem_get_info(self.device)
                budget = int(free * kv_fraction)
            else:
                budget = 256 << 20
            kv_pages = PagedKVCache.size_pages(budget, cfg.n_layers, self.model.hkv, page_size, cfg.head_dim,
                                               kv_dtype=self.kv_dtype)
            # no point holding more than every slot at full length
            kv_pages = min(kv_pages, 1 + self.max_num_seqs * -(-self.max_model_len // page_size))
        self.kv = PagedKVCache(cfg.n_layers, kv_pages, self.model.hkv, page_size, cfg.head_dim, dtype, self.device,
                               kv_dtype=self.kv_dtype)
        self.max_pages = -(-self.max_model_len // page_size)
        self.state = DecodeState(self.max_num_seqs, self.max_pages, max_new_cap, self.device, eos_ids)
        # block tables of requests whose prefill is interleaved with the running decode (they hold no
        # decode slot until their last slice has run, so no decode step can touch their pages)
        self.pf_tables = torch.zeros(self.max_num_seqs, self.max_pages, dtype=torch.int32, device=self.device)
        self.interleave = os.environ.get("MRSUM_INTERLEAVE", "1") == "1"
        # test hook (SURVEY §5.3 fault injection): "rank:seconds" -- TP rank ``rank`` sleeps on the host
        # before its first decode window, so its peers' P2P all-reduce waits time out (recovery test)
        spec = os.environ.get("MRSUM_FAULT_AR_DELAY", "")
        self._fault_delay = tuple(float(x) for x in spec.split(":")) if spec else None
        self.use_graphs = use_graphs and self.device.type == "cuda"
        if self.use_graphs and self.model.tp_size > 1 and self.model.custom_ar is None:
            # TP without the P2P all-reduce would put RCCL collectives inside the captured graphs;
            # replay them eagerly instead (RCCL stays outside any capture)
            log.warning("TP=%d without the custom all-reduce: decode hipGraphs disabled", self.model.tp_size)
            self.use_graphs = False
        # decode graphs / attention workspaces per (batch bucket, context class): the attention's split
        # plan depends on how long the contexts get (ops.hip.decode_attn_plan)
        self._graphs: Dict[Tuple[int, int], "torch.cuda.CUDAGraph"] = {}
        self._ctx_cls = 0
        self._on_prefill = None
        self._workspaces: Dict[Tuple[int, int], object] = {}
        self.stats = {"prefill_tokens": 0, "prefill_s": 0.0, "decode_steps": 0, "decode_tokens": 0,
                      "decode_s": 0.0, "generate_calls": 0, "graph_captures": 0, "peak_active": 0}

    # ------------------------------------------------------------------ helpers
    def _bucket(self, n: int) -> int:
        for b in BUCKETS:
            if b >= n:
                return min(b, self.max_num_seqs)
        return self.max_num_seqs

    def _ctx_classes(self) -> int:
        """Number of context classes this engine can reach (ops.hip.CTX_CLASSES up to max_model_len)."""
        from ..ops.hip import ctx_class
        return ctx_class(self.max_model_len) + 1

    def _workspace(self, B: int):
        if self.device.type != "cuda":
            return None
        key = (B, self._ctx_cls)
        ws = self._workspaces.get(key)
        if ws is None:
            from ..ops.hip import CTX_CLASSES, DecodeWorkspace, decode_attn_plan, decode_groups
            ng = decode_groups(self.model.hq, self.model.hkv)  # kv heads, or query heads for odd GQA ratios
            s, fused = decode_attn_plan(B, ng, min(CTX_CLASSES[self._ctx_cls], self.max_model_len),
                                        kv8=self.kv.kv_dtype if self.kv.fp8 else False)
            ws = DecodeWorkspace(B, self.model.hq, self.cfg.head_dim, s, self.device, ng, fused_combine=fused)
            self._workspaces[key] = ws
        return ws

    def _sync(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ prefill
    def _prefill(self, seqs: List[_Seq]) -> None:
        """Prefill ``seqs`` (already holding pages + consecutive slots) and sample their first tokens.

        Chunked prefill (``prefill_chunk`` > 0 and some prompt longer than it): every prompt is cut into
        slices of at most ``prefill_chunk`` tokens aligned to its END, and pass r packs the r-th-from-last
        slice of every prompt that has one, so the final slices -- whose last rows are sampled -- all run
        in the last pass.  A slice's queries attend to the cached positions before it through the paged
        cache (ops.PagedPrefill, attn_prefill_paged); the K/V of every slice enter the cache before its
        attention, as in one-shot prefill."""
        chunk = self.prefill_chunk
        if self.model.tp_size > 1 and self.model.sequence_parallel and self.model._sp_backend_ok() and \
                (not chunk or max(len(s.prompt) for s in seqs) <= chunk):
            # tensor parallel, one pass: the layer-major path (sequence-parallel norms, async reductions)
            x = self._pass_inputs(seqs, [(0, len(s.prompt)) for s in seqs], paged=True)
            logits = self.model.prefill_passes([x], self.state.block_tables, self.kv.k, self.kv.v,
                                               gather=not self.model.tp_sampling)
            self.stats["prefill_tokens"] += int(x.ids.numel())
            self._sample_first(seqs, logits)
            return
        if not chunk or max(len(s.prompt) for s in seqs) <= chunk:
            self._prefill_pass(seqs, [(0, len(s.prompt)) for s in seqs], paged=self.paged_prefill)
            return
        rounds = max(-(-len(s.prompt) // chunk) for s in seqs)
        passes = []
        for r in range(rounds):
            k = rounds - 1 - r  # slices still to come after this one
            part, spans = [], []
            for s in seqs:
                n = len(s.prompt)
                end = n - k * chunk
                if end > 0:
                    part.append(s)
                    spans.append((max(0, end - chunk), end))
            passes.append((part, spans))
            self.stats["prefill_slices"] = self.stats.get("prefill_slices", 0) + len(part)
        if self.model.tp_size > 1:
            # tensor parallel: all passes layer-major, each pass's all-reduces under the next one's GEMMs
            inputs = [self._pass_inputs(part, spans, paged=True) for part, spans in passes]
            logits = self.model.prefill_passes(inputs, self.state.block_tables, self.kv.k, self.kv.v,
                                               gather=not self.model.tp_sampling)
            self.stats["prefill_tokens"] += sum(int(x.ids.numel()) for x in inputs)
            self._sample_first(passes[-1][0], logits)
            return
        for r, (part, spans) in enumerate(passes):
            self._prefill_pass(part, spans, paged=True, final=(r == rounds - 1))

    def _pass_inputs(self, seqs: List[_Seq], spans, paged: bool, tables: Optional[torch.Tensor] = None,
                     slots: Optional[List[int]] = None, sample: Optional[List[bool]] = None):
        """Device inputs of one packed forward over prompt slices ``spans`` [(start, end)] of ``seqs``
        (block-table rows ``slots`` of ``tables``: default the decode slots of the decode state;
        ``sample``: which sequences' last rows feed the LM head, default all)."""
        st, dev = self.state, self.device
        tables = st.block_tables if tables is None else tables
        slots = [s.slot for s in seqs] if slots is None else slots
        # numpy assembly: torch.tensor() over Python lists of a 16k-token pass cost ~5 ms of host time
        lens = [e - b for b, e in spans]
        cu = np.zeros(len(spans) + 1, dtype=np.int32)
        np.cumsum(lens, out=cu[1:])
        ids = np.concatenate([np.asarray(s.prompt[b:e], dtype=np.int32) for s, (b, e) in zip(seqs, spans)])
        pos = np.concatenate([np.arange(b, e, dtype=np.int32) for b, e in spans])
        sidx = np.repeat(np.asarray(slots, dtype=np.int32), lens)
        last = [int(cu[k + 1]) - 1 for k in range(len(spans)) if sample is None or sample[k]]
        h = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.int32)).to(dev, non_blocking=True)  # noqa: E731
        items = None
        if dev.type == "cuda":
            from ..ops.hip import prefill_items
            items = prefill_items(lens, self.model.hq // self.model.hkv).to(dev, non_blocking=True)
        pp = None
        if paged:
            pre = [b for b, _ in spans]
            pp = ops.PagedPrefill(tables, h(slots), h(pre), list(slots), pre)
        return SimpleNamespace(ids=h(ids), positions=h(pos), seq_idx=h(sidx), cu_seqlens=h(cu),
                               last_rows=torch.tensor(last, dtype=torch.long).to(dev, non_blocking=True),
                               seqlens=lens, items=items, paged=pp, tables=tables)

    def _sample_first(self, seqs: List[_Seq], logits: torch.Tensor) -> None:
        """Sample every sequence's first generated token from its prompt's last row (fed position
        prompt_len - 1); ``seqs`` occupy consecutive slots."""
        st = self.state
        v = st.view(seqs[0].slot, len(seqs))
        v.positions.copy_(torch.tensor([len(s.prompt) - 1 for s in seqs], dtype=torch.int32).to(
            self.device, non_blocking=True))
        self._sample(logits, v)

    def _prefill_pass(self, seqs: List[_Seq], spans, paged: bool, final: bool = True) -> None:
        """One packed forward over prompt slices ``spans`` [(start, end)] of ``seqs``; on the final pass,
        sample each sequence's first token from its last row."""
        x = self._pass_inputs(seqs, spans, paged)
        logits = self.model.prefill(x.ids, x.positions, x.seq_idx, x.cu_seqlens, x.last_rows, self.state.block_tables,
                                    self.kv.k, self.kv.v, seqlens=x.seqlens, items=x.items,
                                    gather=not self.model.tp_sampling, paged=x.paged, logits=final)
        self.stats["prefill_tokens"] += int(x.ids.numel())
        if final:
            self._sample_first(seqs, logits)

    # ------------------------------------------------------------------ decode
    def _sample(self, logits: torch.Tensor, st_view) -> None:
        if self.model.tp_sampling:  # local vocab shard + cross-rank max of the 8-byte Gumbel keys
            ops.sample_tp(logits, st_view, self.model.vocab_offset, self.model.custom_ar.max_u64_)
        else:
            ops.sample(logits, st_view)

    def _decode_once(self, B: int) -> None:
        st = self.state
        logits = self.model.decode(st.next_ids[:B], st.positions[:B], st.seq_idx[:B], st.block_tables[:B],
                                   self.kv.k, self.kv.v, workspace=self._workspace(B),
                                   gather=not self.model.tp_sampling)
        self._sample(logits, st.view(0, B))

    def _decode_steps(self, B: int, steps: int) -> None:
        if self._fault_delay is not None and int(self._fault_delay[0]) == self.model.tp_rank \
                and self.model.custom_ar is not None:
            delay, self._fault_delay = self._fault_delay[1], None  # once
            log.warning("fault injection: TP rank %d sleeps %.1f s before a decode window", self.model.tp_rank, delay)
            time.sleep(delay)
        if not self.use_graphs:
            for _ in range(steps):
                self._decode_once(B)
            return
        g = self._graphs.get((B, self._ctx_cls))
        if g is None:
            g = self._capture(B)
        for _ in range(steps):
            g.replay()

    def capture_graphs(self, max_batch: Optional[int] = None) -> int:
        """Capture the decode hipGraph of every batch bucket up to ``max_batch`` now (engine start-up,
        like a serving engine) instead of on first use; returns the number captured.  On a TP engine
        every rank must call this with the same ``max_batch`` (the warm-up step runs the all-reduces)."""
        if not self.use_graphs:
            return 0
        n = 0
        keep = self._ctx_cls
        try:
            for B in BUCKETS:
                if B > min(max_batch or self.max_num_seqs, self.max_num_seqs):
                    break
                # every context class for single-sequence steps (a final reduce over a long prompt), the
                # short class for batches
                for cls in range(self._ctx_classes() if B == 1 else 1):
                    self._ctx_cls = cls
                    if (B, cls) not in self._graphs:
                        self._capture(B)
                        n += 1
        finally:
            self._ctx_cls = keep
        self._sync()
        return n

    def _capture(self, B: int):
        # snapshot state rows the warm-up step will advance, run it eagerly once (lazy kernel-library
        # load, workspace and split-K ticket allocation), restore, then capture.
        st = self.state
        snap = {f: getattr(st, f)[:B].clone() for f in DecodeState._ROW_FIELDS}
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._decode_once(B)
        torch.cuda.current_stream(self.device).wait_stream(s)
        for f, t in snap.items():
            getattr(st, f)[:B].copy_(t)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._decode_once(B)
        # capture does not execute; restore anyway in case the backend ran the work
        for f, t in snap.items():
            getattr(st, f)[:B].copy_(t)
        self._graphs[(B, self._ctx_cls)] = g
        self.stats["graph_captures"] += 1
        return g

    # ------------------------------------------------------------------ API
    def generate(self, prompts: Sequence[Sequence[int]], params: Sequence[SamplingParams],
                 ignore_eos: bool = False, imported: Optional[Dict[int, ImportedPrefill]] = None,
                 on_prefill=None, feeder=None, on_sync=None) -> List[GenOutput]:
        """Generate for every prompt.  ``ignore_eos`` pins the work to max_new_tokens per request
        (benchmark mode, SURVEY §7.4: random weights emit EOS at random).

        ``imported``: request index -> ImportedPrefill; those requests skip the prefill (their KV pages
        are copied in and decoding starts from the imported first token).  ``on_prefill(seqs)`` is
        called after every prefill forward with the just-prefilled sequences (pages still held).

        ``feeder(done)``: streaming hook, called at every host sync point with the requests that
        finished since the last call (``[(request index, GenOutput)]``); it returns new
        ``(prompt, SamplingParams)`` requests, which join the running batch (continuous batching) and
        take the next request indices.  The returned list covers every request, fed ones included.

        ``on_sync({request index: token ids so far})``: streaming hook, called at every host sync point
        with the tokens of every active sequence (one device -> host copy of the token buffer per sync);
        an ``on_sync.wanted()`` attribute, when present, is asked first at every sync point and a False
        skips that copy (a server passes the hook always and wants it only while a client streams).
        (The map -> level-1 reduce pipeline uses it: a reduce batch starts as soon as its chunks are
        summarised)"""
        if len(prompts) != len(params):
            raise ValueError("prompts and params differ in length")
        eos = list(self.state.eos_ids)
        if ignore_eos:  # device-side stop set: captured graphs see it at replay (sampler.hip EOS_SLOTS)
            self.state.set_eos([])
        try:
            ar = self.model.custom_ar
            failed: Optional[BaseException] = None
            try:
                out = self._generate(prompts, params, imported or {}, on_prefill, feeder, on_sync)
            except Exception as e:  # noqa: BLE001 -- re-raised below, after the group's vote
                failed = e
            if ar is not None:
                # every TP rank votes whatever happened locally, so the group's collective sequence stays
                # aligned: a local exception fails the call on every rank; a timed-out P2P wait anywhere
                # (the sticky error word) makes every rank re-run the requests on RCCL.  Scope: this covers
                # failures that let the peers reach the vote -- the custom all-reduce's own waits end after
                # 4 s (sticky error word).  A rank that raises BEFORE an RCCL collective inside _generate (the
                # sequence-parallel prefill's reduce-scatter / all-gather, an RCCL logits gather) leaves its
                # peers in that collective until the process-group timeout (MRSUM_DIST_TIMEOUT), which then
                # fails them too.
                ar_err, any_failed = ar.agree_error(failed is not None)
                if any_failed:
                    # the failing call may have stopped between a push and its wait, leaving epochs / granules
                    # half-advanced on some ranks: clear the P2P state on the whole group (collective: every
                    # rank saw the same vote) so the next generate starts clean
                    ar.reset()
                if failed is None and any_failed:
                    raise RuntimeError("a tensor-parallel peer failed during this generate")
                if failed is None and ar_err:
                    out = self._recover_custom_ar(prompts, params, imported or {}, on_prefill, feeder, on_sync)
            if failed is not None:
                raise failed
        finally:
            if ignore_eos:
                self.state.set_eos(eos)
        return out

    def _recover_custom_ar(self, prompts, params, imported, on_prefill, feeder, on_sync) -> List[GenOutput]:
        """A wait of the P2P all-reduce timed out on some rank during this generate (a peer stalled > 4 s:
        host jitter, a slow rank), so its results are garbage on every rank.  Every rank got here (the error
        vote is collective): clear the all-reduce state on the whole group, then run the SAME requests again
        on RCCL (torch.distributed, eager: RCCL never runs inside a captured graph) -- the retry of the
        reference's executor (llm_executor.py:198-228), done inside the engine so it hits a working path.
        The handle is usable again afterwards; later generates use it."""
        if feeder is not None or on_sync is not None:
            # streamed requests were already handed out: they cannot be taken back
            raise RuntimeError("custom all-reduce: a wait for a peer timed out during a streamed generate")
        ar = self.model.custom_ar
        log.error("custom all-reduce: a wait for a peer timed out (TP rank %d); resetting the P2P buffers and "
                  "re-running %d requests on RCCL", self.model.tp_rank, len(prompts))
        self.stats["custom_ar_recoveries"] = self.stats.get("custom_ar_recoveries", 0) + 1
        ar.reset()
        graphs = self.use_graphs
        self.model.custom_ar, self.use_graphs = None, False
        try:
            out = self._generate(prompts, params, imported, on_prefill, None, None)
        finally:
            self.model.custom_ar, self.use_graphs = ar, graphs
        return out

    def _new_seq(self, i: int, p: Sequence[int], sp: SamplingParams, imported=None) -> _Seq:
        p = list(p)
        if not p:
            raise ValueError("empty prompt")
        mn = max(1, min(sp.max_new_tokens, self.max_new_cap))
        if len(p) + mn > self.max_model_len:
            raise ValueError("prompt of %d tokens + %d new exceeds max_model_len %d"
                             % (len(p), mn, self.max_model_len))
        if max(p) >= self.cfg.vocab_size or min(p) < 0:
            raise ValueError("token id out of range")
        return _Seq(i, p, SamplingParams(mn, sp.temperature, sp.seed), imported=imported)

    def _fit_ctx_class(self, seqs: Sequence[_Seq]) -> None:
        """Decode attention split plan (graphs are keyed by it) for the longest sequence in flight."""
        if seqs and self.device.type == "cuda":
            from ..ops.hip import ctx_class
            self._ctx_cls = max(self._ctx_cls, ctx_class(max(len(s.prompt) + s.params.max_new_tokens for s in seqs)))

    def _generate(self, prompts: Sequence[Sequence[int]], params: Sequence[SamplingParams],
                  imported: Dict[int, ImportedPrefill], on_prefill, feeder=None, on_sync=None) -> List[GenOutput]:
        self.stats["generate_calls"] += 1
        self._on_prefill = on_prefill
        results: List[Optional[GenOutput]] = [None] * len(prompts)
        finished: List[int] = []  # request indices done since the last feeder call
        waiting: List[_Seq] = []
        for i, (p, sp) in enumerate(zip(prompts, params)):
            s = self._new_seq(i, p, sp, imported.get(i))
            if s.imported is not None:
                tok = int(s.imported.first_token)
                mn = s.params.max_new_tokens
                if mn == 1 or tok in self.state.eos_ids:
                    results[i] = GenOutput([tok], len(s.prompt), "length" if mn == 1 else "stop")  # done at prefill
                    finished.append(i)
                    continue
            waiting.append(s)
        # longest first: better packing and no late long straggler
        waiting.sort(key=lambda s: -(len(s.prompt) + s.params.max_new_tokens))
        self._ctx_cls = 0
        self._fit_ctx_class(waiting)
        active: List[_Seq] = []
        st = self.state
        if feeder is not None and finished:
            self._feed(feeder, finished, results, waiting)
        prefilling: List[_Seq] = []  # admitted while a batch decodes: prefilled slice by slice
        t_window_end = None
        while waiting or active or prefilling:
            if active and self.interleave:
                # requests joining a RUNNING batch: admit them into the prefill table and run ONE packed
                # slice pass before each decode window, so the running sequences keep advancing (their
                # longest inter-token gap is one slice's forward, not the joiners' whole prefill)
                self._admit_interleaved(waiting, active, prefilling)
                if prefilling:
                    self._interleaved_pass(prefilling, active)
                admitted = None
            else:
                while prefilling:  # nothing decodes: no one waits for the remaining slices
                    self._interleaved_pass(prefilling, active)
                admitted = self._admit(waiting, active)
            if not active:
                if prefilling:
                    continue
                raise MemoryError("cannot admit any request: KV cache too small")
            n = len(active)
            self.stats["peak_active"] = max(self.stats["peak_active"], n)
            B = self._bucket(n)
            # one readback: stop flags and steps left of every row
            snap = torch.stack((st.done[:n], st.max_new[:n] - st.gen_count[:n])).cpu()
            left = [int(r) for d, r in zip(snap[0].tolist(), snap[1].tolist()) if not d]
            steps = self._window(left, feeder is not None or on_sync is not None or bool(prefilling))
            if steps:
                t0 = time.perf_counter()
                if t_window_end is not None:  # host work + prefill between two windows of running rows
                    self.stats["max_window_gap_s"] = max(self.stats.get("max_window_gap_s", 0.0), t0 - t_window_end)
                self._decode_steps(B, steps)
                self._sync()
                t_window_end = time.perf_counter()
                self.stats["decode_s"] += t_window_end - t0
                self.stats["decode_steps"] += steps
                self.stats["decode_windows"] = self.stats.get("decode_windows", 0) + 1
            done, gen = torch.stack((st.done[:n], st.gen_count[:n])).cpu()
            if on_sync is not None and steps and getattr(on_sync, "wanted", _always)():
                toks_all = st.out_tokens[:n].cpu()
                on_sync({active[i].rid: toks_all[i, :int(gen[i])].tolist() for i in range(n)})
            fin = [i for i in range(n) if int(done[i])]
            if fin:
                toks = st.out_tokens[:n].cpu()
                for i in fin:
                    s = active[i]
                    g = int(gen[i])
                    ids = toks[i, :g].tolist()
                    reason = "length" if g >= s.params.max_new_tokens else "stop"
                    results[s.rid] = GenOutput(ids, len(s.prompt), reason)
                    finished.append(s.rid)
                    self.stats["decode_tokens"] += g
                    self.kv.alloc.free(s.pages)
                self._compact(active, set(fin))
                if not active:
                    t_window_end = None
            if feeder is not None:  # every sync point: new requests join without waiting for a finish
                self._feed(feeder, finished, results, waiting)
            del admitted
        return [r for r in results]  # type: ignore[return-value]

    def _window(self, left: List[int], hooked: bool) -> int:
        """Decode steps to replay before the next host sync, given the steps ``left`` of every running row.

        Default: ``sync_every`` (a row may stop at an EOS id any step; the sync retires it and admits
        waiting requests).  With no stop ids armed (``ignore_eos``: every request runs to its
        max_new_tokens) and nobody to serve at sync points (no feeder, no streaming hook, no interleaved
        prefill in progress), nothing can change before the first row runs out of steps, so the window
        is that many steps (at most ``MAX_WINDOW``): the host does not stop the device every
        ``sync_every`` steps to read flags it can predict (each such stop idles the GPU for the
        read-back and the next graph launch, ~0.5 ms; 188 of them per step of the 10 h bench)."""
        left = [x for x in left if x > 0]
        if not left:
            return 0
        if self.state.eos_ids or hooked:
            return min(self.sync_every, max(left))
        return min(MAX_WINDOW, min(left))

    def _feed(self, feeder, finished: List[int], results: List[Optional[GenOutput]], waiting: List[_Seq]) -> None:
        """Hand the just-finished requests to ``feeder`` and queue the requests it returns."""
        done = [(i, results[i]) for i in finished]
        finished.clear()
        new = []
        for p, sp in feeder(done) or ():
            s = self._new_seq(len(results), p, sp)
            results.append(None)
            new.append(s)
        if new:
            self.stats["fed_requests"] = self.stats.get("fed_requests", 0) + len(new)
            waiting.extend(sorted(new, key=lambda s: -(len(s.prompt) + s.params.max_new_tokens)))
            self._fit_ctx_class(new)

    def _admit(self, waiting: List[_Seq], active: List[_Seq]) -> List[_Seq]:
        """Admit waiting requests into decode slots, prefilling them in packed batches of at most
        ``max_prefill_tokens``.  The batches are enqueued back to back and the device is synchronised once,
        after the last: the host assembles batch k+1 while batch k runs (a sync per batch idled the GPU for
        that assembly, ~3-5 ms per 16k-token pass)."""
        st = self.state
        batch: List[_Seq] = []
        tokens = 0
        t0 = time.perf_counter()
        ran = False
        while waiting and len(active) + len(batch) < self.max_num_seqs:
            s = waiting[0]
            need = self.kv.pages_for(len(s.prompt) + s.params.max_new_tokens)
            if need > self.kv.alloc.available():
                break
            if batch and (s.imported is not None or tokens + len(s.prompt) > self.max_prefill_tokens):
                # full prefill batch, or an imported prefill (slots stay in admission order): flush
                self._run_prefill(batch, active)
                ran = True
                batch, tokens = [], 0
                continue
            waiting.pop(0)
            s.pages = self.kv.alloc.alloc(need)
            s.slot = len(active) + len(batch)
            row = torch.zeros(self.max_pages, dtype=torch.int32)
            row[:need] = torch.tensor(s.pages, dtype=torch.int32)
            st.block_tables[s.slot].copy_(row.to(self.device, non_blocking=True))
            st.max_new[s.slot] = s.params.max_new_tokens
            st.gen_count[s.slot] = 0
            st.done[s.slot] = 0
            st.temps[s.slot] = float(s.params.temperature)
            st.seeds[s.slot] = int(s.params.seed)
            st.result[s.slot] = 0
            if s.imported is not None:  # no forward pass: KV + first token come from elsewhere
                self._install(s)
                active.append(s)
                continue
            batch.append(s)
            tokens += len(s.prompt)
        if batch:
            self._run_prefill(batch, active)
            ran = True
        if ran:
            self._sync()
            self.stats["prefill_s"] += time.perf_counter() - t0
        return batch

    def _slices(self, n: int) -> List[Tuple[int, int]]:
        """Prefill slices of an ``n``-token prompt, aligned to its END exactly as ``_prefill`` cuts them
        (so an interleaved prefill runs the same slices as a blocking one)."""
        c = self.prefill_chunk
        if not c or n <= c:
            return [(0, n)]
        r = -(-n // c)
        return [(max(0, n - (k + 1) * c), n - k * c) for k in reversed(range(r))]

    def _admit_interleaved(self, waiting: List[_Seq], active: List[_Seq], prefilling: List[_Seq]) -> None:
        """Reserve pages (and a prefill-table row) for waiting requests while a batch decodes; their
        forward passes run slice by slice in ``_interleaved_pass``.  Imported prefills need no forward:
        they are installed into a decode slot at once."""
        st = self.state
        used = {s.pf_slot for s in prefilling}
        while waiting and len(active) + len(prefilling) < self.max_num_seqs:
            s = waiting[0]
            need = self.kv.pages_for(len(s.prompt) + s.params.max_new_tokens)
            if need > self.kv.alloc.available():
                break
            waiting.pop(0)
            s.pages = self.kv.alloc.alloc(need)
            row = torch.zeros(self.max_pages, dtype=torch.int32)
            row[:need] = torch.tensor(s.pages, dtype=torch.int32)
            if s.imported is not None:
                s.slot = len(active)
                self._setup_slot(s, row)
                self._install(s)
                active.append(s)
                continue
            s.pf_slot = next(i for i in range(self.max_num_seqs) if i not in used)
            used.add(s.pf_slot)
            self.pf_tables[s.pf_slot].copy_(row.to(self.device, non_blocking=True))
            s.spans = self._slices(len(s.prompt))
            prefilling.append(s)
            self.stats["interleaved_prefills"] = self.stats.get("interleaved_prefills", 0) + 1

    def _setup_slot(self, s: _Seq, row: torch.Tensor) -> None:
        """Decode-state row of ``s`` at ``s.slot``: its pages, budget and sampling parameters."""
        st = self.state
        st.block_tables[s.slot].copy_(row.to(self.device, non_blocking=True))
        st.max_new[s.slot] = s.params.max_new_tokens
        st.gen_count[s.slot] = 0
        st.done[s.slot] = 0
        st.temps[s.slot] = float(s.params.temperature)
        st.seeds[s.slot] = int(s.params.seed)
        st.result[s.slot] = 0

    def _interleaved_pass(self, prefilling: List[_Seq], active: List[_Seq], max_parts: Optional[int] = None) -> None:
        """One packed forward of the next slices of the prefilling requests (at most ``prefill_chunk``
        tokens, or ``max_prefill_tokens`` without chunking; always at least one slice; at most
        ``max_parts`` slices).  Requests whose LAST slice ran take the next decode slots and sample their
        first token there.  A device out-of-memory error in the forward (TP=1) re-runs the pass with half
        as many slices, down to one -- the running decode batch and the other joiners are unaffected
        (SURVEY §5.3 failure isolation, as ``_prefill_isolated`` for blocking admission)."""
        budget = self.prefill_chunk or self.max_prefill_tokens
        part, spans, tokens = [], [], 0
        for s in prefilling:
            b, e = s.spans[0]
            if part and (tokens + (e - b) > budget or (max_parts is not None and len(part) >= max_parts)):
                break
            part.append(s)
            spans.append((b, e))
            tokens += e - b
        final = [len(s.spans) == 1 for s in part]
        t0 = time.perf_counter()
        try:
            x = self._pass_inputs(part, spans, paged=True, tables=self.pf_tables, slots=[s.pf_slot for s in part],
                                  sample=final)
            logits = self.model.prefill(x.ids, x.positions, x.seq_idx, x.cu_seqlens, x.last_rows, self.pf_tables,
                                        self.kv.k, self.kv.v, seqlens=x.seqlens, items=x.items,
                                        gather=not self.model.tp_sampling, paged=x.paged, logits=any(final))
        except torch.OutOfMemoryError:
            # nothing of this pass is committed yet (spans are popped and slots taken only below; the K/V
            # rows it may have written are rewritten by the retry)
            if len(part) == 1 or self.model.tp_size > 1:
                raise
            if self.device.type == "cuda":
                torch.cuda.empty_cache()
            self.stats["prefill_oom_splits"] = self.stats.get("prefill_oom_splits", 0) + 1
            log.warning("interleaved prefill pass of %d slices ran out of device memory: retrying with %d",
                        len(part), len(part) // 2)
            return self._interleaved_pass(prefilling, active, max_parts=len(part) // 2)
        self.stats["prefill_tokens"] += tokens
        self.stats["prefill_slices"] = self.stats.get("prefill_slices", 0) + len(part)
        for s in part:
            s.spans.pop(0)
        done = [s for s, f in zip(part, final) if f]
        if done:
            for s in done:  # consecutive decode slots after the running rows
                s.slot = len(active)
                self._setup_slot(s, self.pf_tables[s.pf_slot])
                active.append(s)
                prefilling.remove(s)
            self._sample_first(done, logits)
            if self._on_prefill is not None:
                self._on_prefill(done)
        self._sync()
        dt = time.perf_counter() - t0
        self.stats["prefill_s"] += dt
        self.stats["interleaved_pass_max_s"] = max(self.stats.get("interleaved_pass_max_s", 0.0), dt)

    def _install(self, s: _Seq) -> None:
        """Copy an imported prefill's KV into ``s``'s pages and set its slot as the sampler would have."""
        st, imp = self.state, s.imported
        n = len(s.prompt)
        npg = self.kv.pages_for(n)
        if imp.kv is not None:
            if tuple(imp.kv.shape) != self.import_shape(n) or imp.kv.dtype != self.kv.k.dtype:
                raise ValueError("imported KV has shape %s %s" % (tuple(imp.kv.shape), imp.kv.dtype))
            idx = torch.tensor(s.pages[:npg], dtype=torch.long, device=self.device)
            kv = imp.kv.to(self.device, non_blocking=True)
            self.kv.k.index_copy_(1, idx, kv[0])
            self.kv.v.index_copy_(1, idx, kv[1])
        i = s.slot
        st.out_tokens[i, 0] = int(imp.first_token)
        st.next_ids[i] = int(imp.first_token)
        st.gen_count[i] = 1
        st.positions[i] = n
        st.done[i] = 0
        s.imported = None  # release the staging buffer
        self.stats["imported_prefills"] = self.stats.get("imported_prefills", 0) + 1

    def _prefill_isolated(self, batch: List[_Seq]) -> None:
        """Prefill ``batch``; on a device out-of-memory error (activations of a long packed batch), retry
        it as two halves, down to single sequences (SURVEY §5.3 failure isolation).  TP engines never
        split: their ranks must issue the same collectives."""
        try:
            self._prefill(batch)  # allocation failures raise here, at enqueue time: no sync needed
        except torch.OutOfMemoryError:
            if len(batch) == 1 or self.model.tp_size > 1:
                raise
            torch.cuda.empty_cache()
            self.stats["prefill_oom_splits"] = self.stats.get("prefill_oom_splits", 0) + 1
            log.warning("prefill of %d sequences ran out of device memory: retrying as two halves", len(batch))
            half = len(batch) // 2
            self._prefill_isolated(batch[:half])
            self._prefill_isolated(batch[half:])

    def _run_prefill(self, batch: List[_Seq], active: List[_Seq]) -> None:
        self._prefill_isolated(batch)  # enqueued; _admit synchronises once after its last batch
        active.extend(batch)
        if self._on_prefill is not None:
            self._on_prefill(batch)

    # ------------------------------------------------------------------ disaggregated prefill
    def prefill_export(self, prompts: Sequence[Sequence[int]], params: Sequence[SamplingParams], groups: int,
                       ignore_eos: bool = False):
        """Prefill ``prompts`` here (full model, all KV heads) and hand them to a TP=``groups`` engine.

        Returns ``(first_tokens, packs)``: the first sampled token of every prompt and, per TP rank
        g, one flat bf16 tensor holding -- prompt after prompt -- the K pages then the V pages of
        KV heads [g * Hkv / groups, (g + 1) * Hkv / groups): [2, n_layers, ceil(len / page),
        Hkv / groups, page, head_dim] each, the layout ImportedPrefill expects.  The pages here are
        released when this returns.  (Used by the provider: DP prefill, all-to-all, TP decode.)"""
        if self.model.tp_size != 1 or self.model.hkv % groups:
            raise ValueError("prefill_export needs a TP=1 engine and Hkv divisible by %d" % groups)
        hl = self.model.hkv // groups
        chunks: Dict[int, List[List[torch.Tensor]]] = {}

        def grab(seqs):
            for s in seqs:
                npg = self.kv.pages_for(len(s.prompt))
                idx = torch.tensor(s.pages[:npg], dtype=torch.long, device=self.device)
                k = self.kv.k.index_select(1, idx)  # [L, npg, Hkv, P, D]
                v = self.kv.v.index_select(1, idx)
                chunks[s.rid] = [torch.stack([k[:, :, g * hl:(g + 1) * hl], v[:, :, g * hl:(g + 1) * hl]])
                                 .reshape(-1) for g in range(groups)]

        one = [SamplingParams(1, p.temperature, p.seed) for p in params]
        outs = self.generate(prompts, one, ignore_eos=ignore_eos, on_prefill=grab)
        firsts = [o.token_ids[0] for o in outs]
        packs = [torch.cat([chunks[i][g] for i in range(len(prompts))]) if prompts else
                 torch.empty(0, dtype=self.kv.k.dtype, device=self.device) for g in range(groups)]
        return firsts, packs

    @staticmethod
    def cp_slices(n: int, world: int) -> List[List[Tuple[int, int]]]:
        """Zigzag context-parallel split of an ``n``-token prompt: 2 x world near-equal chunks, rank r
        takes chunks r and 2 world - 1 - r, so every rank gets one early (cheap causal attention) and one
        late (expensive) chunk -- balanced attention work; rank 0 holds the prompt's last token."""
        b = [round(k * n / (2 * world)) for k in range(2 * world + 1)]
        return [[(b[r], b[r + 1]), (b[2 * world - 1 - r], b[2 * world - r])] for r in range(world)]

    def cp_preflight(self, prompt: Sequence[int], world: int) -> Optional[str]:
        """Why prefill_export_cp cannot run here (None: it can) -- checked and agreed on by every rank
        before the collective part starts."""
        try:
            self._new_seq(0, prompt, SamplingParams(1))
        except ValueError as e:
            return str(e)
        if self.model.tp_size != 1 or self.model.hkv % world:
            return "needs a TP=1 engine and Hkv divisible by %d" % world
        if self.kv.fp8:
            return "the fp8 KV cache has no context-parallel K/V exchange"
        if len(prompt) < 2 * world:
            return "prompt of %d tokens is too short for %d ranks" % (len(prompt), world)
        if self.kv.pages_for(len(prompt) + 1) > self.kv.alloc.available():
            return "KV cache too small for %d tokens" % len(prompt)
        return None

    def prefill_export_cp(self, prompt: Sequence[int], params: SamplingParams, rank: int, world: int, group=None):
        """Context-parallel prefill of ONE prompt over the ``world`` ranks of ``group`` (every rank calls
        this with the same prompt on its full, TP=1 engine) for a TP=``world`` decode.

        Each rank runs its zigzag slices (``cp_slices``) through all layers (model.prefill_cp); after each
        layer's QKV stage the slices' K/V rows are all-gathered into every rank's paged cache, so the
        slices' attention sees the whole prefix and, at the end, every rank holds the prompt's full KV.
        Compute per rank is 1 / world of the prompt; the only traffic is each layer's K/V (128 KiB/token
        over the whole Llama-3-8B stack, vs 2 x 32 x 8 KiB of activation all-reduces per token for a TP
        forward), and no all-to-all is needed afterwards: each rank keeps the KV heads its TP shard owns.
        Returns ``(first_token, kv)`` with kv [2, n_layers, pages, Hkv / world, page, head_dim] (this
        rank's heads), the ImportedPrefill layout of the TP engine."""
        import torch.distributed as dist
        if self.model.tp_size != 1 or self.model.hkv % world or self.kv.fp8:
            raise ValueError("prefill_export_cp needs a TP=1 bf16-KV engine and Hkv divisible by %d" % world)
        s = self._new_seq(0, prompt, SamplingParams(1, params.temperature, params.seed))
        n = len(s.prompt)
        if n < 2 * world:
            raise ValueError("prompt of %d tokens is too short for context parallelism over %d ranks" % (n, world))
        st, dev, P = self.state, self.device, self.page
        need = self.kv.pages_for(n + 1)
        if need > self.kv.alloc.available():
            raise MemoryError("context-parallel prefill: KV cache too small for %d tokens" % n)
        s.pages = self.kv.alloc.alloc(need)
        s.slot = 0
        try:
            row = torch.zeros(self.max_pages, dtype=torch.int32)
            row[:need] = torch.tensor(s.pages, dtype=torch.int32)
            st.block_tables[0].copy_(row.to(dev, non_blocking=True))
            st.max_new[0], st.gen_count[0], st.done[0], st.result[0] = 1, 0, 0, 0
            st.temps[0], st.seeds[0] = float(params.temperature), int(params.seed)
            slices = self.cp_slices(n, world)
            mine = [(b, e) for b, e in slices[rank] if e > b]
            if len(mine) != len(slices[rank]):  # n >= 2 world: every zigzag chunk holds a token
                raise ValueError("context-parallel prefill: empty slice for %d tokens over %d ranks" % (n, world))
            passes = [self._pass_inputs([s], [span], paged=True) for span in mine]
            exchange = _CPExchange(self, s.pages, slices, rank, world, group)
            t0 = time.perf_counter()
            last = next((k for k, (b, e) in enumerate(mine) if e == n), None)
            logits = self.model.prefill_cp(passes, st.block_tables, self.kv.k, self.kv.v, exchange, logits_pass=last)
            self.stats["prefill_tokens"] += sum(e - b for b, e in mine)
            self.stats["cp_prefills"] = self.stats.get("cp_prefills", 0) + 1
            tok = 0
            if logits is not None:
                self._sample_first([s], logits)
                tok = int(st.next_ids[0].item())
            toks = [0] * world
            if exchange.nccl:
                t = torch.tensor([tok], dtype=torch.int64, device=dev)
                out = [torch.empty_like(t) for _ in range(world)]
                dist.all_gather(out, t, group=group)
                toks = [int(x.item()) for x in out]
            else:
                dist.all_gather_object(toks, tok, group=group)
            owner = next(q for q in range(world) if any(e == n for _, e in slices[q]))
            first = toks[owner]
            hl = self.model.hkv // world
            npg = self.kv.pages_for(n)
            pidx = torch.tensor(s.pages[:npg], dtype=torch.long, device=dev)
            k = self.kv.k.index_select(1, pidx)[:, :, rank * hl:(rank + 1) * hl]
            v = self.kv.v.index_select(1, pidx)[:, :, rank * hl:(rank + 1) * hl]
            kv = torch.stack([k, v]).contiguous()
            self._sync()
            self.stats["prefill_s"] += time.perf_counter() - t0
            return first, kv
        finally:
            self.kv.alloc.free(s.pages)
            st.park_row(0)  # slot 0 was borrowed: idle again (stopped, pages -> scratch page 0)

    def import_shape(self, prompt_len: int):
        """Shape of this engine's ImportedPrefill.kv for a prompt of ``prompt_len`` tokens (its cache layout:
        [.., hkv, page, head_dim] bf16 or [.., hkv, slab bytes] fp8)."""
        return (2, self.cfg.n_layers, self.kv.pages_for(prompt_len)) + tuple(self.kv.k.shape[2:])

    def _compact(self, active: List[_Seq], fin: set) -> None:
        st = self.state
        keep = [s for i, s in enumerate(active) if i not in fin]
        n_old = len(active)
        for new_slot, s in enumerate(keep):
            if s.slot != new_slot:
                st.move_row(s.slot, new_slot)
                s.slot = new_slot
        for i in range(len(keep), n_old):
            st.park_row(i)
        active[:] = keep

    def engine_stats(self) -> Dict[str, float]:
        s = dict(self.stats)
        s["prefill_tok_s"] = s["prefill_tokens"] / s["prefill_s"] if s["prefill_s"] else 0.0
        s["decode_tok_s"] = s["decode_tokens"] / s["decode_s"] if s["decode_s"] else 0.0
        s["kv_pages"] = self.kv.num_pages
        s["kv_dtype"] = self.kv.kv_dtype
        s["weights_gib"] = self.model.weight_bytes() / 2 ** 30
        if self.device.type == "cuda":
            s["hbm_peak_gib"] = torch.cuda.max_memory_allocated(self.device) / 2 ** 30
        if self.model.tp_size > 1:
            ar = self.model.custom_ar
            s["p2p_selftest"] = ar.selftest_report() if ar is not None else "off (RCCL)"
            s["custom_ar_recoveries"] = int(self.stats.get("custom_ar_recoveries", 0))
        return s
