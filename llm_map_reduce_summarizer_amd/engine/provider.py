"""``local`` provider: the MI355X engine behind the executor / aggregator.

Replaces the reference's per-chunk HTTPS calls (``llm_executor.py:250-409``;
aggregator ``result_aggregator.py:222-253``) with ONE batched generate per
stage, data-parallel over the ranks of the job:

1. every rank holds the same request list (the CPU front-end is
   deterministic and SPMD);
2. requests are assigned to DP replicas by a greedy longest-processing-time
   balance on (prompt + max_new) tokens -- no communication needed;
3. each replica runs its share through its own engine (continuous batching:
   every request of the replica is in flight at once);
4. results (text + token counts) are all-gathered over RCCL
   (``parallel.dist.all_gather_json``) so every rank ends the stage with
   every summary, in request order.

Sampling seeds are derived from the request content, so a summary does not
depend on which rank produced it or how the batch was formed.

Failures are collective-safe: an engine error on one rank is caught there,
the rank still enters the stage's all-gather (with error records for its
requests), and every rank ends the stage with the SAME results -- so the
executor's retry loop (reference ``llm_executor.py:196-228``) retries the same
requests on every rank, re-balanced over the replicas (a request that failed
on a sick replica may land on a healthy one).  TP stages agree on an ok/error
vector before and after the sharded generate.  ``MRSUM_FAULT_INJECT=
"rank:count"`` (or ``fault_inject=``) raises in the engine call of ``rank``
for its first ``count`` calls (-1: every call) -- the test hook.

With several GPUs a stage may instead run on engines sharded over groups of
k consecutive GPUs (TP = k, world / k such replicas; k = world is one engine
over the whole node): decode is bound by streaming weights + KV from HBM,
which DP replicas do not shorten and TP divides.  ``parallel`` selects the
policy: ``dp`` (every stage data-parallel), ``reduce_tp`` (map DP, reduce
stages TP = world), ``tp`` (every stage TP = world), ``tpK`` (every stage
TP = K x DP = world / K), an explicit per-stage layout such as
``map:tp2,reduce_l1:tp4,reduce_final:tp8`` (``reduce`` matches every reduce
stage, unnamed stages stay DP), or ``auto`` (per stage, the cheapest TP degree
among the divisors of the world size under the cost model of
``parallel/plan.py``, fed with the all-reduce latency and bandwidth measured
on this job's GPUs at start-up).
"""

from __future__ import annotations

import hashlib
import json
import logging
import math
import os
import time
from typing import Any, Dict, List, Optional, Sequence

from ..config import LLMConfig
from ..parallel import dist as pdist
from ..pipeline.providers import GenRequest, GenResult, Provider
from .chat import render_chat, render_messages
from .tokenizer import get_tokenizer

log = logging.getLogger("mrsum.local")


def _req_seed(base: int, req: GenRequest) -> int:
    key = "%d|%s|%s" % (base, req.system or "", req.user)
    if req.messages:
        key += "|" + json.dumps(req.messages, sort_keys=True)
    h = hashlib.sha1(key.encode("utf-8")).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 62) - 1)


def parse_parallel(spec: str, world: int) -> Dict[str, int]:
    """Stage -> TP degree of an explicit layout: ``tpK`` (every stage, key ``*``) or comma-separated
    ``stage:tpK`` / ``stage:dp`` items (``reduce`` = every reduce stage).  Degrees must divide ``world``."""
    out: Dict[str, int] = {}
    items = [spec] if ":" not in spec else spec.split(",")
    for it in items:
        stage, _, lay = it.strip().rpartition(":")
        lay = lay.strip().lower()
        if lay == "dp":
            k = 1
        elif lay.startswith("tp") and lay[2:].isdigit():
            k = int(lay[2:])
        else:
            raise ValueError("bad parallel layout %r (want dp, tpK or stage:tpK,...)" % it)
        if k < 1 or world % k:
            raise ValueError("TP degree %d does not divide the world size %d" % (k, world))
        out[stage.strip() or "*"] = k
    return out


def divisors(n: int) -> List[int]:
    return [k for k in range(1, n + 1) if n % k == 0]


def assign_balanced(costs: Sequence[int], n_bins: int) -> List[int]:
    """Greedy LPT: returns bin index per item; deterministic."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0] * n_bins
    out = [0] * len(costs)
    for i in order:
        b = min(range(n_bins), key=lambda j: (load[j], j))
        out[i] = b
        load[b] += costs[i]
    return out


class LocalEngineProvider(Provider):
    name = "local"
    batched = True

    def __init__(self, model: str = "llama3-8b", config: Optional[LLMConfig] = None, device: Optional[str] = None,
                 tp: int = 1, seed: Optional[int] = None, max_model_len: Optional[int] = None, engine=None,
                 engine_options: Optional[Dict[str, Any]] = None, dtype: Optional[str] = None,
                 kv_fraction: Optional[float] = None, use_graphs: bool = True, max_num_seqs: Optional[int] = None,
                 tokenizer: Optional[str] = None, ignore_eos: bool = False, reduce_tp: Optional[bool] = None,
                 weights: Optional[str] = None, parallel: Optional[str] = None,
                 fault_inject: Optional[str] = None, kv_dtype: Optional[str] = None, **_ignored):
        super().__init__(model, config)
        spec = fault_inject or os.environ.get("MRSUM_FAULT_INJECT", "")
        self._fault_rank, self._fault_left = (int(x) for x in spec.split(":")) if spec else (-1, 0)
        self.tokenizer = get_tokenizer(tokenizer)
        if dtype not in (None, "bf16", "fp8"):
            raise ValueError("dtype must be bf16 or fp8, got %s" % dtype)
        self.tp = tp
        self.ignore_eos = ignore_eos
        self.seed = self.config.ENGINE_SEED if seed is None else seed
        self._engine = engine
        self._device = device
        self._engine_options = dict(engine_options or {})
        self._engine_options.setdefault("use_graphs", use_graphs)
        if weights:  # HF safetensors checkpoint (engine/weights.py); else seeded random init
            self._engine_options.setdefault("weights_path", weights)
        # context budget: 32k for the Llama-3 presets (map prompts ~4k, reduce prompts <= ~12k), the
        # model's full window for long-context models (Llama-3.1: 128k, a single-pass reduce of a day)
        if max_model_len is None:
            try:
                mp = self.model_config().max_position
            except Exception:  # noqa: BLE001 -- unknown model: the engine reports it when built
                mp = 32768
            max_model_len = mp if mp > 40960 else min(mp, 32768)
        self.max_model_len = max_model_len
        if dtype == "fp8":
            self._engine_options.setdefault("weight_dtype", "fp8")
        if kv_fraction is not None:
            self._engine_options.setdefault("kv_fraction", kv_fraction)
        kv_dtype = kv_dtype or self.config.ENGINE_KV_DTYPE
        if kv_dtype not in ("bf16", "fp8v"):
            # fp8 K + V (the engine's "fp8" format) is not offered: 13-22 % logit error on the parity checkpoint
            # (tests/test_forward_parity_gpu.py), above the 0.15 a variant must meet; fp8v is 8 %
            raise ValueError("kv_dtype must be bf16 or fp8v, got %s" % kv_dtype)
        self._engine_options.setdefault("kv_dtype", kv_dtype)
        if max_num_seqs is not None:
            self._engine_options.setdefault("max_num_seqs", max_num_seqs)
        self.timings: Dict[str, float] = {"generate_s": 0.0, "allgather_s": 0.0}
        # work actually done, from the all-gathered results (identical on every rank): bench.py checks that
        # a pinned run generated exactly its requested tokens (no generation cut short inside the timed work)
        self.work: Dict[str, int] = {"requests": 0, "errors": 0, "completion_tokens": 0, "requested_tokens": 0}
        self.par = pdist.setup_parallel(tp)
        # parallel policy (module docstring); the legacy reduce_tp flag maps onto it
        if parallel is None:
            parallel = os.environ.get("MRSUM_PARALLEL") or {None: "auto", True: "reduce_tp", False: "dp"}[reduce_tp]
        self.fixed_tp: Dict[str, int] = {}
        if parallel not in ("auto", "dp", "reduce_tp", "tp"):
            self.fixed_tp = parse_parallel(parallel, max(1, self.par.world))
            bad = [k for k in self.fixed_tp.values() if k > 1 and not self._tp_ok(k)]
            if bad:
                raise ValueError("%s does not shard over TP=%d" % (self.model, bad[0]))
            parallel = "fixed"
        import torch
        multi = self.par.world > 1 and tp == 1 and (self._tp_ok(self.par.world) or parallel == "fixed")
        if parallel == "auto" and not torch.cuda.is_available():
            parallel = "dp"  # the planner's constants are GPU measurements
        if parallel == "fixed" and all(k == 1 for k in self.fixed_tp.values()):
            parallel = "dp"
        self.parallel = parallel if multi else "dp"
        self.use_tp_engine = self.parallel != "dp"  # a TP engine exists for some stage
        self._tp_engines: Dict[int, Any] = {}  # TP degree -> this rank's engine of its k-rank group
        self._tp_bad: set = set()  # degrees whose engine had no graph-safe all-reduce
        self._dp_needed = self.parallel != "tp"
        self.hw = None  # plan.HWModel with this job's measured all-reduce constants (auto mode)
        # TP stages prefill data-parallel on the TP=1 engines and move the KV with one all-to-all
        self.handoff = self.use_tp_engine and os.environ.get("MRSUM_HANDOFF", "1") == "1"
        if self.handoff:
            self._dp_needed = True
        self.stage_plan: Dict[str, Any] = {}
        # per stage: the planner's predicted seconds (parallel/plan.py stage_seconds at the layout the stage
        # ran) next to the measured wall time of its generate calls -- the record that makes the first real
        # multi-GPU run diagnosable (which stage missed its model, by how much)
        self.stage_seconds: Dict[str, Dict[str, Any]] = {}
        # TP degree -> the cross-GPU cost of one decode all-reduce per path, measured when its engine is built
        self.p2p_latency: Dict[str, Dict[str, float]] = {}
        self.owner_maps: Dict[str, List[List[int]]] = {}  # stage -> replica of every request, per call
        if self.use_tp_engine:
            self._engine_options.setdefault("kv_fraction", float(os.environ.get("MRSUM_DP_KV_FRACTION", "0.5")))

    def _tp_ok(self, k: int) -> bool:
        """The model shards over TP=k (heads, KV heads, FFN and vocab divisible; at most 8 GPUs)."""
        if k <= 1 or k > 8 or self.par.world % k:
            return False
        try:
            c = self.model_config()
        except Exception:
            return False
        return c.n_kv_heads % k == 0 and c.n_heads % k == 0 and c.ffn % k == 0 and c.vocab_size % k == 0

    # ------------------------------------------------------------------ engine
    def model_config(self):
        """Preset by name, or the checkpoint's config.json when weights are given and the name is
        not a preset (e.g. ``--model hf --weights /ckpt``)."""
        from .config import PRESETS, get_model_config
        wp = self._engine_options.get("weights_path")
        if wp and self.model.lower() not in PRESETS:
            from .weights import config_from_hf
            return config_from_hf(wp, self.model)
        return get_model_config(self.model)

    @property
    def engine(self):
        if self._engine is None:
            import torch
            from .config import get_model_config
            from .engine import LLMEngine
            if self._device is None:
                self._device = ("cuda:%d" % (self.par.local_rank % max(1, torch.cuda.device_count()))
                                if torch.cuda.is_available() else "cpu")
            opts = dict(max_model_len=self.max_model_len, max_num_seqs=self.config.ENGINE_MAX_NUM_SEQS,
                        kv_fraction=self.config.ENGINE_KV_FRACTION, eos_ids=self.tokenizer.eos_ids)
            opts.update(self._engine_options)
            self._engine = LLMEngine(self.model_config(), device=self._device, seed=self.seed,
                                     tp_rank=self.par.tp_rank, tp_size=self.par.tp, tp_group=self.par.tp_group,
                                     **opts)
            log.info("local engine up: %s on %s (tp=%d, dp=%d) in %.1f s", self.model, self._device, self.par.tp,
                     self.par.dp, self._engine.init_seconds)
        return self._engine

    @property
    def tp_engine(self):
        """TP=world engine of the same model/seed (the ``tp`` engine of the module docstring)."""
        return self.tp_engine_for(self.par.world)

    @property
    def _tp_engine(self):
        return self._tp_engines.get(self.par.world)

    def tp_engine_for(self, k: int):
        """This rank's engine of its TP=``k`` group (ranks [k * (rank // k), k * (rank // k + 1))), built
        on first use -- collectively: every rank asks for the same degree at the same point of the
        pipeline.  None when that degree had no graph-safe all-reduce (the stage then stays DP)."""
        if k in self._tp_bad:
            return None
        eng = self._tp_engines.get(k)
        if eng is None:
            import torch
            from .engine import LLMEngine
            world = self.par.world
            opts = dict(self._engine_options)
            frac = "0.6" if self.parallel == "tp" else "0.35"  # leave HBM for the DP engine
            if k < world:
                frac = "0.25"  # one more engine beside the DP / TP=world ones
            opts.update(max_model_len=self.max_model_len, max_num_seqs=self.config.ENGINE_MAX_NUM_SEQS,
                        kv_fraction=float(os.environ.get("MRSUM_REDUCE_KV_FRACTION", frac)),
                        eos_ids=self.tokenizer.eos_ids)
            if self._device is None:
                self._device = ("cuda:%d" % (self.par.local_rank % max(1, torch.cuda.device_count()))
                                if torch.cuda.is_available() else "cpu")
            eng = LLMEngine(self.model_config(), device=self._device, seed=self.seed,
                            tp_rank=self.par.rank % k, tp_size=k, tp_group=pdist.tp_group_for(k), **opts)
            log.info("TP engine up: %s TP=%d (x DP=%d)", self.model, k, world // k)
            if eng.model.custom_ar is None and torch.cuda.is_available() \
                    and self.parallel in ("auto", "reduce_tp", "fixed"):
                # every rank built the same engine and got the same collective verdict: drop it (its
                # decode could not run in hipGraphs) and run the stages that wanted it data-parallel
                log.warning("no P2P all-reduce for the TP=%d engine: its stages stay data-parallel", k)
                self._tp_bad.add(k)
                del eng
                torch.cuda.empty_cache()
                if k == world and self.parallel in ("auto", "reduce_tp"):
                    self.parallel, self.use_tp_engine, self._dp_needed = "dp", False, True
                return None
            self._tp_engines[k] = eng
            self._measure_p2p(k, eng)
        return eng

    def _measure_p2p(self, k: int, eng) -> None:
        """COLLECTIVE within the TP=k group (every rank builds the engine at the same point): the cross-GPU
        cost of one decode all-reduce on each path the decode can take -- the TP push of the down projection's
        shard (the path it runs) and the fused all-reduce + add + RMSNorm (its fallback) -- as a + b x rows
        over the same kernel on a group of one (CustomAllReduce.measure_latency).  Recorded per degree for the
        bench JSON; MRSUM_P2P_LATENCY=0 skips it."""
        ar = eng.model.custom_ar
        if ar is None or os.environ.get("MRSUM_P2P_LATENCY", "1") != "1":
            return
        m = eng.model
        rec: Dict[str, float] = {}
        try:
            for path, push_k in (("push", m.ffn_local), ("fused", None)):
                if path == "push" and not ar.paths.get("push_stream"):
                    continue
                lat, per_row = ar.measure_latency(rows=(1, 64), hidden=eng.cfg.hidden, push_k=push_k,
                                                  fp8=m.weight_dtype == "fp8")
                rec[path + "_us"] = round(lat * 1e6, 2)
                rec[path + "_us_per_row"] = round(per_row * 1e6, 4)
        except Exception as e:  # noqa: BLE001 -- a diagnostic: never fail the job on it
            log.warning("P2P latency probe of the TP=%d engine failed: %s", k, e)
            rec["error"] = str(e)[:200]
        self.p2p_latency["tp%d" % k] = rec
        log.info("TP=%d decode all-reduce, cross-GPU part: %s", k, rec)

    def _predict_stage(self, prompts, reqs, tp: int, handoff: bool) -> Optional[float]:
        """The planner's estimate (seconds) of this generate at TP degree ``tp`` over this job's ranks."""
        try:
            from ..parallel import plan
            d = plan.ModelDims.of(self.model_config(),
                                  1.0 if self._engine_options.get("weight_dtype") == "fp8" else 2.0)
            hw = self.hw or plan.HWModel()
            world = max(1, self.par.world)
            if self.par.tp > 1:  # DP replicas of a TP engine
                tp = self.par.tp
            return plan.stage_seconds(d, hw, [len(p) for p in prompts], [r.max_tokens for r in reqs], tp, world,
                                      handoff)
        except Exception as e:  # noqa: BLE001 -- a diagnostic
            log.debug("stage prediction failed: %s", e)
            return None

    def _record_stage(self, stage: str, tp: int, predicted: Optional[float], measured: float) -> None:
        rec = self.stage_seconds.setdefault(stage, {"tp": tp, "calls": 0, "predicted_s": 0.0, "measured_s": 0.0})
        rec["calls"] += 1
        rec["tp"] = tp
        rec["measured_s"] = round(rec["measured_s"] + measured, 6)
        if predicted is None or rec["predicted_s"] is None:
            rec["predicted_s"] = None
        else:
            rec["predicted_s"] = round(rec["predicted_s"] + predicted, 7)

    def warm(self, capture_batch: Optional[int] = None) -> None:
        """Build the engines (and measure the planner's constants) outside any timed region; with
        ``capture_batch``, also capture the decode graphs of every batch bucket up to it."""
        if self.parallel == "fixed":
            for k in sorted({k for k in self.fixed_tp.values() if k > 1}, reverse=True):
                eng = self.tp_engine_for(k)
                if capture_batch and eng is not None:
                    eng.capture_graphs(-(-capture_batch // (self.par.world // k)))
        elif self.use_tp_engine:
            _ = self.tp_engine
            if self.parallel == "auto":
                self._measure()
            if capture_batch and self.use_tp_engine:
                self._tp_engine.capture_graphs(capture_batch)
        if self._dp_needed:
            _ = self.engine
            if capture_batch and self.parallel in ("dp", "auto", "reduce_tp", "fixed"):
                self._engine.capture_graphs(-(-capture_batch // self.par.dp))

    def _measure(self):
        """plan.HWModel with the all-reduce latency / bandwidth of THIS job's GPUs (auto mode)."""
        if self.hw is None:
            import torch
            from ..parallel import plan
            hw = plan.HWModel()
            eng = self.tp_engine
            ar = eng.model.custom_ar if eng is not None else None
            if ar is None or self.parallel != "auto":
                self.hw = plan.with_measurements(hw, tp_ok=ar is not None)
                return self.hw
            m = eng.model
            # the cross-GPU cost of the decode's own all-reduce: the TP push of the down projection's shard
            # (measured when the engine was built, _measure_p2p; again here if that probe was skipped)
            rec = self.p2p_latency.get("tp%d" % self.par.world, {})
            key = "push" if "push_us" in rec else ("fused" if "fused_us" in rec else None)
            if key is not None:
                lat, per_row = rec[key + "_us"] * 1e-6, rec[key + "_us_per_row"] * 1e-6
            else:
                lat, per_row = ar.measure_latency(rows=(1, 64), hidden=eng.cfg.hidden, push_k=m.ffn_local,
                                                  fp8=m.weight_dtype == "fp8")
            bw = _rccl_bandwidth(eng.model.tp_group, eng.cfg.hidden, torch.device(self._device))
            self.hw = plan.with_measurements(hw, ar_lat_s=lat, ar_lat_row_s=per_row, ar_bw=bw, tp_ok=True)
            log.info("planner constants: all-reduce %.1f us + %.3f us/row (%s path, over the same kernel on a "
                     "group of one), RCCL all-reduce %.1f GB/s", lat * 1e6, per_row * 1e6,
                     getattr(ar, "latency_path", "fused"), bw / 1e9)
        return self.hw

    def _fixed_degree(self, stage: str) -> int:
        f = self.fixed_tp
        if stage in f:
            return f[stage]
        if stage.startswith("reduce") and "reduce" in f:
            return f["reduce"]
        return f.get("*", 1)

    def _stage_tp(self, stage: str, prompts: Sequence[Sequence[int]], reqs: Sequence[GenRequest]):
        """(TP degree k, disaggregated prefill?) for this stage's generate: 1 = DP replicas, k > 1 =
        world / k replicas of a TP=k engine (world: one engine sharded over every GPU)."""
        world = self.par.world
        if self.parallel == "fixed":
            k = self._fixed_degree(stage) if reqs else 1
            if k > 1 and self.tp_engine_for(k) is None:
                k = 1
            self.stage_plan[stage] = {"tp": k, "handoff": bool(k > 1 and self._handoff_pays(prompts, reqs, k))}
            return k, self.stage_plan[stage]["handoff"]
        if self.parallel != "dp":
            _ = self.tp_engine  # may fall back to dp (no P2P all-reduce on this node)
        if self.parallel == "dp" or not reqs:
            return 1, False
        if self.parallel in ("tp", "reduce_tp"):
            if self.parallel == "reduce_tp" and stage == "map":
                return 1, False
            return world, self._handoff_pays(prompts, reqs)
        from ..parallel import plan
        hw = self._measure()
        if self.parallel != "auto":  # _measure found no P2P all-reduce and fell back to dp
            return 1, False
        d = plan.ModelDims.of(self.model_config(),
                              1.0 if self._engine_options.get("weight_dtype") == "fp8" else 2.0)
        cands = [k for k in divisors(world) if k == 1 or (self._tp_ok(k) and k not in self._tp_bad)]
        choice = plan.choose(d, hw, [len(p) for p in prompts], [r.max_tokens for r in reqs], world,
                             candidates=cands, handoff=self.handoff)
        k = int(choice["tp"])
        if k > 1 and self.tp_engine_for(k) is None:  # that degree has no graph-safe all-reduce
            k = 1
            choice = dict(choice, tp=1)
        self.stage_plan[stage] = choice
        return k, bool(choice.get("handoff", False))

    def _handoff_pays(self, prompts, reqs, k: Optional[int] = None) -> bool:
        """Disaggregated prefill for a TP=k stage (default k = world) when the cost model says it beats
        the TP forward: always for many prompts (each rank of the group prefills its share, no activation
        all-reduces); for ONE prompt (the final reduce) it weighs the context-parallel prefill over the
        group against the TP forward's 2 x n_layers RCCL all-reduces of the activations
        (parallel/plan.py)."""
        if not self.handoff or not reqs:
            return False
        if len(reqs) > 1:
            return True
        k = k or self.par.world
        from ..parallel import plan
        d = plan.ModelDims.of(self.model_config(), 1.0 if self._engine_options.get("weight_dtype") == "fp8" else 2.0)
        hw = self.hw or plan.HWModel()
        lens = [len(p) for p in prompts]
        return plan.handoff_prefill_s(d, hw, lens, k) < plan.prefill_s(d, hw, sum(lens), k, max(lens))

    def _handoff(self, prompts: Sequence[Sequence[int]], sp, k: Optional[int] = None) -> Dict[int, Any]:
        """Disaggregated prefill for a TP stage: every rank prefills its LPT share of the prompts on
        its full (TP=1) engine -- no activation all-reduces -- and ships each prompt's KV heads to the
        TP rank that owns them in ONE all-to-all (RCCL over xGMI: ~prompt tokens x 128 KiB x
        (world-1)/world per Llama-3-8B prompt); first tokens are all-gathered.  Returns the
        ImportedPrefill map for the TP engine's generate -- or None when the single-prompt context-parallel
        prefill cannot run here (every rank's pre-flight verdict, agreed: a prompt too short for the group,
        an fp8 KV cache, a DP engine whose KV pool cannot hold the prompt); the TP engine then prefills the
        prompt itself (a TP forward, nothing lost but the hand-off's speed)."""
        import torch
        import torch.distributed as dist

        from .engine import ImportedPrefill
        t0 = time.perf_counter()
        world = k or self.par.world  # the TP group: ranks [world * g, world * (g + 1))
        rank = self.par.rank % world
        group = pdist.tp_group_for(world)
        if len(prompts) == 1 and len(prompts[0]) >= 2 * world and not self.engine.kv.fp8:
            # one prompt (the final reduce): context-parallel prefill over every rank instead of one rank
            # prefilling it alone; every rank ends with its TP shard's KV heads, no all-to-all
            # (rank-local faults were agreed on by the caller; the pre-flight check makes the ranks agree
            # on their local resources BEFORE the per-layer all-gathers, which no rank may leave early)
            pre = self.engine.cp_preflight(prompts[0], world)
            errs = [x for x in pdist.all_gather_json(pre and "rank %d: %s" % (self.par.rank, pre), group) if x]
            if errs:  # every rank of the group saw the same verdicts: all fall back alike
                log.warning("context-parallel prefill not possible (%s): the TP engine prefills the prompt",
                            "; ".join(errs))
                self.timings["cp_fallbacks"] = self.timings.get("cp_fallbacks", 0) + 1
                return None
            first, kv = self.engine.prefill_export_cp(prompts[0], sp[0], rank, world, group=group)
            self.timings["handoff_s"] = self.timings.get("handoff_s", 0.0) + time.perf_counter() - t0
            self.timings["cp_prefills"] = self.timings.get("cp_prefills", 0) + 1
            return {0: ImportedPrefill(first, kv)}
        owner = assign_balanced([len(p) for p in prompts], world)
        mine = [i for i in range(len(prompts)) if owner[i] == rank]
        tp_eng = self.tp_engine_for(world)
        shapes = [tp_eng.import_shape(len(p)) for p in prompts]
        numel = [math.prod(s) for s in shapes]
        recv_sizes = [sum(numel[i] for i in range(len(prompts)) if owner[i] == s) for s in range(world)]
        nccl = dist.get_backend() == "nccl"
        err, oom = None, False
        try:
            self._maybe_fault()
            firsts, packs = self.engine.prefill_export([prompts[i] for i in mine], [sp[i] for i in mine], world,
                                                       ignore_eos=self.ignore_eos)
            send = torch.cat(packs) if packs else torch.empty(0, dtype=self.engine.kv.k.dtype)
            send_sizes = [p.numel() for p in packs]
        except Exception as e:  # noqa: BLE001 -- still enter the all-to-all with the sizes the peers expect
            oom = isinstance(e, MemoryError)
            err = "rank %d prefill: %s: %s" % (self.par.rank, type(e).__name__, e)
            log.error("%s", err)
            firsts = [0] * len(mine)
            send_sizes = [sum(numel[i] for i in mine)] * world
            send = torch.zeros(sum(send_sizes), dtype=self.engine.kv.k.dtype,
                               device=torch.device(self._device) if nccl else "cpu")
        dev = send.device if nccl else torch.device("cpu")
        send = send.to(dev)
        recv = torch.empty(sum(recv_sizes), dtype=send.dtype, device=dev)
        dist.all_to_all_single(recv, send, recv_sizes, send_sizes, group=group)
        tok, errs, ooms = {}, [], []
        for part in pdist.all_gather_json({"tok": {str(i): int(t) for i, t in zip(mine, firsts)}, "err": err,
                                           "oom": oom}, group):
            tok.update({int(k): v for k, v in part["tok"].items()})
            if part["err"]:
                errs.append(part["err"])
                ooms.append(bool(part.get("oom")))
        if errs and all(ooms):
            # only KV-pool exhaustion on the DP engines (their pools are sized for the DP stages, not for a TP
            # group's whole share): every rank of the group saw the same verdicts, so all fall back alike to the
            # TP engine's own prefill -- the hand-off's speed is lost, not the requests
            log.warning("disaggregated prefill does not fit the DP engines' KV pools (%s): the TP=%d engine "
                        "prefills the prompts", "; ".join(errs), world)
            self.timings["handoff_fallbacks"] = self.timings.get("handoff_fallbacks", 0) + 1
            return None
        if errs:  # every rank raises the same error: the stage fails as a whole, consistently
            raise RuntimeError("; ".join(errs))
        out, off = {}, 0
        for s in range(world):
            for i in range(len(prompts)):
                if owner[i] == s:
                    out[i] = ImportedPrefill(tok[i], recv[off:off + numel[i]].view(shapes[i]))
                    off += numel[i]
        self.timings["handoff_s"] = self.timings.get("handoff_s", 0.0) + time.perf_counter() - t0
        return out

    def encode_request(self, req: GenRequest) -> List[int]:
        ids = (render_messages(self.tokenizer, req.messages) if req.messages
               else render_chat(self.tokenizer, req.user, req.system))
        budget = self.max_model_len - max(1, req.max_tokens)
        if len(ids) > budget:
            log.warning("prompt of %d tokens truncated to %d (max_model_len %d)", len(ids), budget,
                        self.max_model_len)
            ids = ids[:budget - 5] + ids[-5:]  # keep the assistant header
        return ids

    # ------------------------------------------------------------------ API
    def _maybe_fault(self) -> None:
        """Test hook (MRSUM_FAULT_INJECT / fault_inject="rank:count"): raise on this rank's engine call."""
        if self._fault_left != 0 and self.par.rank == self._fault_rank:
            if self._fault_left > 0:
                self._fault_left -= 1
            raise RuntimeError("injected engine fault on rank %d" % self.par.rank)

    async def generate(self, req: GenRequest) -> GenResult:
        return (await self.generate_batch([req]))[0]

    def _tally(self, results: Sequence[Optional[GenResult]], max_tokens: Sequence[int]) -> None:
        for r, mt in zip(results, max_tokens):
            if r is None:
                continue
            self.work["requests"] += 1
            if r.error:
                self.work["errors"] += 1
                continue
            self.work["completion_tokens"] += int(r.completion_tokens)
            self.work["requested_tokens"] += int(mt)

    def _generate_tp_groups(self, prompts, reqs, k: int, sp, stage: str) -> List[GenResult]:
        """TP=k x DP=world/k: requests LPT-balanced over the world / k groups of k consecutive ranks, each
        group runs its share on its TP=k engine (disaggregated / context-parallel prefill inside the group
        when it pays), results all-gathered over the world (tp_rank 0 copies kept).  An engine error
        fails the requests of that group only, identically on every rank."""
        world, rank = self.par.world, self.par.rank
        owner = assign_balanced([len(p) + r.max_tokens for p, r in zip(prompts, reqs)], world // k)
        self.owner_maps.setdefault(stage, []).append(owner)
        mine = [i for i in range(len(reqs)) if owner[i] == rank // k]
        local: List[Dict[str, Any]] = []
        if mine:
            sub_p, sub_sp = [prompts[i] for i in mine], [sp[i] for i in mine]
            try:
                ho = self._handoff_pays(sub_p, [reqs[i] for i in mine], k)
                imported = self._handoff(sub_p, sub_sp, k) if ho else None
                outs = self.tp_engine_for(k).generate(sub_p, sub_sp, ignore_eos=self.ignore_eos, imported=imported)
                for i, o in zip(mine, outs):
                    local.append({"i": i, "text": self.tokenizer.decode(o.token_ids), "pt": o.prompt_len,
                                  "ct": len(o.token_ids), "fr": o.finish_reason})
            except Exception as e:  # noqa: BLE001 -- SPMD inside the group: its every rank raises alike
                msg = "rank %d: %s: %s" % (rank, type(e).__name__, e)
                log.error("TP=%d group %d failed on %d requests: %s", k, rank // k, len(mine), msg)
                local = [{"i": i, "err": msg} for i in mine]
        merged = {}
        for r, part in enumerate(pdist.all_gather_json(local)):
            if r % k == 0:
                for rec in part:
                    merged[rec["i"]] = rec
        return [_result(merged[i]) if i in merged else GenResult("", error="request %d produced no result" % i)
                for i in range(len(reqs))]

    def _generate_tp(self, prompts, reqs, handoff: bool, k: Optional[int] = None,
                     stage: str = "map") -> List[GenResult]:
        """TP=k engines over every request (default k = world: one engine, every rank runs every request);
        ranks agree on ok / error before and after, so a rank-local error (raised before the sharded
        forward) fails the stage on every rank alike."""
        from .engine import SamplingParams
        sp = [SamplingParams(r.max_tokens, r.temperature, _req_seed(self.seed, r)) for r in reqs]
        k = k or self.par.world
        err = None
        try:
            self._maybe_fault()  # (the TP engine itself was built by _stage_tp, collectively)
        except Exception as e:  # noqa: BLE001
            err = "rank %d: %s: %s" % (self.par.rank, type(e).__name__, e)
        errs = [x for x in pdist.all_gather_json(err) if x]
        if not errs and k < self.par.world:
            return self._generate_tp_groups(prompts, reqs, k, sp, stage)
        outs = None
        if not errs:
            try:
                imported = self._handoff(prompts, sp) if handoff else None
                outs = self.tp_engine.generate(prompts, sp, ignore_eos=self.ignore_eos, imported=imported)
            except Exception as e:  # noqa: BLE001 -- deterministic (SPMD) errors are raised on every rank
                err = "rank %d: %s: %s" % (self.par.rank, type(e).__name__, e)
            errs = [x for x in pdist.all_gather_json(err) if x]
        if errs:
            log.error("TP stage failed: %s", "; ".join(errs))
            return [GenResult("", error="; ".join(errs)) for _ in reqs]
        return [GenResult(self.tokenizer.decode(o.token_ids), o.prompt_len, len(o.token_ids), 0.0,
                          extra={"finish_reason": o.finish_reason}) for o in outs]

    async def generate_batch(self, reqs: Sequence[GenRequest]) -> List[GenResult]:
        from .engine import SamplingParams
        t0 = time.perf_counter()
        prompts = [self.encode_request(r) for r in reqs]
        stage = reqs[0].stage if reqs else "map"
        tp, handoff = self._stage_tp(stage, prompts, reqs) if self.par.world > 1 and self.tp == 1 else (1, False)
        self.stage_plan.setdefault(stage, {"tp": tp, "handoff": handoff})
        predicted = self._predict_stage(prompts, reqs, tp, handoff)
        if tp > 1:
            # TP=tp groups (tp = world: every rank runs every request); the TP ranks sample identically
            res = self._generate_tp(prompts, reqs, handoff, tp, stage)
            self.timings["generate_s"] += time.perf_counter() - t0
            self._record_stage(stage, tp, predicted, time.perf_counter() - t0)
            self._tally(res, [r.max_tokens for r in reqs])
            return res
        dp, dp_rank = self.par.dp, self.par.dp_rank
        owner = assign_balanced([len(p) + r.max_tokens for p, r in zip(prompts, reqs)], dp)
        self.owner_maps.setdefault(stage, []).append(owner)
        mine = [i for i in range(len(reqs)) if owner[i] == dp_rank]
        local: List[Dict[str, Any]] = []
        pre_err = None
        if self.par.tp > 1:
            # TP replicas: agree on local pre-checks first, so no TP rank of a replica enters the sharded
            # forward (all-reduces) while a peer of the same replica has already given up
            try:
                self._maybe_fault()
            except Exception as e:  # noqa: BLE001
                pre_err = "rank %d: %s: %s" % (self.par.rank, type(e).__name__, e)
            errs = pdist.all_gather_json(pre_err)
            g0 = dp_rank * self.par.tp
            pre_err = next((x for x in errs[g0:g0 + self.par.tp] if x), None)
        if mine and pre_err:
            local = [{"i": i, "err": pre_err} for i in mine]
        elif mine:
            try:
                if self.par.tp == 1:
                    self._maybe_fault()
                outs = self.engine.generate(
                    [prompts[i] for i in mine],
                    [SamplingParams(reqs[i].max_tokens, reqs[i].temperature, _req_seed(self.seed, reqs[i]))
                     for i in mine],
                    ignore_eos=self.ignore_eos)
                for i, o in zip(mine, outs):
                    local.append({"i": i, "text": self.tokenizer.decode(o.token_ids), "pt": o.prompt_len,
                                  "ct": len(o.token_ids), "fr": o.finish_reason})
            except Exception as e:  # noqa: BLE001 -- never skip the all-gather below: the peers are in it
                msg = "rank %d: %s: %s" % (self.par.rank, type(e).__name__, e)
                log.error("engine failed on %d requests: %s", len(mine), msg)
                local = [{"i": i, "err": msg} for i in mine]
        t1 = time.perf_counter()
        self.timings["generate_s"] += t1 - t0
        if pdist.is_initialized():  # also at world 1 under torchrun: same RCCL code path as N > 1
            gathered = pdist.all_gather_json(local)
            # with TP, every rank of a replica holds identical results: keep the tp_rank 0 copies
            merged = {}
            for rank, part in enumerate(gathered):
                if rank % self.par.tp == 0:
                    for r in part:
                        merged[r["i"]] = r
        else:
            merged = {r["i"]: r for r in local}
        self.timings["allgather_s"] += time.perf_counter() - t1
        self._record_stage(stage, self.par.tp, predicted, time.perf_counter() - t0)
        res = [_result(merged[i]) if i in merged else GenResult("", error="request %d produced no result" % i)
               for i in range(len(reqs))]
        self._tally(res, [r.max_tokens for r in reqs])
        return res

    async def generate_groups(self, reqs: Sequence[GenRequest], groups: Sequence[Sequence[int]], build):
        """Streamed two-stage generate (map -> level-1 reduce): ``groups`` partitions
        ``reqs``; as soon as every request of group g has finished, ``build(g, results)`` (results in
        group order) returns group g's follow-up request (or None), which joins the SAME running
        engine batch -- no stage barrier, no second prefill wave behind the slowest chunk.

        Data-parallel: whole groups are LPT-assigned to the replicas, so a group's follow-up runs where
        its inputs were produced and the only collective is ONE all-gather of both stages' results at
        the end (every rank enters it, errors included).  Returns ``(first, second)`` result lists
        (second[g] None when build returned None), or None when this job runs stages on a TP engine
        (the caller then falls back to two barrier-separated generates)."""
        from .engine import SamplingParams
        if self.par.tp > 1 or (self.par.world > 1 and self.parallel != "dp"):
            return None
        t0 = time.perf_counter()
        prompts = [self.encode_request(r) for r in reqs]
        dp, dp_rank = self.par.dp, self.par.dp_rank
        cost = [sum(len(prompts[i]) + 2 * reqs[i].max_tokens for i in g) for g in groups]
        gowner = assign_balanced(cost, dp)
        owner = [0] * len(reqs)
        for g, members in enumerate(groups):
            for i in members:
                owner[i] = gowner[g]
        self.owner_maps.setdefault(reqs[0].stage if reqs else "map", []).append(owner)
        for st in ("map", "reduce_l1"):
            self.stage_plan.setdefault(st, {"tp": 1, "handoff": False, "streamed": True})
        mine_g = [g for g in range(len(groups)) if gowner[g] == dp_rank]
        mine = [i for g in mine_g for i in groups[g]]
        group_of = {i: g for g in mine_g for i in groups[g]}
        left = {g: len(groups[g]) for g in mine_g}
        first: Dict[int, Dict[str, Any]] = {}
        second: Dict[int, Dict[str, Any]] = {}
        fed: List[int] = []  # engine request index len(mine) + k -> group fed[k]
        fed_mt: Dict[int, int] = {}  # group -> max_tokens of its follow-up request

        def rec(key, idx, o):
            return {key: idx, "text": self.tokenizer.decode(o.token_ids), "pt": o.prompt_len, "ct": len(o.token_ids),
                    "fr": o.finish_reason}

        def feeder(done):
            new = []
            for rid, o in done:
                if rid >= len(mine):
                    g = fed[rid - len(mine)]
                    second[g] = dict(rec("g", g, o), mt=fed_mt[g])
                    continue
                i = mine[rid]
                first[i] = rec("i", i, o)
                g = group_of[i]
                left[g] -= 1
                if left[g]:
                    continue
                r2 = build(g, [_result(first[j]) for j in groups[g]])
                if r2 is None:
                    continue
                fed.append(g)
                fed_mt[g] = r2.max_tokens
                new.append((self.encode_request(r2),
                            SamplingParams(r2.max_tokens, r2.temperature, _req_seed(self.seed, r2))))
            return new

        try:
            if mine:
                self._maybe_fault()
                self.engine.generate([prompts[i] for i in mine],
                                     [SamplingParams(reqs[i].max_tokens, reqs[i].temperature,
                                                     _req_seed(self.seed, reqs[i])) for i in mine],
                                     ignore_eos=self.ignore_eos, feeder=feeder)
        except Exception as e:  # noqa: BLE001 -- never skip the all-gather below: the peers are in it
            msg = "rank %d: %s: %s" % (self.par.rank, type(e).__name__, e)
            log.error("engine failed on %d streamed requests: %s", len(mine), msg)
            first = {i: {"i": i, "err": msg} for i in mine}
            second = {g: {"g": g, "err": msg} for g in mine_g}
        local = list(first.values()) + list(second.values())
        t1 = time.perf_counter()
        self.timings["generate_s"] += t1 - t0
        if pdist.is_initialized():
            parts = pdist.all_gather_json(local)
            local = [r for part in parts for r in part]
        self.timings["allgather_s"] += time.perf_counter() - t1
        m1 = {r["i"]: r for r in local if "i" in r}
        m2 = {r["g"]: r for r in local if "g" in r}
        res1 = [_result(m1[i]) if i in m1 else GenResult("", error="request %d produced no result" % i)
                for i in range(len(reqs))]
        res2 = [_result(m2[g]) if g in m2 else None for g in range(len(groups))]
        self._tally(res1, [r.max_tokens for r in reqs])
        self._tally([res2[g] for g in m2], [int(m2[g].get("mt", 0)) for g in m2])
        return res1, res2

    def stats(self) -> Dict[str, Any]:
        s: Dict[str, Any] = {"model": self.model, "dp": self.par.dp, "tp": self.par.tp, "parallel": self.parallel,
                             **self.timings}
        if self.stage_plan:
            s["stage_plan"] = dict(self.stage_plan)
        if self.stage_seconds:
            s["stage_seconds"] = {k: dict(v) for k, v in self.stage_seconds.items()}
        if self.p2p_latency:
            s["p2p_latency"] = {k: dict(v) for k, v in self.p2p_latency.items()}
        if self.hw is not None:
            s["planner_hw"] = {"ar_lat_us": round(self.hw.ar_lat_s * 1e6, 2),
                               "ar_us_per_row": round(self.hw.ar_lat_row_s * 1e6, 4),
                               "ar_gbps": round(self.hw.ar_bw / 1e9, 1)}
        if self._engine is not None:
            s.update(self._engine.engine_stats())
        if self._tp_engine is not None:
            s["tp_engine"] = self._tp_engine.engine_stats()
        others = {str(k): e.engine_stats() for k, e in self._tp_engines.items() if k != self.par.world}
        if others:
            s["tp_engines"] = others
        return s


def _result(r: Dict[str, Any]) -> GenResult:
    """GenResult of an all-gathered result record ({"text", "pt", "ct", "fr"} or {"err"})."""
    if "err" in r:
        return GenResult("", error=r["err"])
    return GenResult(r["text"], r["pt"], r["ct"], 0.0, extra={"finish_reason": r["fr"]})


def _rccl_bandwidth(group, hidden: int, device, rows: int = 4096) -> float:
    """Algorithm bandwidth (bytes/s) of one all-reduce of a prefill-sized bf16 activation on ``group``
    (second of two calls), MAX-reduced over the ranks."""
    import torch
    import torch.distributed as dist
    nccl = dist.get_backend(group) == "nccl"
    x = torch.ones(rows, hidden, dtype=torch.bfloat16, device=device if nccl else "cpu")
    best = float("inf")
    for _ in range(2):
        pdist.barrier()
        if nccl:
            torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        dist.all_reduce(x, group=group)
        if nccl:
            torch.cuda.synchronize(device)
        best = min(best, time.perf_counter() - t0)
    t = torch.tensor([best], dtype=torch.float64, device=device if nccl else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return x.numel() * 2 / max(float(t.item()), 1e-9)
