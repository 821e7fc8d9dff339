"""One-shot P2P all-reduce for latency-bound tensor-parallel decode.

RCCL's ring/tree all-reduce costs tens of microseconds for the B x 16 KiB messages of a TP decode
step, two per layer.  ``CustomAllReduce`` keeps one uncached, IPC-shared buffer per rank
(csrc/kernels/custom_ar.hip): every rank writes its input into its own buffer, flags every peer,
and then sums all peers' buffers directly over xGMI -- one kernel, no host involvement, legal
inside a hipGraph.  Handles are exchanged once through the group (any backend); messages larger
than ``max_bytes`` or non-fp32 tensors go to ``torch.distributed.all_reduce`` (RCCL).

The decode projections use a second, *push-mode* kernel (``add_rmsnorm``): every rank sums its own
split-K slabs, writes the row (bf16 payload) straight into every peer's buffer (posted remote stores
-- no remote read round trip), flags, and then reduces the rows from LOCAL memory in rank order in
fp32, adds the residual and applies the RMSNorm -- the all-reduce, the split-K reduction and the
add_rmsnorm kernel of the TP=1 graph in one launch.

The decode projections at up to 16 rows go one step further (``push_handle``, "TP push" in
csrc/kernels/stream_gemm.hip): the row-parallel GEMM's split-K last arriver pushes its column tile to
every peer itself and updates the residual after the rank-ordered sum, so neither a separate
all-reduce nor an add + RMSNorm launch runs -- the consumer GEMM applies the norm (deferred norm).
``LocalPush`` is the same handle over a group of one rank: a single-GPU TP-shard measurement runs the
identical kernels.

The reference has no collective of any kind (its only "communication" is HTTPS, reference
llm_executor.py:290-297); this is the MI355X replacement for the TP reduce path it implies.
"""

from __future__ import annotations

import ctypes
import os
import logging
from typing import Optional

import torch
import torch.distributed as dist

log = logging.getLogger("mrsum.custom_ar")

_SIGS = {
    "mrsum_ar_create": ([ctypes.c_int, ctypes.c_int, ctypes.c_size_t], ctypes.c_void_p),
    "mrsum_ar_ipc_handle": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mrsum_ar_open": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mrsum_ar_allreduce_f32": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p],
                               ctypes.c_int),
    "mrsum_ar_allreduce_max_u64": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_void_p], ctypes.c_int),
    "mrsum_ar_add_rmsnorm": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                              ctypes.c_void_p], ctypes.c_int),
    "mrsum_ar_error": ([ctypes.c_void_p], ctypes.c_int),
    "mrsum_ar_reset": ([ctypes.c_void_p], ctypes.c_int),
    "mrsum_ar_destroy": ([ctypes.c_void_p], None),
}



def _lib():
    from ..ops._lib import kernels_lib
    lib = kernels_lib()
    for name, (args, res) in _SIGS.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    return lib


class CustomAllReduce:
    """In-place fp32 sum over ``group`` for tensors of at most ``max_bytes`` (one per process/GPU)."""

    MAX_RANKS = 8
    # the P2P paths the decode uses, each self-tested at the model's shapes (self_test):
    #   one_shot    -- mrsum_ar_allreduce_f32 (fp32 split-K slabs of the non-fused path)
    #   fused_norm  -- mrsum_ar_add_rmsnorm (push-mode all-reduce + residual add + RMSNorm)
    #   push_stream -- the stream GEMM's split-K last arriver pushing its tile (stream_gemm.hip "TP push")
    #   push_skinny -- the register-streaming producer pushing its tile (every workgroup spins on its peers)
    #   max_u64     -- the vocab-parallel sampler's 8-byte Gumbel-key max
    PATHS = ("one_shot", "fused_norm", "push_stream", "push_skinny", "max_u64")

    def __init__(self, group=None, max_bytes: int = 4 << 20):
        """``max_bytes`` bounds one message: the one-shot kernel takes at most 1 MiB of it, the fused
        add_rmsnorm (push mode, bf16 rows of 8 KiB for Llama-3-8B, 16 KiB for Llama-3-70B) its
        MAX_ROWS = 256 rows."""
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > self.MAX_RANKS:
            raise ValueError("custom all-reduce supports at most %d ranks" % self.MAX_RANKS)
        self.max_bytes = int(max_bytes)
        # per-path verdicts of the start-up self-test (self_test): a path that failed on ANY rank is off on
        # every rank and its callers take the next path (push -> fused add + RMSNorm -> one-shot slabs)
        self.paths = {p: True for p in self.PATHS}
        self._lib = _lib()
        # every step ends in a collective whatever happened locally, so all ranks agree on the
        # outcome (a rank that raised alone would leave its peers waiting in the next collective)
        self._h = self._lib.mrsum_ar_create(self.rank, self.world, self.max_bytes)
        handle = None
        if self._h:
            buf = ctypes.create_string_buffer(64)
            if self._lib.mrsum_ar_ipc_handle(self._h, buf) == 0:
                handle = bytes(buf.raw)
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        if any(h is None for h in handles):
            self.close()
            raise RuntimeError("custom all-reduce: allocation / IPC export failed on some rank")
        rc = self._lib.mrsum_ar_open(self._h, b"".join(handles))
        oks = [None] * self.world
        dist.all_gather_object(oks, rc == 0, group=group)
        if not all(oks):
            self.close()
            raise RuntimeError("custom all-reduce: hipIpcOpenMemHandle failed on some rank (rc %d here)" % rc)

    ONE_SHOT_MAX = 1 << 20  # bytes the one-shot kernel takes per call

    def fits(self, t: torch.Tensor) -> bool:
        return (self.paths["one_shot"] and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                and t.numel() % 4 == 0 and t.numel() * 4 <= min(self.max_bytes, self.ONE_SHOT_MAX))

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """Sum ``t`` over the group in place (RCCL for tensors the P2P path does not take)."""
        if not self.fits(t):
            dist.all_reduce(t, group=self.group)
            return t
        rc = self._lib.mrsum_ar_allreduce_f32(self._h, t.data_ptr(), t.data_ptr(), t.numel(),
                                              torch.cuda.current_stream(t.device).cuda_stream)
        if rc:
            raise RuntimeError("custom all-reduce launch failed (%d)" % rc)
        return t

    MAX_ROWS = 256

    def fits_rows(self, parts: torch.Tensor) -> bool:
        """Can ``add_rmsnorm`` take these fp32 split-K slabs [S, T, D]?"""
        if not (parts.is_cuda and parts.dtype == torch.float32 and parts.is_contiguous() and parts.dim() == 3):
            return False
        _, T, D = parts.shape
        return (self.paths["fused_norm"] and T <= self.MAX_ROWS and D % 4 == 0 and D <= 8192
                and T * D * 2 <= self.max_bytes)

    def add_rmsnorm(self, parts: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Fused push-mode all-reduce of this rank's split-K slabs ``parts`` [S, T, D] (fp32) +
        ``residual += sum`` (bf16, in place) + RMSNorm: returns ``rmsnorm(residual) * w`` [T, D] bf16.
        One kernel (csrc/kernels/custom_ar.hip: ar_add_rmsnorm_kernel); graph-safe."""
        if not self.fits_rows(parts):
            raise ValueError("add_rmsnorm: parts must be contiguous fp32 [S, T<=256, D] within max_bytes")
        S, T, D = parts.shape
        if not (residual.dtype == torch.bfloat16 and residual.is_contiguous() and residual.shape == (T, D)
                and w.dtype == torch.bfloat16 and w.numel() == D):
            raise ValueError("add_rmsnorm: residual [T, D] / w [D] bf16 expected")
        if out is None:
            out = torch.empty(T, D, dtype=torch.bfloat16, device=parts.device)
        rc = self._lib.mrsum_ar_add_rmsnorm(self._h, parts.data_ptr(), S, T, residual.data_ptr(), w.data_ptr(),
                                            out.data_ptr(), D, out.stride(0), float(eps),
                                            torch.cuda.current_stream(parts.device).cuda_stream)
        if rc:
            raise RuntimeError("custom all-reduce (add_rmsnorm) launch failed (%d)" % rc)
        return out

    # granule-push (GEMM epilogue) limits: csrc/kernels/ar_common.h MAX_GRAN x GRAN columns
    PUSH_MAX_HIDDEN = 8192

    def push_ok(self, rows: int, hidden: int) -> bool:
        """Can a TP-push GEMM epilogue all-reduce ``rows`` x ``hidden`` over this group?"""
        return (bool(self._h) and bool(self.push_kinds()) and 1 <= rows <= 64 and hidden % 16 == 0
                and hidden <= self.PUSH_MAX_HIDDEN and rows * hidden * 4 <= self.max_bytes)

    def push_kinds(self) -> set:
        """The TP-push producers that passed the self-test: {"stream", "skinny"} or a subset."""
        return {k for k in ("stream", "skinny") if self.paths["push_" + k]}

    def push_handle(self) -> int:
        """The native handle a TP-push GEMM epilogue takes (ops.hip.stream_resid ``tp``)."""
        return self._h

    def max_u64_(self, t: torch.Tensor) -> torch.Tensor:
        """Element-wise max over the group, in place, of an int64 tensor holding unsigned 64-bit keys
        (the sampler's Gumbel-max keys; values are compared as unsigned)."""
        if not (t.is_cuda and t.dtype == torch.int64 and t.is_contiguous() and t.numel() * 8 <= self.max_bytes):
            raise ValueError("max_u64_: contiguous int64 cuda tensor of <= max_bytes expected")
        rc = self._lib.mrsum_ar_allreduce_max_u64(self._h, t.data_ptr(), t.data_ptr(), t.numel(),
                                                  torch.cuda.current_stream(t.device).cuda_stream)
        if rc:
            raise RuntimeError("custom all-reduce (max) launch failed (%d)" % rc)
        return t

    def self_test(self, shapes: Optional[dict] = None, iters: int = 3) -> bool:
        """COLLECTIVE start-up check of every P2P path against torch.distributed, at the MODEL's shapes:
        ``shapes`` = {"hidden": H, "k": {"o": K_o, "down": K_down} (this rank's shard K of the row-parallel
        projections), "fp8": bool, "rows": decode row counts (default 1, 16, 64)}; None: Llama-3-8B's
        hidden 4096 with TP=8 shard K.  Per path (PATHS): eager calls with values that change per call (a
        stale slot, flag or epoch shows up as a mismatch) and hipGraph replays, compared with RCCL / the fp32
        reference and across ranks.  Each path's verdict is agreed over the group (a path that failed on one
        rank is off everywhere; ``self.paths``); the group then resets the P2P state.  Returns whether the
        handle is usable at all (graph_safe): a graph-safe decode reduction for every decode bucket -- the
        fused path, or the one-shot path where one fp32 slab of the largest bucket fits it -- AND the key max
        (the vocab-parallel sampler has no graph-safe fallback)."""
        sh = dict(hidden=4096, k={"o": 512, "down": 1792}, fp8=False, rows=(1, 16, 64))
        sh.update(shapes or {})
        dev = torch.device("cuda", torch.cuda.current_device())
        H, rows = int(sh["hidden"]), tuple(int(r) for r in sh["rows"])
        local = {}

        self.why = {}

        def run(name, fn):
            try:
                ok = bool(fn())
                if not ok:
                    self.why.setdefault(name, "mismatch against the reference")
            except Exception as e:  # keep the collective sequence aligned across ranks
                log.warning("custom all-reduce self-test of %s raised: %s", name, e)
                ok = False
                self.why[name] = "raised: %s" % (str(e)[:200],)
            # a timed-out wait (sticky error word, on the waiting rank only) poisons the handle's later
            # calls: the group agrees on it and clears the P2P state together before the next path
            err_any, _ = self.agree_error()
            if err_any:
                ok = False
                self.why.setdefault(name, "a wait for a peer timed out (error word %d)" % err_any)
                self.reset()
            local[name] = ok

        run("one_shot", lambda: self._test_one_shot(dev, H, rows, iters))
        run("fused_norm", lambda: self._test_fused(dev, iters, rows, H))
        run("max_u64", lambda: self._test_max_u64(dev, rows, iters))
        exercised = {"one_shot": True, "fused_norm": True, "max_u64": True}
        for kind in ("stream", "skinny"):
            def t(kind=kind):
                # every (role, M) case runs on every rank, whatever an earlier case gave on any rank, and the
                # group agrees on each case's outcome before the next one starts: a case that failed or raised
                # on one rank only must not leave that rank in a different collective (or a push kernel
                # waiting on a peer that has moved on) than its peers
                tested, ok = False, True
                for role, K in sorted(sh["k"].items()):
                    for M in rows:
                        if _push_case(self, kind, M, H, int(K), bool(sh["fp8"]), role) is None:
                            continue
                        tested = True
                        graph = M in (rows[0], rows[-1])
                        try:
                            case = _test_push(self, dev, iters, group=self.group, M=M, N=H, K=int(K), kind=kind,
                                              fp8=bool(sh["fp8"]), role=role, graph=graph)
                        except Exception as e:
                            log.warning("custom all-reduce self-test: %s push raised at %s M=%d: %s", kind, role,
                                        M, e)
                            self.why.setdefault("push_" + kind, "raised at %s M=%d: %s" % (role, M, str(e)[:160]))
                            case = False
                        err_any, failed_any = self.agree_error(local_failed=not case)
                        if err_any:
                            self.reset()
                        if not case or err_any or failed_any:
                            log.warning("custom all-reduce self-test: %s push failed at %s M=%d N=%d K=%d",
                                        kind, role, M, H, K)
                            self.why.setdefault("push_" + kind, "mismatch at %s M=%d on some rank" % (role, M))
                            ok = False
                exercised["push_" + kind] = tested
                return ok
            run("push_" + kind, t)
        votes = [None] * self.world
        dist.all_gather_object(votes, local, group=self.group)
        for p in self.PATHS:
            self.paths[p] = all(v is not None and v.get(p, False) for v in votes)
        # report: "ok" / "failed" per path, "n/a" where the model's shapes never take that path (e.g. the
        # register-streaming push under fp8 weights)
        self.report = {p: ("ok" if self.paths[p] else "failed") if exercised.get(p, True) or not self.paths[p]
                       else "n/a" for p in self.PATHS}
        self.report["shapes"] = "hidden %d, shard K %s, rows %s%s" % (H, dict(sh["k"]), list(rows),
                                                                     ", fp8" if sh["fp8"] else "")
        why = [None] * self.world
        dist.all_gather_object(why, self.why, group=self.group)
        reasons = {p: sorted({w[p] for w in why if w and p in w}) for p in self.PATHS if not self.paths[p]}
        if reasons:
            self.report["why"] = {p: "; ".join(r) for p, r in reasons.items()}
            log.warning("custom all-reduce self-test: paths off: %s", self.report["why"])
        # the test's tagged words sit at offsets that later belong to other granules / rows: start the real
        # traffic from zeroed slots and epoch 1 on every rank, whatever the test's iteration count
        self.reset()
        log.info("custom all-reduce self-test (hidden %d, rows %s): %s", H, rows, self.paths)
        usable = graph_safe(self.paths, H, self.ONE_SHOT_MAX, self.MAX_ROWS)
        if not usable:
            self.report["unusable"] = ("the passing paths leave decode batches up to %d rows at hidden %d "
                                       "without a graph-safe all-reduce" % (self.MAX_ROWS, H))
        return usable

    def selftest_report(self) -> dict:
        """Per path "ok" / "failed" / "n/a" of the start-up self-test (+ the shapes it ran at)."""
        return dict(getattr(self, "report", {p: "untested" for p in self.PATHS}))

    def _test_one_shot(self, dev, H: int, rows, iters: int) -> bool:
        """mrsum_ar_allreduce_f32 at the decode's message sizes (rows x hidden fp32, capped at the kernel's
        1 MiB), eager and graph-replayed, bit-equal to RCCL (integer-valued fp32: the sum is exact)."""
        ok = True
        for M in rows:
            n = min(M * H, self.ONE_SHOT_MAX // 4)
            n -= n % 4
            x = torch.empty(n, device=dev)
            ref = torch.empty(n, device=dev)
            base = torch.arange(n, device=dev, dtype=torch.float32).remainder_(251)

            def fill(i):
                x.copy_(base).mul_(self.rank + 1).add_(i)
                ref.copy_(x)

            for i in range(iters):
                fill(i)
                self.all_reduce(x)
                dist.all_reduce(ref, group=self.group)
                ok &= bool(torch.equal(x, ref))
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                self.all_reduce(x)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self.all_reduce(x)
            for i in range(iters):
                fill(10 + i)
                g.replay()
                dist.all_reduce(ref, group=self.group)
                torch.cuda.synchronize(dev)
                ok &= bool(torch.equal(x, ref))
        return ok

    def _test_max_u64(self, dev, rows, iters: int) -> bool:
        """max_u64_ over keys with the top bit set and clear (compared UNSIGNED), eager and graph-replayed,
        against the keys all-gathered over the group and reduced on the host."""
        import numpy as np
        ok = True
        for B in rows:
            t = torch.empty(B, dtype=torch.int64, device=dev)
            keep = torch.empty_like(t)

            def fill(i):
                g = torch.Generator(device="cpu").manual_seed(7919 * i + 31 * self.rank + B)
                k = torch.randint(-(1 << 62), 1 << 62, (B,), generator=g, dtype=torch.int64) * 2 + (i & 1)
                t.copy_(k)
                keep.copy_(k)

            def check():
                allk = [torch.empty_like(keep) for _ in range(self.world)]
                if dist.get_backend(self.group) == "nccl":
                    dist.all_gather(allk, keep, group=self.group)
                else:
                    cpu = [torch.empty(B, dtype=torch.int64) for _ in range(self.world)]
                    dist.all_gather(cpu, keep.cpu(), group=self.group)
                    allk = cpu
                want = np.max(np.stack([a.cpu().numpy().view(np.uint64) for a in allk]), axis=0)
                return bool(np.array_equal(t.cpu().numpy().view(np.uint64), want))

            for i in range(iters):
                fill(i)
                self.max_u64_(t)
                torch.cuda.synchronize(dev)
                ok &= check()
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                self.max_u64_(t)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self.max_u64_(t)
            for i in range(iters):
                fill(40 + i)
                g.replay()
                torch.cuda.synchronize(dev)
                ok &= check()
        return ok

    def reset(self) -> None:
        """COLLECTIVE: clear the flags, slots, epochs and the sticky error word on every rank of the group
        (after a timed-out wait: the handle is usable again).  Every rank must call it at the same point
        with no kernel of this handle queued; the barriers around the local clear keep a fast rank from
        pushing into a peer's region before that peer has cleared it."""
        dist.barrier(group=self.group)
        rc = self._lib.mrsum_ar_reset(self._h)
        oks = [None] * self.world
        dist.all_gather_object(oks, rc == 0, group=self.group)
        if not all(oks):
            raise RuntimeError("custom all-reduce: reset failed on some rank (rc %d here)" % rc)

    def agree_error(self, local_failed: bool = False):
        """COLLECTIVE: (the error words of every rank OR-ed, whether any rank reports ``local_failed``).  A rank
        whose own waits all succeeded may still hold garbage pushed by a timed-out peer, and a rank whose
        call raised must not leave its peers alone in the next collective, so the group decides together."""
        votes = [None] * self.world
        dist.all_gather_object(votes, (self.error(), bool(local_failed)), group=self.group)
        err, failed = 0, False
        for v in votes:
            e, f = v if v is not None else (1, True)
            err |= int(e) if e is not None and e >= 0 else 1
            failed |= bool(f)
        return err, failed

    def _test_fused(self, dev, iters: int, rows=(5,), D: int = 512, S: int = 2) -> bool:
        """add_rmsnorm at D = hidden for every decode row count in ``rows``."""
        ok = True
        for T in rows:
            if T * D * 2 <= self.max_bytes and T <= self.MAX_ROWS:
                ok &= self._test_fused_one(dev, iters, T, D, S)
        return ok

    def _test_fused_one(self, dev, iters: int, T: int, D: int, S: int) -> bool:
        """add_rmsnorm against (collective sum of the slabs) + the fp32 reference add_rmsnorm, eager
        and graph-replayed; every rank must also produce the bit-identical residual."""
        from ..ops import reference
        ok = True
        g = torch.Generator(device="cpu").manual_seed(1234)
        w = (torch.rand(D, generator=g) + 0.5).to(torch.bfloat16).to(dev)
        parts = torch.empty(S, T, D, device=dev)
        res0 = torch.randn(T, D, generator=g).to(torch.bfloat16).to(dev)
        res = res0.clone()
        out = torch.empty(T, D, dtype=torch.bfloat16, device=dev)

        def fill(i):
            gi = torch.Generator(device="cpu").manual_seed(100 * i + self.rank)
            parts.copy_(torch.randn(S, T, D, generator=gi))
            res.copy_(res0)

        def check():
            # the kernel's arithmetic exactly: each rank's slab sum rounded to the bf16 payload, summed in rank
            # order in fp32, added to the residual with one bf16 rounding (an fp32 all-reduce as the reference
            # leaves the payload rounding of `world` ranks in the error: 0.04 worst case at 8 ranks)
            mine = parts.sum(0).to(torch.bfloat16)
            allv = [torch.empty_like(mine) for _ in range(self.world)]
            if dist.get_backend(self.group) == "nccl":
                dist.all_gather(allv, mine, group=self.group)
            else:
                cpu = [torch.empty(mine.shape, dtype=mine.dtype) for _ in range(self.world)]
                dist.all_gather(cpu, mine.cpu(), group=self.group)
                allv = [c.to(dev) for c in cpu]
            tot = torch.zeros(T, D, device=dev)
            for v in allv:
                tot += v.float()
            ref_res = res0.clone()
            ref_out = reference.add_rmsnorm(tot, ref_res, w, 1e-5)
            g1 = bool(torch.allclose(res.float(), ref_res.float(), atol=1e-3, rtol=1e-2))
            g2 = bool(torch.allclose(out.float(), ref_out.float(), atol=3e-2, rtol=2e-2))
            mine = res.float().sum().reshape(1)
            hi, lo = mine.clone(), mine.clone()
            dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
            g3 = bool(torch.equal(hi, lo))
            if not (g1 and g2 and g3):
                self.why.setdefault("fused_norm", "T=%d D=%d: residual %s (max err %.3g), out %s (max err %.3g), "
                                    "ranks %s" % (T, D, "ok" if g1 else "MISMATCH",
                                                  float((res.float() - ref_res.float()).abs().max()),
                                                  "ok" if g2 else "MISMATCH",
                                                  float((out.float() - ref_out.float()).abs().max()),
                                                  "agree" if g3 else "DISAGREE"))
            return g1 and g2 and g3

        for i in range(iters):
            fill(i)
            self.add_rmsnorm(parts, res, w, 1e-5, out)
            torch.cuda.synchronize(dev)
            ok &= check()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            self.add_rmsnorm(parts, res, w, 1e-5, out)
        for i in range(iters):
            fill(50 + i)
            gr.replay()
            torch.cuda.synchronize(dev)
            ok &= check()
        return ok

    def measure_latency(self, rows=(1, 64), hidden: int = 4096, calls: int = 64, reps: int = 3,
                        push_k: Optional[int] = None, fp8: bool = False):
        """(a, b): a decode all-reduce over this group costs a + b * rows seconds MORE than the same kernel
        over a group of one rank (LocalPush: the push to its own slot, the wait and the rank-ordered sum, which
        a TP-shard decode step measured on one GPU already contains) -- the cross-GPU part of a decode
        all-reduce.  Timed on the path the decode runs: with ``push_k`` (the shard K of a row-parallel
        projection) and a passing push producer, the TP-push residual producer at N = ``hidden``, K = push_k
        (stream kernel, the plan's launch parameters); else the fused all-reduce + add_rmsnorm.  Least squares
        over ``rows``; timed inside replayed hipGraphs; MAX over the ranks, so every rank plans with the same
        numbers."""
        from ..ops import hip
        from ..ops.reference import Fp8Weight
        dev = torch.device("cuda", torch.cuda.current_device())
        local = LocalPush(self.max_bytes)
        pts = []
        use_push = push_k is not None and self.paths["push_stream"]
        for r in rows:
            r = max(1, min(int(r), self.max_bytes // (hidden * 4), self.MAX_ROWS, 64 if use_push else self.MAX_ROWS))
            parts = torch.zeros(1, r, hidden, device=dev)
            res = torch.zeros(r, hidden, dtype=torch.bfloat16, device=dev)
            w = torch.ones(hidden, dtype=torch.bfloat16, device=dev)
            out = torch.empty_like(res)
            rp = _push_case(self, "stream", r, hidden, int(push_k), fp8) if use_push else None
            if rp is not None:
                x = torch.zeros(r, int(push_k), dtype=torch.bfloat16, device=dev)
                wm = torch.zeros(hidden, int(push_k), dtype=torch.bfloat16, device=dev)
                wm = Fp8Weight.quantize(wm) if fp8 else wm

                def fn_of(h):
                    return lambda: hip.stream_resid(x, wm, res, rp[1], rp[2], tp=h.push_handle())
            else:
                def fn_of(h):
                    return lambda: h.add_rmsnorm(parts, res, w, 1e-5, out)

            def timed(fn) -> float:
                s = torch.cuda.Stream(device=dev)
                s.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(s):
                    fn()
                torch.cuda.synchronize(dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(calls):
                        fn()
                g.replay()
                torch.cuda.synchronize(dev)
                best = float("inf")
                for _ in range(reps):
                    dist.barrier(group=self.group)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g.replay()
                    e1.record()
                    torch.cuda.synchronize(dev)
                    best = min(best, e0.elapsed_time(e1) / 1000.0 / calls)
                return best

            t_ar = timed(fn_of(self))
            t_local = timed(fn_of(local))
            pts.append((r, max(0.0, t_ar - t_local)))
        local.close()
        self.reset()  # the timed pushes advanced the epochs of this handle and of nothing else: start clean
        n = len(pts)
        mx = sum(p[0] for p in pts) / n
        my = sum(p[1] for p in pts) / n
        var = sum((p[0] - mx) ** 2 for p in pts)
        b = max(0.0, sum((p[0] - mx) * (p[1] - my) for p in pts) / var) if var else 0.0
        a = max(0.0, my - b * mx)
        v = torch.tensor([a, b], dtype=torch.float64, device=dev if dist.get_backend(self.group) == "nccl" else "cpu")
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=self.group)
        self.latency_path = "push" if use_push else "fused"
        return float(v[0].item()), float(v[1].item())

    def error(self) -> int:
        """Non-zero if a wait for a peer timed out (the result of that call is garbage)."""
        return int(self._lib.mrsum_ar_error(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.mrsum_ar_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter teardown
            pass


def _push_case(h, kind: str, M: int, N: int, K: int, fp8: bool, role: str = "o"):
    """The producer launch parameters of a TP push of ``kind`` at M x N x K as the decode runs it
    (ops._resid_plan with tp=True, forced to ``kind``), or None when that producer does not take the shape."""
    from .. import ops
    from ..ops import hip
    if M > 64 or K % 128 or N % 16:
        return None
    a = torch.empty(M, K, dtype=torch.bfloat16, device="meta")
    w = _meta_weight(N, K, fp8)
    try:
        rp = ops._resid_plan(hip, a, w, role, tp=True, force=kind)
    except Exception:  # noqa: BLE001 -- a plan the producer cannot take
        return None
    if rp is None or rp[0] != kind:
        return None
    if kind == "skinny" and N // 16 > (hip.skinny_fp8_resid_capacity() if fp8 else hip.skinny_resid_capacity(N)):
        return None
    return rp


def _meta_weight(N: int, K: int, fp8: bool):
    from ..ops.reference import Fp8Weight
    if fp8:
        return Fp8Weight(torch.empty(N, K, dtype=torch.float8_e4m3fn, device="meta"),
                         torch.empty(N, dtype=torch.float32, device="meta"))
    return torch.empty(N, K, dtype=torch.bfloat16, device="meta")


def _test_push(h, dev, iters: int, group=None, M: int = 3, N: int = 2048, K: int = 512, kind: str = "stream",
               fp8: bool = False, role: str = "o", graph: bool = True, wpb: Optional[int] = None,
               S: Optional[int] = None) -> bool:
    """The TP-push residual producer ``kind`` ("stream": ops.hip.stream_resid, bf16 or fp8 weights;
    "skinny": ops.hip.skinny_resid) at M x N x K with the launch parameters the decode's plan gives that
    shape (or ``wpb`` / ``S``), against the collective sum of every rank's x @ w^T on the same residual,
    eager and (``graph``) graph-replayed, values changing per call (a stale slot, flag or epoch shows up);
    the residual must also be bit-identical across ranks.  ``group`` None with a LocalPush ``h``."""
    from ..ops import hip
    from ..ops.reference import Fp8Weight
    rp = _push_case(h, kind, M, N, K, fp8, role) if (wpb is None or S is None) else ("stream", wpb, S)
    if rp is None:
        raise ValueError("no %s push producer for M=%d N=%d K=%d" % (kind, M, N, K))
    ok = True
    g = torch.Generator(device="cpu").manual_seed(4321 + M)
    res0 = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    res = res0.clone()
    x = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
    wb = torch.empty(N, K, dtype=torch.bfloat16, device=dev)
    w8 = [None]
    ssp = [None]
    rank = h.rank

    def fill(i):
        gi = torch.Generator(device="cpu").manual_seed(1000 * i + 7 * rank + M)
        x.copy_((torch.randn(M, K, generator=gi) * 0.5).to(torch.bfloat16))
        wb.copy_((torch.randn(N, K, generator=gi) * 0.05).to(torch.bfloat16))
        if fp8:
            q = Fp8Weight.quantize(wb)
            if w8[0] is None:
                w8[0] = q
            else:  # keep the captured pointers
                w8[0].q.copy_(q.q)
                w8[0].scale.copy_(q.scale)
        res.copy_(res0)

    def weight():
        return w8[0] if fp8 else wb

    def run():
        if rp[0] == "skinny":
            ssp[0] = hip.skinny_resid(x, weight(), res, tp=h.push_handle())
        else:
            ssp[0] = hip.stream_resid(x, weight(), res, rp[1], rp[2], tp=h.push_handle())

    def check():
        wf = (w8[0].q.float() * w8[0].scale[:, None]) if fp8 else wb.float()
        tot = x.float() @ wf.t()
        if h.world > 1:
            dist.all_reduce(tot, group=group)
        ref = (res0.float() + tot).to(torch.bfloat16).float()
        good = bool(torch.allclose(res.float(), ref, atol=6e-2, rtol=2e-2))
        tiles = ssp[0].shape[1]
        ss = res.float().pow(2).reshape(M, tiles, N // tiles).sum(-1)
        good &= bool(torch.allclose(ssp[0], ss, rtol=1e-3, atol=1e-2))
        if h.world > 1:
            mine = res.float().sum().reshape(1)
            hi, lo = mine.clone(), mine.clone()
            dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
            good &= bool(torch.equal(hi, lo))
        return good

    for i in range(iters):
        fill(i)
        run()
        torch.cuda.synchronize(dev)
        ok &= check()
    if graph:
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            fill(90)
            run()
        torch.cuda.synchronize(dev)
        ok &= check()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            run()
        for i in range(iters):
            fill(60 + i)
            gr.replay()
            torch.cuda.synchronize(dev)
            ok &= check()
    return ok and h.error() == 0


class LocalPush:
    """A custom all-reduce over a group of ONE rank (no IPC, no process group): the decode of a TP shard
    measured on one GPU runs the same kernels as a rank of a real group -- the TP-push GEMM epilogue and
    the fused push-mode all-reduce + add + RMSNorm (push to its own slot, wait, rank-ordered sum) --
    without the xGMI latency of the remote stores."""

    rank, world = 0, 1
    PUSH_MAX_HIDDEN = CustomAllReduce.PUSH_MAX_HIDDEN

    def __init__(self, max_bytes: int = 4 << 20):
        self.max_bytes = int(max_bytes)
        # per-path verdicts of the start-up self-test (self_test): a path that failed on ANY rank is off on
        # every rank and its callers take the next path (push -> fused add + RMSNorm -> one-shot slabs)
        self.paths = {p: True for p in self.PATHS}
        self._lib = _lib()
        self._h = self._lib.mrsum_ar_create(0, 1, self.max_bytes)
        if not self._h:
            raise RuntimeError("LocalPush: allocation failed")

    MAX_ROWS = CustomAllReduce.MAX_ROWS
    PATHS = CustomAllReduce.PATHS
    paths = {p: True for p in CustomAllReduce.PATHS}
    push_kinds = CustomAllReduce.push_kinds
    push_ok = CustomAllReduce.push_ok
    push_handle = CustomAllReduce.push_handle
    fits_rows = CustomAllReduce.fits_rows
    add_rmsnorm = CustomAllReduce.add_rmsnorm
    error = CustomAllReduce.error
    close = CustomAllReduce.close

    def reset(self) -> None:
        rc = self._lib.mrsum_ar_reset(self._h)
        if rc:
            raise RuntimeError("LocalPush: reset failed (%d)" % rc)
    __del__ = CustomAllReduce.__del__


def graph_safe(paths: dict, hidden: int, one_shot_max: int, max_rows: int) -> bool:
    """Whether the self-tested ``paths`` leave a graph-safe TP reduction for EVERY decode batch up to
    ``max_rows`` rows (the engine's largest graph bucket) at ``hidden``: the fused all-reduce + add + RMSNorm
    takes any of them; without it the decode falls back to the one-shot kernel over one fp32 slab [M, hidden],
    which must then fit ``one_shot_max`` bytes at ``max_rows`` rows -- otherwise a captured large-batch step
    would reach the RCCL path inside the capture (model._all_reduce refuses that).  The vocab-parallel
    sampler's key max has no graph-safe fallback.  A False verdict drops the handle: the engine then runs
    RCCL and no decode graphs."""
    if not paths.get("max_u64"):
        return False
    if paths.get("fused_norm"):
        return True
    return bool(paths.get("one_shot")) and max_rows * hidden * 4 <= one_shot_max


def maybe_custom_all_reduce(group=None, max_bytes: int = 4 << 20, shapes: Optional[dict] = None
                            ) -> Optional[CustomAllReduce]:
    """A CustomAllReduce for ``group`` when every rank is on a GPU and its self-test at ``shapes`` (the
    model's hidden size / shard K, see CustomAllReduce.self_test) leaves a graph-safe path, else None (RCCL /
    gloo path).  Paths that failed the test are off (``paths``); their callers take the next path."""
    if not (dist.is_initialized() and torch.cuda.is_available()):
        return None
    from .. import IPC_MODE_TOO_LATE
    try:
        ar = CustomAllReduce(group, max_bytes)
    except Exception as e:  # no IPC (e.g. container without dmabuf): fall back to RCCL
        if IPC_MODE_TOO_LATE:
            log.error("custom all-reduce: HIP was initialised before HSA_ENABLE_IPC_MODE_LEGACY=0 was set "
                      "(set it in the environment before the first GPU call); dmabuf IPC is unavailable")
        log.warning("custom all-reduce unavailable, using RCCL: %s", e)
        return None
    if not ar.self_test(shapes):
        log.warning("custom all-reduce failed its self-test on some rank (%s); using RCCL", ar.paths)
        ar.close()
        return None
    return ar
