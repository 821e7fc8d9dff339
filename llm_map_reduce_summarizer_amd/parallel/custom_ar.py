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

    def fits(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() % 4 == 0
                and t.numel() * 4 <= min(self.max_bytes, 1 << 20))

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
        return T <= self.MAX_ROWS and D % 4 == 0 and D <= 8192 and T * D * 2 <= self.max_bytes

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
        return (bool(self._h) and 1 <= rows <= 64 and hidden % 16 == 0 and hidden <= self.PUSH_MAX_HIDDEN
                and rows * hidden * 4 <= self.max_bytes)

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

    def self_test(self, iters: int = 4, n: int = 65536) -> bool:
        """Collective check against torch.distributed on every rank: eager and hipGraph-replayed
        calls with values that change per call (a stale slot or flag shows up as a mismatch).  All
        ranks return the same verdict."""
        ok = True
        dev = torch.device("cuda", torch.cuda.current_device())
        try:
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
            ok &= self._test_fused(dev, iters)
            ok &= _test_push(self, dev, iters, group=self.group)
            ok &= self.error() == 0
        except Exception as e:  # keep the collective sequence aligned across ranks
            log.warning("custom all-reduce self-test raised: %s", e)
            ok = False
        votes = [None] * self.world
        dist.all_gather_object(votes, ok, group=self.group)
        # the test's tagged words sit at offsets that later belong to other granules / rows: start the real
        # traffic from zeroed slots and epoch 1 on every rank, whatever the test's iteration count
        self.reset()
        return all(votes)

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

    def _test_fused(self, dev, iters: int, T: int = 5, D: int = 512, S: int = 2) -> bool:
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
            tot = parts.sum(0)
            dist.all_reduce(tot, group=self.group)
            ref_res = res0.clone()
            ref_out = reference.add_rmsnorm(tot, ref_res, w, 1e-5)
            good = torch.allclose(res.float(), ref_res.float(), atol=3e-2, rtol=2e-2)
            good &= torch.allclose(out.float(), ref_out.float(), atol=6e-2, rtol=3e-2)
            mine = res.float().sum().reshape(1)
            hi, lo = mine.clone(), mine.clone()
            dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
            return bool(good) and bool(torch.equal(hi, lo))

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

    def measure_latency(self, rows=(1, 64), hidden: int = 4096, calls: int = 64, reps: int = 3):
        """(a, b): a fused all-reduce + add_rmsnorm call over this group costs a + b * rows seconds MORE
        than the same kernel over a group of one rank (LocalPush: the push to its own slot, the wait and
        the rank-ordered sum, which a TP-shard decode step measured on one GPU already contains) -- the
        cross-GPU part of a decode all-reduce, the TP push of the GEMM epilogues included (the same
        remote stores and polls).  Least squares over ``rows``; both timed inside replayed hipGraphs.
        MAX over the ranks, so every rank plans with the same numbers."""
        dev = torch.device("cuda", torch.cuda.current_device())
        local = LocalPush(self.max_bytes)
        pts = []
        for r in rows:
            r = max(1, min(int(r), self.max_bytes // (hidden * 2), self.MAX_ROWS))
            parts = torch.zeros(1, r, hidden, device=dev)
            res = torch.zeros(r, hidden, dtype=torch.bfloat16, device=dev)
            w = torch.ones(hidden, dtype=torch.bfloat16, device=dev)
            out = torch.empty_like(res)

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

            t_ar = timed(lambda: self.add_rmsnorm(parts, res, w, 1e-5, out))
            t_local = timed(lambda: local.add_rmsnorm(parts, res, w, 1e-5, out))
            pts.append((r, max(0.0, t_ar - t_local)))
        local.close()
        n = len(pts)
        mx = sum(p[0] for p in pts) / n
        my = sum(p[1] for p in pts) / n
        var = sum((p[0] - mx) ** 2 for p in pts)
        b = max(0.0, sum((p[0] - mx) * (p[1] - my) for p in pts) / var) if var else 0.0
        a = max(0.0, my - b * mx)
        v = torch.tensor([a, b], dtype=torch.float64, device=dev if dist.get_backend(self.group) == "nccl" else "cpu")
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=self.group)
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


def _test_push(h, dev, iters: int, group=None, M: int = 3, N: int = 2048, K: int = 512, wpb: int = 4,
               S: int = 4) -> bool:
    """The TP-push residual producer (ops.hip.stream_resid with ``tp``) against the collective sum of every
    rank's x @ w^T on the same residual, eager and graph-replayed (values change per call: a stale slot,
    flag or epoch shows up); the residual must also be bit-identical across ranks.  ``group`` None with
    a LocalPush ``h`` (one rank)."""
    from ..ops import hip
    ok = True
    g = torch.Generator(device="cpu").manual_seed(4321)
    res0 = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    res = res0.clone()
    x = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
    w = torch.empty(N, K, dtype=torch.bfloat16, device=dev)
    ssp = [None]
    rank = h.rank

    def fill(i):
        gi = torch.Generator(device="cpu").manual_seed(1000 * i + 7 * rank)
        x.copy_((torch.randn(M, K, generator=gi) * 0.5).to(torch.bfloat16))
        w.copy_((torch.randn(N, K, generator=gi) * 0.05).to(torch.bfloat16))
        res.copy_(res0)

    def run():
        ssp[0] = hip.stream_resid(x, w, res, wpb, S, tp=h.push_handle())

    def check():
        tot = x.float() @ w.float().t()
        if h.world > 1:
            dist.all_reduce(tot, group=group)
        ref = (res0.float() + tot).to(torch.bfloat16).float()
        good = bool(torch.allclose(res.float(), ref, atol=6e-2, rtol=2e-2))
        ss = res.float().pow(2).reshape(M, N // (16 * wpb), 16 * wpb).sum(-1)
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
        self._lib = _lib()
        self._h = self._lib.mrsum_ar_create(0, 1, self.max_bytes)
        if not self._h:
            raise RuntimeError("LocalPush: allocation failed")

    MAX_ROWS = CustomAllReduce.MAX_ROWS
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


def maybe_custom_all_reduce(group=None, max_bytes: int = 4 << 20) -> Optional[CustomAllReduce]:
    """A CustomAllReduce for ``group`` when every rank is on a GPU, else None (RCCL/gloo path)."""
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
    if not ar.self_test():
        log.warning("custom all-reduce failed its self-test on some rank; using RCCL")
        ar.close()
        return None
    return ar
