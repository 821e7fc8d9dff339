"""One-shot P2P all-reduce for latency-bound tensor-parallel decode.

RCCL's ring/tree all-reduce costs tens of microseconds for the B x 16 KiB messages of a TP decode
step, two per layer.  ``CustomAllReduce`` keeps one uncached, IPC-shared buffer per rank
(csrc/kernels/custom_ar.hip): every rank writes its input into its own buffer, flags every peer,
and then sums all peers' buffers directly over xGMI -- one kernel, no host involvement, legal
inside a hipGraph.  Handles are exchanged once through the group (any backend); messages larger
than ``max_bytes`` or non-fp32 tensors go to ``torch.distributed.all_reduce`` (RCCL).

The reference has no collective of any kind (its only "communication" is HTTPS, reference
llm_executor.py:290-297); this is the MI355X replacement for the TP reduce path it implies.
"""

from __future__ import annotations

import ctypes
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
    "mrsum_ar_error": ([ctypes.c_void_p], ctypes.c_int),
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

    def __init__(self, group=None, max_bytes: int = 1 << 20):
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
            ok &= self.error() == 0
        except Exception as e:  # keep the collective sequence aligned across ranks
            log.warning("custom all-reduce self-test raised: %s", e)
            ok = False
        votes = [None] * self.world
        dist.all_gather_object(votes, ok, group=self.group)
        return all(votes)

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


def maybe_custom_all_reduce(group=None, max_bytes: int = 1 << 20) -> Optional[CustomAllReduce]:
    """A CustomAllReduce for ``group`` when every rank is on a GPU, else None (RCCL/gloo path)."""
    if not (dist.is_initialized() and torch.cuda.is_available()):
        return None
    try:
        ar = CustomAllReduce(group, max_bytes)
    except Exception as e:  # no IPC (e.g. container without dmabuf): fall back to RCCL
        log.warning("custom all-reduce unavailable, using RCCL: %s", e)
        return None
    if not ar.self_test():
        log.warning("custom all-reduce failed its self-test on some rank; using RCCL")
        ar.close()
        return None
    return ar
