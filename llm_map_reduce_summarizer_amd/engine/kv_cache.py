"""Paged KV cache sized for 288 GB of HBM per GPU.

Layout per layer: ``k``/``v`` [num_pages, Hkv, P, head_dim] bf16, i.e. a page
holds P consecutive positions of ONE kv head contiguously (16 KiB at P=64,
hd=128) -- the unit the decode-attention workgroups stream.  Page 0 is a
scratch page: idle decode slots point at it, real sequences never do.

``kv_dtype="fp8"``: ``k``/``v`` are uint8 [num_pages, Hkv, SLAB] byte slabs,
SLAB = P * hd + 4 * P -- the P rows of e4m3fn bytes then the P fp32 row scales
of one (page, kv head) (csrc/kernels/kv8.h): 8.25 KiB instead of 16 KiB, so a
decode step streams half the KV bytes and the cache holds ~1.94x the tokens.
``kv_dtype="fp8v"``: only ``v`` is fp8 slabs, ``k`` stays bf16 -- the scores'
K rounding is what peaked attention amplifies (a CPU emulation on the parity
checkpoint: K+V fp8 20 % logit error, V only 6 %, profiles/r4_fp8_kv_emulation.txt),
so this keeps 3/4 of the bf16 bytes at a third of the full variant's error.

Allocation is whole-sequence: a request reserves ceil((prompt + max_new) / P)
pages at admission, so a captured decode graph can run many steps without
the host touching block tables.  The free list is the native C++ allocator
(``csrc/runtime/page_alloc.cpp``) when built, else a Python list with the
same LIFO policy.
"""

from __future__ import annotations

import ctypes
import logging
from typing import List

import torch

from ..ops._lib import runtime_lib

log = logging.getLogger("mrsum.kv")


class PageAllocator:
    def __init__(self, num_pages: int):
        self.num_pages = num_pages
        self._lib = runtime_lib(required=False)
        self._h = None
        if self._lib is not None and hasattr(self._lib, "mrsum_pages_create"):
            L = self._lib
            L.mrsum_pages_create.restype = ctypes.c_void_p
            L.mrsum_pages_create.argtypes = [ctypes.c_int, ctypes.c_int]
            L.mrsum_pages_alloc.restype = ctypes.c_int
            L.mrsum_pages_alloc.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.mrsum_pages_free.restype = ctypes.c_int
            L.mrsum_pages_free.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
            L.mrsum_pages_available.restype = ctypes.c_int
            L.mrsum_pages_available.argtypes = [ctypes.c_void_p]
            L.mrsum_pages_destroy.argtypes = [ctypes.c_void_p]
            self._h = L.mrsum_pages_create(num_pages, 1)
        else:
            self._free = list(range(num_pages - 1, 0, -1))

    @property
    def native(self) -> bool:
        return self._h is not None

    def available(self) -> int:
        if self._h is not None:
            return self._lib.mrsum_pages_available(self._h)
        return len(self._free)

    def alloc(self, n: int) -> List[int]:
        if n <= 0:
            return []
        if self._h is not None:
            buf = (ctypes.c_int * n)()
            if self._lib.mrsum_pages_alloc(self._h, n, buf) != 0:
                raise MemoryError("KV cache exhausted (%d pages requested, %d free)" % (n, self.available()))
            return list(buf)
        if n > len(self._free):
            raise MemoryError("KV cache exhausted (%d pages requested, %d free)" % (n, len(self._free)))
        out = self._free[-n:][::-1]
        del self._free[-n:]
        return out

    def free(self, pages: List[int]) -> None:
        if not pages:
            return
        if self._h is not None:
            buf = (ctypes.c_int * len(pages))(*pages)
            if self._lib.mrsum_pages_free(self._h, len(pages), buf) != 0:
                raise ValueError("double free / bad page id")
            return
        self._free.extend(reversed(pages))

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            try:
                self._lib.mrsum_pages_destroy(self._h)
            except Exception:
                pass
            self._h = None


KV_DTYPES = ("bf16", "fp8", "fp8v")


class PagedKVCache:
    def __init__(self, n_layers: int, num_pages: int, n_kv_heads: int, page: int, head_dim: int,
                 dtype: torch.dtype, device: torch.device, kv_dtype: str = "bf16"):
        if num_pages < 2:
            raise ValueError("need at least 2 KV pages (page 0 is scratch)")
        if kv_dtype not in KV_DTYPES:
            raise ValueError("kv_dtype must be one of %s" % (KV_DTYPES,))
        if kv_dtype != "bf16" and (page, head_dim) != (64, 128):
            raise ValueError("the fp8 KV cache needs page 64 and head dim 128")
        self.page = page
        self.num_pages = num_pages
        self.kv_dtype = kv_dtype
        shape16, dt16 = (n_layers, num_pages, n_kv_heads, page, head_dim), dtype
        from ..ops.reference import kv8_slab
        shape8 = (n_layers, num_pages, n_kv_heads, kv8_slab(page, head_dim)) if kv_dtype != "bf16" else None
        kshape, kdt = (shape8, torch.uint8) if kv_dtype == "fp8" else (shape16, dt16)
        vshape, vdt = (shape8, torch.uint8) if kv_dtype in ("fp8", "fp8v") else (shape16, dt16)
        # zeroed, not empty: attention kernels read whole pages and mask the scores of rows past a
        # sequence's end (p = 0), and 0 x a stale NaN bit pattern in such a V row would still be NaN
        self.k = torch.zeros(kshape, dtype=kdt, device=device)
        self.v = torch.zeros(vshape, dtype=vdt, device=device)
        self.alloc = PageAllocator(num_pages)
        log.info("KV cache: %d pages x %d tokens (%.1f GiB)", num_pages, page,
                 (self.k.numel() * self.k.element_size() + self.v.numel() * self.v.element_size()) / 2 ** 30)

    def pages_for(self, n_tokens: int) -> int:
        return -(-n_tokens // self.page)

    @property
    def fp8(self) -> bool:
        """Any fp8 slab cache (K and V, or V only)."""
        return self.kv_dtype != "bf16"

    @staticmethod
    def size_pages(bytes_budget: int, n_layers: int, n_kv_heads: int, page: int, head_dim: int,
                   dtype_bytes: int = 2, kv_dtype: str = "bf16") -> int:
        bf, f8 = page * head_dim * dtype_bytes, page * head_dim + 4 * page
        per_head = {"bf16": 2 * bf, "fp8": 2 * f8, "fp8v": bf + f8}[kv_dtype]
        per_page = n_layers * n_kv_heads * per_head
        return max(2, bytes_budget // per_page)
