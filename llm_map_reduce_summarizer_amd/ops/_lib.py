"""Loading of the in-tree native libraries.

Two shared objects are built by ``build.py`` (``python build.py`` or
``__graft_entry__.build()``) into ``llm_map_reduce_summarizer_amd/_native/``:

* ``libmrsum_kernels.so`` -- every HIP/CDNA4 kernel (hipcc --offload-arch=gfx950),
  exposed through ``extern "C"`` launchers that take raw device pointers and a
  ``hipStream_t``.  Launchers enqueue on the caller's stream, never allocate and
  never synchronise, so they are legal inside hipGraph capture.
* ``libmrsum_runtime.so`` -- host C++ runtime: BPE merge loop, paged-KV block
  allocator, batch packing for the scheduler.

``torch`` must be imported before the kernel library is loaded: both torch and
our library link ``libamdhip64.so.7`` (same SONAME), and loading torch first
makes the dynamic loader bind ours to torch's already-mapped HIP runtime so
streams and device pointers are shared.

Provenance: each library carries ``<lib>.stamp.json`` (``_stamp.py``: sha256 of
the sources + flags it was built from); the default in-tree libraries are
refused when that stamp does not match this tree's sources, so stale binaries
never run silently.

On a machine with a GPU the kernel library is REQUIRED (``kernels_lib()``
raises if it is missing) -- there is deliberately no silent PyTorch fallback
for the hot path.  The pure-PyTorch reference ops (``ops/reference.py``) run
only on CPU tensors (CPU tests) and as the numerics oracle of the GPU tests.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

from .. import _stamp

NATIVE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native")
# MRSUM_KERNELS_SO: an alternative build of the kernel library (A/B experiments of two kernel versions
# in one process tree); default the in-tree build
_KERNELS_OVERRIDE = os.environ.get("MRSUM_KERNELS_SO")
KERNELS_SO = _KERNELS_OVERRIDE or os.path.join(NATIVE_DIR, "libmrsum_kernels.so")
RUNTIME_SO = os.path.join(NATIVE_DIR, "libmrsum_runtime.so")

_lock = threading.Lock()
_kernels: Optional[ctypes.CDLL] = None
_runtime: Optional[ctypes.CDLL] = None
_runtime_tried = False


class NativeLibraryMissing(RuntimeError):
    pass


def kernels_lib() -> ctypes.CDLL:
    """The HIP kernel library; raises if it has not been built."""
    global _kernels
    if _kernels is not None:
        return _kernels
    with _lock:
        if _kernels is None:
            import torch  # noqa: F401  (bind libamdhip64 to torch's copy first)
            if not os.path.isfile(KERNELS_SO):
                raise NativeLibraryMissing(
                    "%s not found: run `python build.py` (hipcc --offload-arch=gfx950) first" % KERNELS_SO)
            if not _KERNELS_OVERRIDE:  # an explicit A/B build carries its own provenance
                why = _stamp.check("kernels")
                if why:
                    raise NativeLibraryMissing("refusing a stale kernel library: " + why)
            _kernels = ctypes.CDLL(KERNELS_SO, mode=ctypes.RTLD_LOCAL)
    return _kernels


def runtime_lib(required: bool = True) -> Optional[ctypes.CDLL]:
    """The host C++ runtime library (None if missing and not required)."""
    global _runtime, _runtime_tried
    if _runtime is not None:
        return _runtime
    with _lock:
        if _runtime is None and not _runtime_tried:
            _runtime_tried = True
            if os.path.isfile(RUNTIME_SO):
                why = _stamp.check("runtime")
                if why and required:
                    raise NativeLibraryMissing("refusing a stale runtime library: " + why)
                if not why:
                    _runtime = ctypes.CDLL(RUNTIME_SO, mode=ctypes.RTLD_LOCAL)
    if _runtime is None and required:
        raise NativeLibraryMissing("%s not found or stale: run `python build.py` first" % RUNTIME_SO)
    return _runtime


def native_stamps() -> dict:
    """{kind: stamp record + "matches_tree"} of the in-tree libraries (smoke() prints it)."""
    out = {}
    for kind in _stamp.LIBS:
        rec = dict(_stamp.read_stamp(kind) or {})
        rec.pop("files", None)
        rec["matches_tree"] = _stamp.check(kind) is None
        out[kind] = rec
    return out
