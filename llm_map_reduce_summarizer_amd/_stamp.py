"""Build provenance of the in-tree native libraries (stdlib only: ``build.py`` imports it before torch).

``build.py`` writes ``<lib>.stamp.json`` next to each shared object it links: a sha256 over the
sources it was compiled from (every ``csrc/kernels/*.hip`` + ``*.h``, or ``csrc/runtime/*.cpp``; file
names and contents) and over the compiler flags, plus the flags themselves.  ``ops/_lib.py`` recomputes
the hash from the tree at load time and refuses a library whose stamp differs -- so a box that received
a prebuilt ``_native/*.so`` together with newer sources fails loudly instead of running stale kernels.
"""

from __future__ import annotations

import glob
import hashlib
import json
import os
from typing import Dict, List, Optional

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
NATIVE = os.path.join(PKG, "_native")

ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIP_FLAGS = ["--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
             "-mcode-object-version=5", "-Wno-unused-result", "-munsafe-fp-atomics",
             "-Rpass-analysis=kernel-resource-usage"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-sign-compare"]

LIBS = {
    "kernels": ("libmrsum_kernels.so", ("kernels/*.hip", "kernels/*.h"), HIP_FLAGS),
    "runtime": ("libmrsum_runtime.so", ("runtime/*.cpp",), CXX_FLAGS),
}


def sources(kind: str) -> List[str]:
    _, pats, _ = LIBS[kind]
    out: List[str] = []
    for p in pats:
        out.extend(glob.glob(os.path.join(CSRC, p)))
    return sorted(out)


def digest(paths: List[str], flags: List[str]) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update("\0".join(flags).encode())
    return h.hexdigest()


def tree_stamp(kind: str) -> str:
    """sha256 of the sources + flags the library of ``kind`` must be built from (this tree)."""
    _, _, flags = LIBS[kind]
    return digest(sources(kind), flags)


def stamp_path(kind: str) -> str:
    return os.path.join(NATIVE, LIBS[kind][0] + ".stamp.json")


def write_stamp(kind: str, extra: Optional[Dict] = None) -> Dict:
    _, _, flags = LIBS[kind]
    rec = {"lib": LIBS[kind][0], "sources_sha256": tree_stamp(kind), "flags": list(flags),
           "files": [os.path.relpath(p, PKG) for p in sources(kind)]}
    rec.update(extra or {})
    tmp = stamp_path(kind) + ".tmp"
    with open(tmp, "w") as f:
        json.dump(rec, f, indent=1)
    os.replace(tmp, stamp_path(kind))
    return rec


def read_stamp(kind: str) -> Optional[Dict]:
    try:
        with open(stamp_path(kind)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def check(kind: str) -> Optional[str]:
    """None when the built library of ``kind`` matches this tree, else why not."""
    rec = read_stamp(kind)
    if rec is None:
        return "no build stamp %s (built by an older build.py?): run `python build.py`" % stamp_path(kind)
    want = tree_stamp(kind)
    if rec.get("sources_sha256") != want:
        return ("%s was built from other sources (stamp %s, tree %s): run `python build.py`"
                % (LIBS[kind][0], str(rec.get("sources_sha256"))[:16], want[:16]))
    return None
