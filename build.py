#!/usr/bin/env python3
"""In-tree build of the native libraries (no pip install, no JIT cache).

* ``_native/libmrsum_kernels.so``: every ``csrc/kernels/*.hip`` compiled by
  ``hipcc --offload-arch=gfx950 -O3`` (gfx950 only -- no other targets, no
  CUDA paths) and linked into one shared object.
* ``_native/libmrsum_runtime.so``: ``csrc/runtime/*.cpp`` host runtime (g++).

Objects are rebuilt when the content hash of their source, the headers of
its directory and the flags differs from the one recorded next to the object
(not by mtime: a snapshot copied to another machine keeps no useful mtimes).
Each library gets a ``<lib>.stamp.json`` (``llm_map_reduce_summarizer_amd/
_stamp.py``): sha256 over its sources + flags, checked by ``ops/_lib.py`` at
load time, which refuses a library built from other sources.
Usage: ``python build.py [--force] [-j N]``.
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from llm_map_reduce_summarizer_amd import _stamp  # noqa: E402  (stdlib only)

PKG = os.path.join(ROOT, "llm_map_reduce_summarizer_amd")
CSRC = _stamp.CSRC
NATIVE = _stamp.NATIVE
OBJ = os.path.join(ROOT, "build", "obj")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
ARCH = _stamp.ARCH
HIP_FLAGS = _stamp.HIP_FLAGS
CXX_FLAGS = _stamp.CXX_FLAGS


def _stale(src: str, dst: str, deps, flags) -> bool:
    """Whether object ``dst`` must be rebuilt: missing, or built from other source/header/flag content."""
    key = _stamp.digest([src] + list(deps), flags)
    try:
        with open(dst + ".sha") as f:
            return not os.path.exists(dst) or f.read().strip() != key
    except OSError:
        return True


def _mark(src: str, dst: str, deps, flags) -> None:
    with open(dst + ".sha", "w") as f:
        f.write(_stamp.digest([src] + list(deps), flags))


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n%s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def _check_resources(src: str, remarks: str) -> None:
    """Fail the build if any kernel spills to scratch (always a bug here: a runtime-indexed or
    address-taken register array -- cdna_hip_programming.md §5.4 rule 20)."""
    fn = None
    bad = []
    for line in remarks.splitlines():
        if "Function Name:" in line:
            fn = line.split("Function Name:")[1].split("[")[0].strip()
        elif "ScratchSize [bytes/lane]:" in line:
            n = int(line.split("ScratchSize [bytes/lane]:")[1].split()[0])
            if n:
                bad.append("%s: %d B/lane" % (fn, n))
    if bad:
        raise RuntimeError("scratch (private memory) in %s:\n  %s" % (os.path.basename(src), "\n  ".join(bad)))


def _compile_hip(job):
    cmd, src, obj, deps = job
    _check_resources(src, _run(cmd))
    _mark(src, obj, deps, HIP_FLAGS)


def build_kernels(force: bool = False, jobs: int = 8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(NATIVE, exist_ok=True)
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(s, o, hdrs, HIP_FLAGS):
            todo.append(([HIPCC] + HIP_FLAGS + ["-I", os.path.join(CSRC, "kernels"), "-c", s, "-o", o], s, o, hdrs))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_compile_hip, todo))
    out = os.path.join(NATIVE, "libmrsum_kernels.so")
    if force or todo or not os.path.exists(out) or _stamp.check("kernels"):
        tmp = out + ".tmp"
        _run([HIPCC, "--offload-arch=%s" % ARCH, "-shared", "-fPIC", "-o", tmp] + objs)
        os.replace(tmp, out)
        _stamp.write_stamp("kernels", {"compiler": _tool_version(HIPCC)})
    return out


def _tool_version(tool: str) -> str:
    try:
        r = subprocess.run([tool, "--version"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=60)
        return " | ".join(ln.strip() for ln in r.stdout.splitlines()[:2])
    except Exception:  # noqa: BLE001 -- informational only
        return "unknown"


def build_runtime(force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    os.makedirs(NATIVE, exist_ok=True)
    out = os.path.join(NATIVE, "libmrsum_runtime.so")
    if force or not os.path.exists(out) or _stamp.check("runtime"):
        tmp = out + ".tmp"
        _run([CXX] + CXX_FLAGS + ["-shared", "-o", tmp] + srcs + ["-lpthread"])
        os.replace(tmp, out)
        _stamp.write_stamp("runtime", {"compiler": _tool_version(CXX)})
    return out


def build_sanitized_stress(sanitizer: str, out_dir: str = None) -> str:
    """Host runtime (csrc/runtime/*.cpp) + csrc/tests/runtime_stress.cpp as one executable under
    ``-fsanitize=<sanitizer>`` (host code only: "address,undefined" or "thread")."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + [os.path.join(CSRC, "tests", "runtime_stress.cpp")]
    tag = sanitizer.replace(",", "_")
    out = os.path.join(out_dir or NATIVE, "runtime_stress_%s" % tag)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    _run([CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=%s" % sanitizer, "-pthread"]
         + srcs + ["-o", out])
    return out


def build_all(force: bool = False, jobs: int = 8, kernels: bool = True) -> None:
    build_runtime(force)
    if kernels:
        if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
            raise RuntimeError("hipcc not found at %s" % HIPCC)
        build_kernels(force, jobs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--runtime-only", action="store_true")
    a = ap.parse_args()
    build_all(a.force, a.jobs, kernels=not a.runtime_only)
    print("built:", ", ".join(sorted(os.listdir(NATIVE))))


if __name__ == "__main__":
    sys.exit(main())
