#!/usr/bin/env python3
"""Build the kernel library of an earlier commit for a same-box A/B: the ``csrc/kernels`` sources of git
ref REF are compiled (same hipcc flags as build.py) into ``_native/libmrsum_kernels_<TAG>.so``, which a
run selects with ``MRSUM_KERNELS_SO`` (ops/_lib.py).  Only for kernel changes that keep every launcher
signature.

    python tools/build_ab.py HEAD~1 base
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import build  # noqa: E402


def main():
    ref, tag = sys.argv[1], sys.argv[2]
    kdir = "llm_map_reduce_summarizer_amd/csrc/kernels"
    with tempfile.TemporaryDirectory() as td:
        if os.path.isdir(ref):  # a directory of (patched) kernel sources instead of a git ref
            names = sorted(os.listdir(ref))
            for n in names:
                with open(os.path.join(ref, n), "rb") as fi, open(os.path.join(td, n), "wb") as f:
                    f.write(fi.read())
        else:
            names = subprocess.check_output(["git", "-C", ROOT, "ls-tree", "--name-only", ref, kdir + "/"],
                                            text=True).split()
            for n in names:
                with open(os.path.join(td, os.path.basename(n)), "wb") as f:
                    f.write(subprocess.check_output(["git", "-C", ROOT, "show", "%s:%s" % (ref, n)]))
        objs = []
        for n in names:
            if not n.endswith(".hip"):
                continue
            src = os.path.join(td, os.path.basename(n))
            obj = src + ".o"
            build._run([build.HIPCC] + build.HIP_FLAGS + ["-I", td, "-c", src, "-o", obj])
            objs.append(obj)
        out = os.path.join(build.NATIVE, "libmrsum_kernels_%s.so" % tag)
        build._run([build.HIPCC, "--offload-arch=%s" % build.ARCH, "-shared", "-fPIC", "-o", out] + objs)
    print(out)


if __name__ == "__main__":
    main()
