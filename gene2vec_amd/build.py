"""Build recipe for ``gene2vec_amd/libg2v.so`` (gfx950 only).

``python -m gene2vec_amd.build`` or ``gene2vec_amd.build.build()``.  The
library is built IN-TREE so it travels with the repository snapshot to the GPU
box; it is git-ignored.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libg2v.so")
SOURCES = ["g2v_kernels.hip", "g2v_api.hip", "g2v_host.cpp", "g2v_ingest.cpp"]
HEADERS = [os.path.join(CSRC, "g2v_internal.h"), os.path.join(ROOT, "include", "g2v.h")]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (need ROCm for gfx950)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + HEADERS + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           # IEEE semantics: every fused multiply-add in the kernels is explicit
           "-ffp-contract=off", "-munsafe-fp-atomics", "-pthread",
           "-I", os.path.join(ROOT, "include"), "-I", CSRC, *srcs, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
