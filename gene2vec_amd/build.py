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
K_COMPILED = tuple(range(1, 21))  # == G2V_FOR_EACH_K in g2v_internal.h
# (source, extra defines, object name): the SGNS kernels are built once per K
UNITS = ([("g2v_sgns_atomic.hip", [f"-DG2V_K={k}"], f"g2v_sgns_atomic_k{k}.o") for k in K_COMPILED]
         + [("g2v_sgns.hip", [f"-DG2V_K={k}"], f"g2v_sgns_k{k}.o") for k in K_COMPILED]
         + [(s, [], os.path.splitext(s)[0] + ".o")
            for s in ("g2v_kernels.hip", "g2v_api.hip", "g2v_coexpr.hip", "g2v_host.cpp",
                      "g2v_ingest.cpp", "g2v_export.cpp")])
SOURCES = sorted({u[0] for u in UNITS})
HEADERS = [os.path.join(CSRC, "g2v_internal.h"), os.path.join(CSRC, "g2v_device.h"),
           os.path.join(ROOT, "include", "g2v.h")]
ARCH = "gfx950"
# k_sgns_atomic's store-or-atomics choice per row is a uniform if / else that
# must stay a diamond for the loop head to wait with vmcnt(#row instructions)
# instead of vmcnt(0) (g2v_sgns_atomic.hip; tests/test_kernel_isa.py)
SGNS_KERNEL_FLAGS = ("-mllvm", "-structurizecfg-skip-uniform-regions=true")
# the sources that determine k_sgns_atomic's code (bench.py accepts a PMC
# traffic profile only when it was measured on this exact kernel code AND the
# same launch layout: grid and stripe tiers, recorded beside the hash)
KERNEL_SOURCES = [os.path.join(CSRC, s) for s in
                  ("g2v_sgns_atomic.hip", "g2v_device.h", "g2v_internal.h")]


def kernel_source_hash() -> str:
    """sha256 (first 16 hex digits) of KERNEL_SOURCES, in that order"""
    import hashlib
    h = hashlib.sha256()
    for p in KERNEL_SOURCES:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (need ROCm for gfx950)")


# the throughput-ablation build (G2V_OPT_DEBUG_WRITE 1, 3-7, 9):
# the same sources with -DG2V_ABLATIONS, a library of its own that is never
# shipped or loaded by the product (scripts load it with _native.use_library)
ABLATIONS_LIB = os.path.join(HERE, "libg2v_ablations.so")


def _stale(lib=LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + HEADERS + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, ablations: bool = False,
          defines=(), tag: str = "", kernel_flags=()) -> str:
    """Compile every translation unit in parallel (one hipcc per file), then link.
    ablations=True: the -DG2V_ABLATIONS library (ABLATIONS_LIB) instead;
    tag + defines: an experiment build gene2vec_amd/libg2v_exp_<tag>.so with
    extra -D flags and extra compiler flags for the SGNS-kernel units
    (kernel_flags; A/B scripts load it with _native.use_library; never the
    product)"""
    if tag:
        out = os.path.join(HERE, f"libg2v_exp_{tag}.so")
        objdir = os.path.join(HERE, "build", f"exp_{tag}")
    elif ablations:
        out, objdir = ABLATIONS_LIB, os.path.join(HERE, "build", "ablations")
    else:
        out, objdir = LIB, os.path.join(HERE, "build")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             # IEEE semantics: every fused multiply-add in the kernels is explicit
             "-ffp-contract=off", "-munsafe-fp-atomics", "-pthread",
             "-I", os.path.join(ROOT, "include"), "-I", CSRC]
    if ablations:
        flags.append("-DG2V_ABLATIONS")
    flags += [f"-D{d}" for d in defines]
    # the objects' compile flags are part of their key: a stamp in
    # the object directory; another flag set rebuilds every object there
    stamp = os.path.join(objdir, "flags.stamp")
    key = " ".join(flags + ["|"] + list(SGNS_KERNEL_FLAGS) + list(kernel_flags))
    old_key = open(stamp).read() if os.path.exists(stamp) else None
    if old_key is not None and old_key != key:
        force = True
    if not force and not _stale(out):
        return out
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, u[2]) for u in UNITS]

    def compile_one(i):
        src, defs, _ = UNITS[i]
        deps = [os.path.join(CSRC, src)] + HEADERS + [__file__]
        if (not force and os.path.exists(objs[i])
                and all(os.path.getmtime(d) <= os.path.getmtime(objs[i]) for d in deps)):
            return ""
        kf = (list(SGNS_KERNEL_FLAGS) + list(kernel_flags)) if src == "g2v_sgns_atomic.hip" else []
        cmd = [hipcc(), *flags, *kf, *defs, "-c", os.path.join(CSRC, src), "-o", objs[i]]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"hipcc failed on {src} {defs}:\n{r.stderr}")
        return r.stderr

    jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(UNITS), os.cpu_count() or 1, 16)
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for err in ex.map(compile_one, range(len(UNITS))):
            if err and verbose:
                print(err, file=sys.stderr)
    with open(stamp, "w") as f:
        f.write(key)
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", *objs, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, ablations="--ablations" in sys.argv))


EXAMPLES = os.path.join(os.path.dirname(HERE), "examples")


def build_examples(verbose=False):
    """examples/g2v_train: a Python-free host of the C ABI (gcc, links libg2v.so
    through an rpath relative to the binary)."""
    src = os.path.join(EXAMPLES, "g2v_train.c")
    out = os.path.join(EXAMPLES, "g2v_train")
    lib = os.path.join(HERE, "libg2v.so")
    header = os.path.join(os.path.dirname(HERE), "include", "g2v.h")
    if (os.path.exists(out)
            and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in (src, lib, header))):
        return out
    cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Wextra",
           "-I", os.path.join(os.path.dirname(HERE), "include"), src, "-L", HERE, "-lg2v",
           "-Wl,-rpath,$ORIGIN/../gene2vec_amd", "-o", out]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"gcc failed on {src}:\n{r.stderr}")
    return out
