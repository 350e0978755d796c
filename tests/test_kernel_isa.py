"""CPU (hipcc cross-compiles gfx950): the production Hogwild kernel keeps its
pipeline in the generated assembly.

k_sgns_atomic loads example e+1's rows before it issues example e's 4 NV
(K+2) row updates (float atomics, or plain stores for cold rows), and the
loop head must wait for those loads with vmcnt(4 NV (K+2)) -- the updates
retiring behind the next compute -- not vmcnt(0).  The store-or-atomics
choice is an if / else that keeps that count only under the build's
-structurizecfg-skip-uniform-regions; without it the wait
drops to vmcnt(0).  This compiles the K = 5 unit exactly as build.py does and
reads the wait at the head of the example loop of k_sgns_atomic<5, 1, 0>."""
import os
import re
import subprocess

import pytest

from gene2vec_amd import build as B

INSTANCE = "_ZN3g2v13k_sgns_atomicILi5ELi1ELi0ELb0EEEvNS_8SgnsArgsE"


def _asm(tmp_path, extra=()):
    out = str(tmp_path / "k5.s")
    cmd = [B.hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-ffp-contract=off",
           "-munsafe-fp-atomics", "-I", os.path.join(B.ROOT, "include"), "-I", B.CSRC,
           "-DG2V_K=5", *extra, "--cuda-device-only", "-S",
           os.path.join(B.CSRC, "g2v_sgns_atomic.hip"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return open(out).read()


def _loop_head_waits(asm):
    i = asm.index(INSTANCE + ":")
    body = asm[i:asm.index(".Lfunc_end", i)].splitlines()
    head = next(k for k, ln in enumerate(body) if "This Loop Header: Depth=2" in ln)
    first_dot = next(k for k in range(head, len(body)) if "v_fma_f64" in body[k])
    return [int(m.group(1)) for ln in body[head:first_dot]
            for m in [re.search(r"s_waitcnt vmcnt\((\d+)\)", ln)] if m]


@pytest.mark.timeout(900)
def test_loop_head_waits_for_loads_not_for_updates(tmp_path):
    waits = _loop_head_waits(_asm(tmp_path, B.SGNS_KERNEL_FLAGS))
    # 4 NV (K + 2) = 28 row-update instructions may stay in flight
    assert 28 in waits, waits


@pytest.mark.timeout(900)
def test_default_structurizer_would_drain(tmp_path):
    """the reason for the flag: without it the same source drains every update"""
    waits = _loop_head_waits(_asm(tmp_path))
    assert 28 not in waits and 0 in waits, waits
