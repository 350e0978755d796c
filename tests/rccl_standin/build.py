"""Build recipe of the TEST-ONLY RCCL stand-in (g2v_rccl_standin.cpp ->
libg2v_rccl_standin.so, in-tree so it travels to the GPU box; git-ignored).
Called by __graft_entry__.build() and by the tests that load it."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "g2v_rccl_standin.cpp")
LIB = os.path.join(HERE, "libg2v_rccl_standin.so")


def build(force=False):
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    from gene2vec_amd.build import hipcc
    tmp = LIB + ".tmp"
    subprocess.run([hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", SRC, "-o", tmp, "-lrt"],
                   check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
