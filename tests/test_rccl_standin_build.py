"""CPU: the test-only RCCL stand-in (tests/rccl_standin) builds, loads and
exports every entry point libg2v's rccl() binds (g2v_api.hip), and two
processes can form and abort a communicator through it (no GPU calls: the
collectives themselves run in tests/test_gpu_rccl_standin.py)."""
import ctypes as C
import multiprocessing as mp
import os
import re

from tests.rccl_standin import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_standin_exports_what_libg2v_binds():
    lib = C.CDLL(B.build())
    src = open(os.path.join(ROOT, "gene2vec_amd", "csrc", "g2v_api.hip")).read()
    bound = set(re.findall(r'dlsym\(h, "(nccl\w+)"\)', src)) | set(
        re.findall(r'sym\(r\.\w+, "(nccl\w+)"\)', src))
    assert {"ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclBroadcast",
            "ncclGroupStart", "ncclGroupEnd", "ncclCommDestroy", "ncclCommAbort"} <= bound
    for name in bound:
        assert hasattr(lib, name), name


class Uid(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


def _rank(path, uid_bytes, rank, q, abort, inited):
    lib = C.CDLL(path)
    comm = C.c_void_p()
    uid = Uid.from_buffer_copy(uid_bytes)
    rc = lib.ncclCommInitRank(C.byref(comm), 2, uid, rank)
    q.put((rank, "init", rc))
    inited[rank].set()
    if rc == 0:
        if abort:
            # abort only once the peer is out of its init barrier: an abort
            # while it still waits there fails its init (the stand-in's
            # documented semantics), which is not what this test checks
            inited[1 - rank].wait(60)
        rc2 = (lib.ncclCommAbort if abort else lib.ncclCommDestroy)(comm)
        q.put((rank, "end", rc2))


def test_two_processes_form_and_leave_a_communicator():
    path = B.build()
    lib = C.CDLL(path)
    uid = Uid()
    assert lib.ncclGetUniqueId(C.byref(uid)) == 0
    assert uid.internal.startswith(b"/g2v_rccl_standin_")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    inited = [ctx.Event(), ctx.Event()]
    ps = [ctx.Process(target=_rank, args=(path, bytes(uid), r, q, r == 1, inited))
          for r in range(2)]
    for p in ps:
        p.start()
    got = [q.get(timeout=60) for _ in range(4)]
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert sorted(got) == [(0, "end", 0), (0, "init", 0), (1, "end", 0), (1, "init", 0)]
