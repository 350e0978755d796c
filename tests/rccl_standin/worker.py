"""One rank of the two-rank transport tests (tests/test_gpu_rccl_standin.py):
a libg2v replica on cuda:0 trains its contiguous shard of a Zipf pair corpus
with in-call merges (distributed.ReplicaTrainer, backend libg2v) over
  --transport rccl  g2v_comm_init: libg2v's kCommRccl lines, carried by the
                    RCCL stand-in when G2V_RCCL_LIB names it
  --transport host  g2v_comm_init_host over gloo (distributed.HostCollective)
gloo (CPU) bootstraps: the unique id and ReplicaTrainer's agreements.  Writes
<out>_rank<r>.npz (final tables) and <out>_rank<r>.json (status)."""
import argparse
import ctypes
import json
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--transport", choices=("rccl", "host"), required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--fail-merge", type=int, default=0, help="rank 1: G2V_OPT_DEBUG_FAIL_MERGE")
    ap.add_argument("--mode", choices=("sequential", "hogwild"), default="sequential")
    ap.add_argument("--rule", choices=("touch", "mean", "align"), default="touch")
    ap.add_argument("--iters", type=int, default=2)
    a = ap.parse_args()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port), RANK=str(a.rank),
                      WORLD_SIZE=str(a.world))
    import torch.distributed as dist

    from gene2vec_amd import _native as N
    from gene2vec_amd import distributed as Dd
    from gene2vec_amd import engine as E
    from gene2vec_amd import synthetic as S
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    status = {"ok": False, "error": None}
    t0 = time.time()
    try:
        V0, D, K, n = 1500, 64, 5, 240_000
        pairs = S.zipf_gene_pairs(n, V0, 1.0, seed=21)
        flat = pairs.reshape(-1)
        counts, first = E.count_ids(flat, V0)
        order, remap = S.vocab_order(counts, first)
        tok = remap[flat]
        V = len(order)
        s0, s1 = Dd.shard_range(n, a.rank, a.world)
        eng = E.SGNSEngine(V, D, K, device=0)
        eng.set_vocab(counts[order].astype(np.int64), 1e-3)
        rng = np.random.Generator(np.random.PCG64(5 + a.rank))  # rank 0's init wins
        eng.set_weights(((rng.random((V, D)) - 0.5) / D).astype(np.float32),
                        np.zeros((V, D), np.float32))
        eng.set_corpus(tok[2 * s0:2 * s1], sent_len=2)
        if a.transport == "rccl":
            box = [eng.comm_unique_id() if a.rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            eng.comm_init(box[0], a.world, a.rank)
        else:
            eng.comm_init_host(Dd.host_collective(), a.world, a.rank)
        if a.fail_merge and a.rank == 1:
            eng.set_option(N.OPT_DEBUG_FAIL_MERGE, a.fail_merge)
        mode = N.MODE_SEQUENTIAL if a.mode == "sequential" else N.MODE_HOGWILD
        tr = Dd.ReplicaTrainer(eng, (), 8, mode, merge=a.rule, backend="libg2v")
        rs = np.random.RandomState(1 + a.rank)
        js = E.plan_jobs(n_sent=s1 - s0, sent_len=2)
        al = E.job_alphas(js, s1 - s0)
        for _ in range(a.iters):
            tr.train_epoch(js, al, E.job_seeds(rs, len(js) - 1))
        eng.sync()
        w0, w1 = eng.get_weights()
        np.savez(f"{a.out}_rank{a.rank}.npz", syn0=w0, syn1neg=w1)
        status.update(ok=True, merges=tr.averages)
    except Exception as e:  # noqa: BLE001 - reported to the test
        status["error"] = f"{type(e).__name__}: {e}"
        status["trace"] = traceback.format_exc()[-3000:]
    status["seconds"] = round(time.time() - t0, 2)
    lib = os.environ.get("G2V_RCCL_LIB")
    if lib:
        status["standin_calls"] = int(ctypes.CDLL(lib).g2v_rccl_standin_calls())
    with open(f"{a.out}_rank{a.rank}.json", "w") as f:
        json.dump(status, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
