"""Simulate N data-parallel replicas on one GPU (the bench's N>1 scheme:
contiguous shards, per-rank model.random seeds, average both tables every
A jobs) and compare the held-in SGNS objective with a single model trained
on all pairs (iterations = gene2vec sawtooth epochs)."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from gene2vec_amd import _native as N, engine as E, synthetic as S, distributed as Dd
from oracle import sgns_oracle as O
NP = int(sys.argv[1]); ITERS = int(sys.argv[2]); NREP = int(sys.argv[3])
V0, D, K, sample = 24447, 200, 5, 1e-3
pairs = S.zipf_gene_pairs(NP, V0, 1.0); flat = pairs.reshape(-1)
counts, first = E.count_ids(flat, V0); order, remap = S.vocab_order(counts, first)
V = len(order); vc = counts[order]; tok = remap[flat]
rng = np.random.Generator(np.random.PCG64(1)); syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
def evl(s0, s1, n_eval=50000, seed=99):
    r = np.random.Generator(np.random.PCG64(seed)); idx = r.integers(0, NP, n_eval)
    c, j = tok[2 * idx], tok[2 * idx + 1]; p = vc.astype(np.float64) ** 0.75
    negs = r.choice(V, size=(n_eval, K), p=p / p.sum()); return O.sgns_loss(s0, s1, c, j, negs)
dev = torch.device("cuda", 0)
def run(nrep, avg_every, merge='mean'):
    engs, tabs, shards = [], [], []
    for r in range(nrep):
        s0, s1 = Dd.shard_range(NP, r, nrep)
        e = E.SGNSEngine(V, D, K); e.set_vocab(vc, sample)
        t0 = torch.zeros((V, e.ld), device=dev); t1 = torch.zeros((V, e.ld), device=dev)
        t0[:, :D] = torch.from_numpy(syn0).to(dev)
        torch.cuda.synchronize()
        e.bind_tables(t0.data_ptr(), t1.data_ptr(), e.ld, keepalive=(t0, t1))
        e.set_corpus(tok[2 * s0:2 * s1], sent_len=2)
        js = E.plan_jobs(n_sent=s1 - s0, sent_len=2)
        engs.append(e); tabs.append((t0, t1)); shards.append((js, E.job_alphas(js, s1 - s0), np.random.RandomState(Dd.rank_seed(1, r))))
    out = []
    old = [tabs[0][k].clone() for k in range(2)]
    for it in range(ITERS):
        seeds = [E.job_seeds(rs, len(js) - 1) for js, _, rs in shards]
        nj = max(len(js) - 1 for js, _, _ in shards)
        for j0 in range(0, nj, avg_every):
            for r in range(nrep):
                js, al, _ = shards[r]
                j1 = min(len(js) - 1, j0 + avg_every)
                if j1 > j0:
                    engs[r].train(js[j0:j1 + 1], al[j0:j1], seeds[r][j0:j1], N.MODE_HOGWILD)
            for r in range(nrep):
                engs[r].sync()
            if nrep > 1:
                for k in range(2):
                    st = torch.stack([tabs[r][k] for r in range(nrep)])
                    if merge == 'mean':
                        m = st.mean(0)
                    else:
                        d = st - old[k]
                        if merge == 'sum':
                            m = old[k] + d.sum(0)
                        else:  # touch: per-row sum / #replicas that changed the row (^beta)
                            cnt = (d != 0).any(dim=2).sum(0).clamp(min=1).to(d.dtype)
                            beta = 0.5 if merge == 'sqrt' else 1.0
                            m = old[k] + d.sum(0) / cnt[:, None] ** beta
                    old[k].copy_(m)
                    for r in range(nrep):
                        tabs[r][k].copy_(m)
                torch.cuda.synchronize()
        out.append(evl(tabs[0][0][:, :D].cpu().numpy(), tabs[0][1][:, :D].cpu().numpy()))
    for e in engs: e.close()
    return out
base = run(1, 10**9)
print("single   ", " ".join("%.4f" % x for x in base), flush=True)
njobs = (NP // NREP) // 5000
for spec in sys.argv[4].split(","):
    per_epoch, merge = spec.split(":")
    per_epoch = int(per_epoch)
    a = max(1, njobs // per_epoch)
    res = run(NREP, a, merge)
    print(f"N={NREP} avg/epoch={per_epoch:3d} {merge:5s}", " ".join("%.4f" % x for x in res), flush=True)
