"""GPU: data-parallel merge machinery at the production cadence, reduced from
C3: the SGNS objectives only.

C3 = 8 ranks x 125 M pairs, a touch merge every 3,584 jobs (the default) =
every 17.9 M pairs per rank, i.e. 7 merges per epoch.  Here a tenth of it: 8
replicas on one GPU through the in-process group (libg2v's merge kernels and
in-call merges, the production path of ReplicaTrainer), 8 x 12.5 M pairs of a
structureless Zipf corpus, a merge every 410 jobs (the same 7 merges per
epoch), the reference's alpha sawtooth over 2 iterations, against one model
trained on the same permuted pairs.  Gate: the SGNS objective on the training
pairs (held-in) and on a fresh draw of the generator (held-out) within 1 % of
the one model's (measured +0.18 % / +0.09 %) -- the merge converges.

This is NOT the north star's quality claim: at 12.5 M pairs per replica the
manuscript target function of merged replicas lags one model by 2.6-8 % on a
corpus with planted modules whatever the rule and cadence,
which is why the CLI does not shard below --dp-min-pairs-per-rank = 80 M.  The
target function within 1 % is gated at C3's full size, 8 x 125 M pairs, and
at 8 x 50 M pairs with the align plan by tests/test_gpu_c3_quality.py."""
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import distributed as Dd
from gene2vec_amd import engine as E
from gene2vec_amd import synthetic as S

pytestmark = pytest.mark.gpu


def _heldin(s0, s1, tok, counts, K, n=40000, seed=99):
    rng = np.random.Generator(np.random.PCG64(seed))
    idx = rng.integers(0, len(tok) // 2, n)
    return _objective(s0, s1, tok[2 * idx], tok[2 * idx + 1], counts, K, seed + 1)


def _objective(s0, s1, c, j, counts, K, seed=98):
    rng = np.random.Generator(np.random.PCG64(seed))
    p = counts.astype(np.float64) ** 0.75
    negs = rng.choice(len(counts), size=(len(c), K), p=p / p.sum())
    u = s0[j].astype(np.float64)
    pos = np.einsum("nd,nd->n", u, s1[c].astype(np.float64))
    neg = np.einsum("nd,nkd->nk", u, s1[negs].astype(np.float64))
    return float((np.logaddexp(0, -pos) + np.logaddexp(0, neg).sum(1)).mean())


def test_eight_replicas_within_one_percent_of_one_model():
    import torch
    R, per, V0, D, K, iters, every = 8, 12_500_000, 24447, 200, 5, 2, 410
    pairs = np.concatenate([S.zipf_gene_pairs(per, V0, 1.0, seed=20250114, shard=r)
                            for r in range(R)])
    n = len(pairs)
    flat = pairs.reshape(-1)
    counts, first = E.count_ids(flat, V0)
    order, remap = S.vocab_order(counts, first)
    tok = remap[flat]
    vc = counts[order].astype(np.int64)
    V = len(order)
    names = S.gene_names(V0)
    syn0 = E.seeded_vectors(
        np.array([zlib.crc32((names[i] + "1").encode()) for i in order], np.uint32), D)
    dev = torch.device("cuda", 0)
    base = torch.from_numpy(tok.view(np.int64)).to(dev)
    perm = torch.empty_like(base)
    st = torch.cuda.current_stream(dev)
    perm_seeds = [1234567 + 17 * it for it in range(iters)]

    def permute(it):
        E.permute_items8(0, base.data_ptr(), perm.data_ptr(), n, 0, n, perm_seeds[it],
                         st.cuda_stream)
        st.synchronize()

    # one model over all pairs
    single = E.SGNSEngine(V, D, K)
    single.set_vocab(vc, 1e-3)
    single.set_weights(syn0, np.zeros_like(syn0))
    js = E.plan_jobs(n_sent=n, sent_len=2)
    al = E.job_alphas(js, n)
    rs = np.random.RandomState(1)
    for it in range(iters):
        permute(it)
        single.set_corpus_device(perm.data_ptr(), 2 * n, sent_len=2, keepalive=perm)
        single.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD)
        single.sync()
    ho = S.zipf_gene_pairs(40000, V0, 1.0, seed=777)
    hc, hj = remap[ho[:, 0]], remap[ho[:, 1]]
    w_single = single.get_weights()
    l_single = _heldin(*w_single, tok, vc, K)
    o_single = _objective(*w_single, hc, hj, vc, K)
    single.close()

    # R replicas, libg2v merge every `every` jobs
    grp = E.LocalGroup(R)
    agree = Dd.ThreadAgreement(R)
    engs = []
    for _ in range(R):
        e = E.SGNSEngine(V, D, K)
        e.set_vocab(vc, 1e-3)
        e.set_weights(syn0, np.zeros_like(syn0))
        engs.append(e)
    with ThreadPoolExecutor(max_workers=R) as ex:
        list(ex.map(lambda r: engs[r].comm_init_local(grp, r), range(R)))
    trainers = [Dd.ReplicaTrainer(engs[r], (), every, N.MODE_HOGWILD, backend="libg2v", world=R,
                                  agree=agree.for_rank(r)) for r in range(R)]
    rs = np.random.RandomState(1)
    for it in range(iters):
        permute(it)
        base_seed = int(rs.randint(0, 2 ** 31 - 1))

        def rank(r):
            s0, s1 = Dd.shard_range(n, r, R)
            engs[r].set_corpus_device(perm.data_ptr() + 8 * s0, 2 * (s1 - s0), sent_len=2,
                                      keepalive=perm)
            jr = E.plan_jobs(n_sent=s1 - s0, sent_len=2)
            sd = E.job_seeds(np.random.RandomState((base_seed + 7919 * r) % 2 ** 32), len(jr) - 1)
            trainers[r].train_epoch(jr, E.job_alphas(jr, s1 - s0), sd)
            engs[r].sync()
        with ThreadPoolExecutor(max_workers=R) as ex:
            list(ex.map(rank, range(R)))
    w = [e.get_weights() for e in engs]
    assert all(np.array_equal(x[0], w[0][0]) and np.array_equal(x[1], w[0][1]) for x in w[1:])
    merges = trainers[0].averages
    for e in engs:
        e.close()
    grp.close()
    l_rep = _heldin(*w[0], tok, vc, K)
    o_rep = _objective(*w[0], hc, hj, vc, K)
    gap = (o_rep - o_single) / o_single
    print(f"{R} replicas (merge every {every} jobs, {merges} merges) vs one model: held-out "
          f"{o_rep:.5f} vs {o_single:.5f} ({gap:+.4%}), held-in {l_rep:.5f} vs {l_single:.5f} "
          f"({(l_rep - l_single) / l_single:+.4%})")
    assert merges == 7 * iters
    assert l_single < 0.7 * (K + 1) * np.log(2)
    assert gap < 0.01, (o_single, o_rep)
    assert (l_rep - l_single) / l_single < 0.01, (l_single, l_rep)
