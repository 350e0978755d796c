"""Golden values for tests/test_gpu_e2e_parity.py: the gensim restatement's
(oracle/sgns_oracle.c, sequential = gensim workers=1 order) north-star metrics
after the reference's 10-iteration flow on tests.helpers.e2e_corpus().

    python tests/golden/make_e2e_golden.py     # ~2 minutes on one CPU
    python tests/golden/make_e2e_golden.py --v5k   # e2e_parity_v5k.json
    python tests/golden/make_e2e_golden.py --c2    # e2e_parity_c2.json

Per model.random seed: the last iteration's training loss (gensim's
compute_loss terms summed in double), the SGNS objective on 40,000 corpus
pairs, and the manuscript target function (oracle/target_oracle.py, the
planted modules as pathways).  Written to tests/golden/e2e_parity.json."""
import json
import os
import sys
import time
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from gene2vec_amd import engine as E  # noqa: E402
from oracle import c_oracle as CO  # noqa: E402
from oracle import target_oracle as TO  # noqa: E402
from tests.helpers import E2E, E2E_C2, E2E_V5K, e2e_corpus, e2e_heldin  # noqa: E402


def main(cfg=E2E, out_name="e2e_parity.json", with_sample0=True):
    t0 = time.time()
    tok, counts, index2word, lines, perms, wseeds = e2e_corpus(cfg)
    n = len(tok) // 2
    D, K, sample = cfg["D"], cfg["K"], cfg["sample"]
    V = len(counts)
    syn0 = E.seeded_vectors(wseeds, D)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    al = E.job_alphas(js, n).astype(np.float32)
    off = np.arange(0, 2 * n + 1, 2, dtype=np.int64)
    cum = CO.make_cum_table(counts)
    out = {"config": dict(cfg, seeds=list(cfg["seeds"])),
           "corpus_crc32": zlib.crc32(tok.tobytes()), "vocab": V, "runs": {}}
    def runs(smp):
        si = CO.sample_int(counts, smp)
        res = {}
        for seed in cfg["seeds"]:
            a0, a1 = syn0.copy(), np.zeros_like(syn0)
            rs = np.random.RandomState(seed)
            for it in range(cfg["iters"]):
                last = it == cfg["iters"] - 1
                lex = np.zeros(1, np.float64) if last else None
                tk = np.ascontiguousarray(tok.reshape(n, 2)[perms[it]].reshape(-1))
                CO.train(tk, off, js, al, E.job_seeds(rs, len(js) - 1), si, smp != 0, cum, a0,
                         a1, np.ones(V, np.float32), K, loss_exact=lex)
            pm, rm, ratio = TO.target_function(index2word, a0, lines)
            res[str(seed)] = {"loss": float(lex[0]), "heldin": e2e_heldin(a0, a1, tok, counts, K),
                              "target_ratio": ratio, "path_mean": pm, "rand_mean": rm}
            print(smp, seed, res[str(seed)], f"{time.time() - t0:.0f} s", flush=True)
        return res
    out["runs"] = runs(sample)
    for key in ("loss", "heldin", "target_ratio"):
        out[key + "_mean"] = float(np.mean([r[key] for r in out["runs"].values()]))
    # sample = 0 (no downsampling): the hot rows' staleness case of
    # g2v_train's stability cap (g2v_api.hip stability_grid)
    if with_sample0:
        s0 = {"runs": runs(0.0)}
        for key in ("loss", "heldin", "target_ratio"):
            s0[key + "_mean"] = float(np.mean([r[key] for r in s0["runs"].values()]))
        out["sample0"] = s0
    with open(os.path.join(HERE, out_name), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    if "--c2" in sys.argv:  # the C2 vocabulary: ~5 minutes per seed
        main(E2E_C2, "e2e_parity_c2.json", with_sample0=False)
    elif "--v5k" in sys.argv:  # the dense 5,000-gene corpus: ~1 minute per seed
        main(E2E_V5K, "e2e_parity_v5k.json", with_sample0=False)
    else:
        main()
