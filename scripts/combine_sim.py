"""How much an on-chip (per combine domain) pending-delta cache of the H
hottest rows would merge: the fraction of row updates that hit a row already
pending in the same window of consecutive examples, on the C2 record stream
(oracle sampler, 2 M pairs) -- DESIGN.md section 5c."""
import os
import sys

import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gene2vec_amd import engine as E, synthetic as S
from oracle import c_oracle as CO
n, V0 = 2_000_000, 24447
pairs = S.zipf_gene_pairs(n, V0, 1.0, seed=20250114)
flat = pairs.reshape(-1)
counts, first = E.count_ids(flat, V0)
order, remap = S.vocab_order(counts, first)
tok = remap[flat]; vc = counts[order].astype(np.int64)
js = E.plan_jobs(n_sent=n, sent_len=2); sd = E.job_seeds(np.random.RandomState(1), len(js)-1)
off = np.arange(0, 2*n+1, 2, dtype=np.int64)
rec = CO.sample_records(tok, off, js, sd, CO.sample_int(vc, 1e-3), True, CO.make_cum_table(vc), 5)
Ex = len(rec)
# syn1neg targets: center + negs; syn0: input (encode syn0 rows as V + row)
V = len(vc)
tg = np.concatenate([rec[:, [0]], rec[:, 2:]], axis=1)      # [E][6]
inp = rec[:, 1:2] + V
rows = np.concatenate([tg, inp], axis=1)                      # [E][7], -1 = skipped
print("examples", Ex)
for H in (64, 256, 1024):
    for win in (32, 128, 512, 2048, 8192):
        # windows of `win` consecutive examples stand for one domain's flush window
        m = (Ex // win) * win
        r = rows[:m].reshape(-1, win * 7)
        valid = r >= 0
        hot = valid & (((r < H)) | ((r >= V) & (r < V + H)))
        tot = valid.sum()
        # per window: distinct hot rows = flushes; hot updates merged into them
        merged = 0
        for w in range(r.shape[0]):
            h = r[w][hot[w]]
            merged += len(h) - len(np.unique(h))
        print(f"H {H:5d} window {win:5d} examples: {merged / tot * 100:5.1f} % of row updates merged")
