"""Host-side overheads around one CLI iteration at C2 size: corpus upload
(g2v_set_corpus from pageable host memory), weight upload/download, engine
creation.  Experiment script."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from gene2vec_amd import engine as E  # noqa: E402

V, D, K = 24447, 200, 5
tok = np.random.RandomState(0).randint(0, V, 200_000_000).astype(np.int32)
counts = np.full(V, 10000, np.int64)
t = time.perf_counter()
eng = E.SGNSEngine(V, D, K)
t_create = time.perf_counter() - t
t = time.perf_counter()
eng.set_vocab(counts, 1e-3)
t_vocab = time.perf_counter() - t
w = np.random.RandomState(1).rand(V, D).astype(np.float32)
t = time.perf_counter()
eng.set_weights(w, w)
t_setw = time.perf_counter() - t
for i in range(3):
    t = time.perf_counter()
    eng.set_corpus(tok, sent_len=2)
    eng.sync()
    print(f"set_corpus 800 MB: {time.perf_counter() - t:.3f} s", flush=True)
t = time.perf_counter()
g0, g1 = eng.get_weights()
t_getw = time.perf_counter() - t
print(f"create {t_create:.3f} s, set_vocab {t_vocab:.3f} s, set_weights {t_setw:.3f} s, "
      f"get_weights {t_getw:.3f} s", flush=True)
