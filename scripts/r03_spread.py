"""Run-to-run spread of the 3-iteration CLI objective (tests/test_gpu_shuffle_cli.py's
setup) for the Python and the device shuffles over several shuffle seeds."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pathlib  # noqa: E402

from gene2vec_amd import Word2Vec  # noqa: E402
from gene2vec_amd.gene2vec import main as cli_main  # noqa: E402
from tests.test_gpu_shuffle_cli import _corpus, _heldin  # noqa: E402

tmp = pathlib.Path(tempfile.mkdtemp())
data, pairs, names = _corpus(tmp)
for seed in (4, 5, 6, 7):
    out = []
    for mode in ("python", "device"):
        d = tmp / f"{mode}{seed}"
        cli_main([str(data), str(d), "txt", "--shuffle", mode, "--iters", "3", "--dim", "64",
                  "--hash", "crc32", "--shuffle-seed", str(seed), "--native-ingest", "--no-txt",
                  "--no-w2v"])
        out.append(_heldin(Word2Vec.load(str(d / "gene2vec_dim_64_iter_3")), pairs, names))
    print(f"SPREAD seed {seed}: python {out[0]:.5f} device {out[1]:.5f}", flush=True)
