# control: the same sample-0 flow with the grid fixed at set_vocab's default (no per-call cap)
import sys, tempfile, pathlib
sys.path.insert(0, "."); 
from tests.test_gpu_e2e_parity import _train_e2e, _gaps, _golden
ref = _golden()["sample0"]
got = _train_e2e(pathlib.Path(tempfile.mkdtemp()), 0.0)
print("capped", got, _gaps(got, ref), flush=True)
g = got["grid"][0]
got = _train_e2e(pathlib.Path(tempfile.mkdtemp()), 0.0, grid=g)
print("uncapped grid", g, got, _gaps(got, ref), flush=True)
