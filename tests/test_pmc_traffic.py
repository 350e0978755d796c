"""CPU: scripts/pmc_traffic.py, the counters behind bench.py's
roofline.traffic (verdict r5 item 3).  Synthetic rocprofv3 counter CSVs for
one k_sgns_atomic launch of known size: FETCH_SIZE is doubled (the gfx950
16-B/lane read correction, MI355X_MICROARCH.md 'HBM'), WRITE_SIZE taken as
is, both labelled L2-to-fabric bytes (Infinity Cache + HBM), and the L2 hit
rate and VALU busy come out of their own passes."""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id",
       "Grid_Size", "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size",
       "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Counter_Name",
       "Counter_Value", "Start_Timestamp", "End_Timestamp"]
KNAME = "void g2v::k_sgns_atomic<5, 1, 0, false>(g2v::SgnsArgs)"


def _pass(d, i, counters):
    os.makedirs(os.path.join(d, f"p{i}", "box"), exist_ok=True)
    with open(os.path.join(d, f"p{i}", "box", "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(HDR)
        for k, v in counters.items():
            w.writerow([1, 1, "Agent 2", 2, 1, 1, 65536, 7, KNAME, 256, 0, 0, 256, 0, 100, k, v,
                        0, 1])
            # another kernel's counters must not count
            w.writerow([2, 2, "Agent 2", 2, 1, 1, 512, 3, "k_job_sample", 256, 0, 0, 64, 0, 32,
                        k, 1e9, 0, 1])


def test_pmc_traffic_labels_and_counters(tmp_path):
    pytest.importorskip("numpy")
    ex = 1_000_000
    d = str(tmp_path)
    bpe = 11200
    line = {"effective_examples": ex, "config": {"vocab": 24447, "vocab_requested": 24447,
                                                 "dim": 200, "negative": 5, "sample": 1e-3,
                                                 "zipf": 1.0},
            "roofline": {"algorithmic_bytes_per_launch": ex * bpe, "bytes_per_example": bpe,
                         "grid_workgroups": 256, "stripes": "4x16",
                         "stripes_tier2": "rows < 20 x4", "tail_store": -1}}
    with open(os.path.join(d, "p1.log"), "w") as f:
        f.write("noise\n" + json.dumps(line) + "\n")
    _pass(d, 1, {"FETCH_SIZE": 3000.0 * ex / 1024})     # KB; x2 -> 6,000 B per example
    _pass(d, 2, {"WRITE_SIZE": 5000.0 * ex / 1024})
    _pass(d, 3, {"TCC_HIT_sum": 30.0, "TCC_MISS_sum": 70.0})
    cyc = 2.4e9 * 0.025  # one 25-ms launch at 2.4 GHz
    _pass(d, 7, {"SQ_ACTIVE_INST_VALU": 0.25 * cyc * 1024 / 4, "SQ_INSTS_VALU": 480.0 * ex,
                 "SQ_BUSY_CYCLES": cyc * 8 * 0.9, "GRBM_GUI_ACTIVE": cyc * 8})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_traffic.py"), d],
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    t = json.loads(r.stdout)
    assert t["fetch_bytes_per_example"] == pytest.approx(6000.0)
    assert t["write_bytes_per_example"] == pytest.approx(5000.0)
    assert t["l2_fabric_bytes_per_launch"] == pytest.approx(11000.0 * ex)
    assert "hbm_bytes_per_launch" not in t
    assert t["traffic_over_algorithmic"] == pytest.approx(11000 / 11200)
    assert t["l2_hit_rate"] == pytest.approx(0.3)
    assert t["valu_busy"] == pytest.approx(0.25)
    assert t["valu_issue_busy"] == pytest.approx(4 * 480.0 * ex / 1024 / cyc)
    assert t["kernel_cycles_per_launch"] == pytest.approx(cyc)
