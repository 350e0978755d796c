"""Per-example HBM traffic of k_sgns_atomic from the PMC passes of
scripts/profile_round.sh (rocprofv3 --pmc CSVs + the bench JSON of the same
10 M-pair run).  FETCH_SIZE is doubled (gfx950 reports half the bytes of 16-B
per-lane reads, MI355X_MICROARCH.md 'HBM'); WRITE_SIZE is exact for float
atomics.  Prints the JSON bench.py reads as --traffic-json."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KERNEL = "k_sgns_atomic"


def counters(d):
    tot = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if KERNEL not in row["Kernel_Name"]:
                    continue
                k = row["Counter_Name"]
                tot[k] = tot.get(k, 0.0) + float(row["Counter_Value"])
    return tot


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench JSON in {log}")


def main(out):
    c = {}
    for i in range(1, 7):
        if os.path.isdir(os.path.join(out, f"p{i}")):
            c.update(counters(os.path.join(out, f"p{i}")))
    b = bench_line(os.path.join(out, "p1.log"))
    ex = b["effective_examples"]
    launches = max(1, round(ex / (b["roofline"]["algorithmic_bytes_per_launch"]
                                  / b["roofline"]["bytes_per_example"])))
    fetch = 2.0 * c["FETCH_SIZE"] * 1024 / ex
    write = c["WRITE_SIZE"] * 1024 / ex
    hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    bpe = b["roofline"]["bytes_per_example"]
    cfg = b["config"]
    from gene2vec_amd.build import kernel_source_hash
    res = {
        # the kernel build these counters belong to (bench.py refuses any other)
        "kernel_src_sha16": kernel_source_hash(),
        "launch": {k: b["roofline"][k] for k in ("grid_workgroups", "stripes", "stripes_tier2",
                                                  "tail_store")},
        "vocab": cfg.get("vocab_requested", cfg["vocab"]), "dim": cfg["dim"], "negative": cfg["negative"],
        "sample": cfg["sample"], "zipf": cfg.get("zipf", 1.0), "kernel": KERNEL,
        "method": "rocprofv3 --pmc, one counter group per run (scripts/profile_round.sh), "
                  "one-step bench of the workload; FETCH_SIZE x2 (gfx950 16-B/lane read correction), "
                  "WRITE_SIZE as is (KB units); summed over the SGNS launches / examples",
        "fetch_bytes_per_example": fetch, "write_bytes_per_example": write,
        "atomic_requests_per_example": c.get("TCC_EA0_ATOMIC_sum", 0.0) / ex,
        "l2_hit_rate_incl_atomic_misses": hit / (hit + miss) if hit + miss else None,
        "examples_per_launch": ex / launches,
        "hbm_bytes_per_launch": (fetch + write) * ex / launches,
        "algorithmic_bytes_per_example": bpe,
        "traffic_over_algorithmic": (fetch + write) / bpe,
    }
    # requests the L2 sends to the memory controller (DRAM side of the fabric;
    # MALL hits are not separable from TCC counters on gfx950)
    if "TCC_EA0_RDREQ_DRAM_sum" in c and c.get("TCC_EA0_RDREQ_sum"):
        res["ea_rdreq_to_mc_share"] = c["TCC_EA0_RDREQ_DRAM_sum"] / c["TCC_EA0_RDREQ_sum"]
    if "TCC_EA0_WRREQ_ATOMIC_DRAM_sum" in c and c.get("TCC_EA0_ATOMIC_sum"):
        res["ea_atomic_to_mc_share"] = c["TCC_EA0_WRREQ_ATOMIC_DRAM_sum"] / c["TCC_EA0_ATOMIC_sum"]
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD",
              "SQ_INSTS_LDS"):
        if k in c:  # wave-instructions per directed example
            res[k.lower() + "_per_example"] = c[k] / ex
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
