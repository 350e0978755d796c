"""Per-example L2-to-fabric traffic (Infinity Cache + HBM) of k_sgns_atomic from the PMC passes of
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
    for i in range(1, 10):
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
        # TCC_HIT / (TCC_HIT + TCC_MISS); the memory-side float atomics count as misses
        "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
        "examples_per_launch": ex / launches,
        # FETCH_SIZE / WRITE_SIZE count the L2's memory-side (fabric) requests:
        # Infinity-Cache (MALL) hits are included, so this is not HBM traffic
        # (MI355X_MICROARCH.md 'HBM'); no gfx950 counter splits MALL from HBM
        "l2_fabric_bytes_per_launch": (fetch + write) * ex / launches,
        "algorithmic_bytes_per_example": bpe,
        "traffic_over_algorithmic": (fetch + write) / bpe,
    }
    # requests the L2 sends to the memory controller (DRAM side of the fabric;
    # MALL hits are not separable from TCC counters on gfx950)
    if "TCC_EA0_RDREQ_DRAM_sum" in c and c.get("TCC_EA0_RDREQ_sum"):
        res["ea_rdreq_to_mc_share"] = c["TCC_EA0_RDREQ_DRAM_sum"] / c["TCC_EA0_RDREQ_sum"]
    if "TCC_EA0_WRREQ_ATOMIC_DRAM_sum" in c and c.get("TCC_EA0_ATOMIC_sum"):
        res["ea_atomic_to_mc_share"] = c["TCC_EA0_WRREQ_ATOMIC_DRAM_sum"] / c["TCC_EA0_ATOMIC_sum"]
    # VALU busy (the gfx94x VALUBusy formula, rocprofv3 has no gfx950 derived
    # set): SQ_ACTIVE_INST_VALU x 4 / SIMDs / kernel cycles, the kernel's
    # cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs, MI355X_MICROARCH.md
    # 'DVFS give-back'); and the issue view, VALU wave-instructions x 4
    # cycles (a wave64 op on a 16-lane SIMD) per SIMD-cycle
    simds = 256 * 4
    if c.get("GRBM_GUI_ACTIVE"):
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        res["kernel_cycles_per_launch"] = cyc / launches
        if "SQ_ACTIVE_INST_VALU" in c:
            res["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4.0 / simds / cyc
        if "SQ_INSTS_VALU" in c:
            res["valu_insts_per_cycle_per_simd"] = c["SQ_INSTS_VALU"] / simds / cyc
            res["valu_issue_busy"] = 4.0 * c["SQ_INSTS_VALU"] / simds / cyc
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD",
              "SQ_INSTS_LDS"):
        if k in c:  # wave-instructions per directed example
            res[k.lower() + "_per_example"] = c[k] / ex
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
