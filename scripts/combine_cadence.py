"""Join replica_quality.py runs of one corpus made in several gpurun calls
(the one-model seeds in the first) into one table of gaps.

Gaps are taken to the MEAN of the one-model seeds, per metric:
    python scripts/combine_cadence.py out.json run1/replica_quality.json run2/...
"""
import json
import sys

import numpy as np

METRICS = {"heldin": "heldin", "heldout": "heldout", "target_ratio": "target", "auc_mean": "auc"}


def main():
    out, paths = sys.argv[1], sys.argv[2:]
    runs, config = {}, None
    for p in paths:
        d = json.load(open(p))
        if config is None:
            config = d["config"]
        elif d["config"] != config:
            raise SystemExit(f"{p}: another corpus ({d['config']} vs {config})")
        runs.update(d["runs"])
    singles = {k: v for k, v in runs.items() if k.startswith("single")}
    if not singles:
        raise SystemExit("no one-model run among the inputs")
    ref = {m: float(np.mean([s[m] for s in singles.values()])) for m in METRICS
           if all(m in s for s in singles.values())}
    table = {}
    for tag, r in runs.items():
        table[tag] = {name + "_gap": round((r[m] - ref[m]) / ref[m], 5)
                      for m, name in METRICS.items() if m in r and m in ref}
        table[tag]["merges_total"] = r.get("merges_total")
    # per cadence: the mean and spread over the job-seed streams
    by_every = {}
    for tag, g in table.items():
        if not tag.startswith("replicas"):
            continue
        every = int(tag.split("_every")[1].split("_")[0])
        by_every.setdefault(every, []).append(g)
    summary = {}
    for every, gs in sorted(by_every.items()):
        summary[every] = {k: [round(min(x[k] for x in gs), 5), round(max(x[k] for x in gs), 5)]
                          for k in gs[0] if k.endswith("_gap")}
    json.dump({"config": config, "one_model_mean": ref, "gaps": table,
               "per_cadence_min_max": summary, "sources": paths}, open(out, "w"), indent=1)
    for every, s in summary.items():
        print(every, s)


if __name__ == "__main__":
    main()
