#!/usr/bin/env python
"""Benchmark: gene pairs/sec of the Gene2vec SGNS hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): synthetic Zipf(1.0) gene pairs over
V = 24,447 genes, 100 M pairs per GPU, dim 200, negative 5, window 1,
sample 1e-3, alpha 0.025 -> 1e-4 restarting every step.  One STEP = one
gensim train() call = one epoch over the GPU's pairs (src/gene2vec.py:87),
i.e. downsampling + negative sampling + SGNS updates for every pair.  Inputs
(token ids, tables, job schedule) are resident in HBM before timing starts.

N > 1 (torchrun, one rank per GPU, RCCL over xGMI): weak scaling, each rank
trains its own 125 M-pair shard (BASELINE configs[2]: 1 B pairs over 8 GPUs)
on a replica of the tables, and every --avg-every-jobs jobs libg2v merges the
replicas itself (g2v_average: fused HIP delta/apply kernels around one grouped
ncclAllReduce on the training stream; torch.distributed only hands out the
RCCL unique id).  N = 1 runs no merge at all.

Prints ONE JSON line on rank 0 (see the contract in the task description):
value = pairs/s over all ranks, plus `roofline` (dominant kernel =
k_sgns_atomic, bound = memory-side float atomics: algorithmic atomic bytes
(K+2)*D*4 per directed example / its average launch time, HIP events on the
launch stream; the HBM view, 2*(K+2)*D*4 bytes, beside it) and `cpu_baseline`
(the C oracle, Hogwild OpenMP, on a bounded sample of the same corpus).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "gene pairs/sec (SGNS dim200 neg5) at 1/2/4/8 MI355X + achieved GB/s"
# BASELINE.json configs[3] (C4): python bench.py --vocab 60000 --dim 512 --negative 15
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ATOMIC_PEAK_GBPS = 1300.0  # MI355X_MICROARCH.md "Global float atomics": chip-wide added bytes
STORE_PEAK_GBPS = 6100.0  # same section: plain dword stores of the same shape, 6.0-6.2 TB/s


def usable_cpus():
    """(usable, os.cpu_count(), affinity, cgroup quota): the CPUs this process
    may run on at once -- the GPU box shows the whole machine in
    os.cpu_count() (256) but grants one GPU's share through the cgroup CPU
    quota (cpu.max 1600000/100000 = 16 CPUs, measured)."""
    host = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = host
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return min(host, aff, quota or host), host, aff, quota


def stored_rows_per_example(vcounts, sample, K, tail_row_syn0, tail_row_syn1neg):
    """Expected rows per directed example that leave as plain stores
    (G2V_OPT_TAIL_STORE): syn1neg rows from tail_row_syn1neg on
    (the centre with its kept-token share p_tok, the K negatives with the
    unigram^0.75 share p_neg), the syn0 input row from tail_row_syn0 on (p_tok);
    -1 = none.  An expectation over the vocabulary: the kernel also keeps
    atomics for examples with a repeated target, so the lost-update probe's
    exact store count runs ~0.6 % lower at C2 (1.476 vs 1.485 rows)."""
    from gene2vec_amd import engine as E
    vc = np.asarray(vcounts)
    pt = E.kept_token_share(vc, sample)
    pn = vc.astype(np.float64) ** 0.75
    pn /= pn.sum()
    rows = 0.0
    if tail_row_syn1neg >= 0:
        rows += pt[tail_row_syn1neg:].sum() + K * pn[tail_row_syn1neg:].sum()
    if tail_row_syn0 >= 0:
        rows += pt[tail_row_syn0:].sum()
    return float(rows)


def composite_roofline(update_bytes, stored_bytes, s_per_example,
                       atomic_peak=ATOMIC_PEAK_GBPS, store_peak=STORE_PEAK_GBPS):
    """(achieved, peak, frac) in GB/s of update bytes for k_sgns_atomic: the
    atomic bytes leave at the memory-side float-atomic rate, the stored bytes
    at the plain-store rate, so the roof time per example is atomic /
    atomic_peak + stored / store_peak and peak = update bytes / that time"""
    atomic_bytes = update_bytes - stored_bytes
    roof_s = atomic_bytes / (atomic_peak * 1e9) + stored_bytes / (store_peak * 1e9)
    peak = update_bytes / roof_s / 1e9
    achieved = update_bytes / s_per_example / 1e9 if s_per_example > 0 else 0.0
    return achieved, peak, achieved / peak


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--pairs", type=int, default=0, help="pairs per GPU (0 = 100M at N=1, 125M at N>1)")
    p.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                   help="weak (default): --pairs per GPU; strong: --total-pairs split over the "
                        "N GPUs (SURVEY 8(d) C3's 1 B / N curve; N = 1 trains all of them)")
    p.add_argument("--total-pairs", type=int, default=1_000_000_000,
                   help="--scaling strong: pairs of the whole job (each rank trains "
                        "total / N, its own shard of the generator)")
    p.add_argument("--vocab", type=int, default=24447)
    p.add_argument("--dim", type=int, default=200)
    p.add_argument("--negative", type=int, default=5)
    p.add_argument("--sample", type=float, default=1e-3)
    p.add_argument("--zipf", type=float, default=1.0)
    p.add_argument("--avg-every-jobs", type=int, default=0,
                   help="replica merge cadence in jobs per rank (N>1; 0 = the CLI's plan, "
                        "distributed.dp_merge_plan: once per epoch up to 4 GPUs, every 3,584 "
                        "jobs beyond)")
    p.add_argument("--merge", choices=("auto", "touch", "mean", "align"), default="auto",
                   help="replica merge rule (auto = the CLI's plan, gene2vec_amd.distributed)")
    p.add_argument("--grid", type=int, default=0, help="SGNS workgroups (0 = library default)")
    p.add_argument("--stripe", default="", help="hot-row stripes ROWSxCOPIES (default: library's)")
    p.add_argument("--stripe2", default="",
                   help="second stripe tier ENDROWxCOPIES, 0x4 = off (default: library's)")
    p.add_argument("--sample-overlap", type=int, choices=(0, 1), default=None,
                   help="G2V_OPT_SAMPLE_OVERLAP (sampler of segment s+1 under segment s's "
                        "SGNS kernel; default: the library's)")
    p.add_argument("--tail-store", type=int, default=None,
                   help="G2V_OPT_TAIL_STORE: -1 = the collision budget (the library's "
                        "default), 0 = every row atomic, n = rows >= n of both tables stored "
                        "(DESIGN.md 5e)")
    p.add_argument("--seg-jobs", type=int, default=0,
                   help="gensim jobs per sampling/update segment (0 = library default)")
    p.add_argument("--cpu-sample-pairs", type=int, default=50_000_000)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the CPU baseline (0 = every CPU this process may use: "
                        "min(os.cpu_count(), affinity, cgroup quota))")
    p.add_argument("--cpu-extra", action="store_true",
                   help="also time the CPU baseline on 1 core and on os.cpu_count() threads")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-eval", action="store_true")
    p.add_argument("--no-gather-roof", action="store_true",
                   help="skip the (untimed) write-free gather-roof measurement")
    p.add_argument("--dist", action="store_true",
                   help="init torch.distributed (RCCL) and average replicas even at N=1")
    p.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                   help="process-group backend (nccl = RCCL over xGMI; gloo only to rehearse "
                        "the N>1 path with several ranks sharing one GPU)")
    p.add_argument("--merge-transport", choices=("auto", "rccl", "torch"), default="auto",
                   help="N>1: auto = libg2v's merge over RCCL (nccl) or over the host "
                        "collective (gloo); rccl = libg2v's RCCL communicator whatever the "
                        "process group (with gloo: the test suite's two-ranks-one-GPU "
                        "stand-in, G2V_RCCL_LIB); torch = torch.distributed merges the bound "
                        "tables")
    p.add_argument("--traffic-json", default=None,
                   help="PMC bytes per example for roofline.traffic (default: the newest "
                        "profiles/**/traffic_r*.json of this workload measured on this kernel build)")
    p.add_argument("--library", default=None,
                   help="A/B hook: load this libg2v build (gene2vec_amd.build.build(tag=...)) "
                        "instead of gene2vec_amd/libg2v.so")
    p.add_argument("--launch-probe", action="store_true",
                   help="test hook: the ranks agree on the world over gloo and rank 0 prints "
                        "{n_gpus, ranks} without touching a GPU (checks --gpus N's own launcher)")
    return p.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) started without a launcher: start ONE child
    `python -m torch.distributed.run --nproc-per-node N bench.py <same argv>`
    (one rank per GPU, rendezvous on 127.0.0.1), forward rank 0's JSON line
    and return the child's exit status.  Called before anything imports torch
    or touches a GPU: the parent only waits (no exec of a GPU process)."""
    import signal
    import subprocess
    assert "torch" not in sys.modules, "the launcher must not initialise torch / the GPU"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get(
        "HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    # same process group: a timeout that kills this process's group ends the ranks too
    child = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=None, text=True)

    def _stop(signum, _frame):
        child.terminate()
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, _stop)
    lines = []
    for ln in child.stdout:  # ranks print progress on stderr; stdout carries the one line
        if ln.startswith("{"):
            lines.append(ln)
        else:
            sys.stderr.write(ln)
    rc = child.wait()
    if lines:
        sys.stdout.write(lines[-1])
        sys.stdout.flush()
    if rc != 0:
        print(f"bench.py: {n}-rank run failed (torch.distributed.run exit {rc})", file=sys.stderr)
    return rc


def pairs_per_rank(a, world):
    """pairs each rank trains per step: weak scaling --pairs (100 M at N = 1,
    the C2 line; 125 M at N > 1, C3's 1 B over 8); strong scaling
    --total-pairs / N"""
    if a.scaling == "strong":
        if a.pairs:
            sys.exit("bench.py: --scaling strong takes --total-pairs, not --pairs")
        return a.total_pairs // world
    return a.pairs or (100_000_000 if world == 1 else 125_000_000)


def launch_probe(a, world, rank):
    """--launch-probe: the N ranks of a spawned run meet over gloo (CPU only)
    and rank 0 reports the world and the shard each rank would train"""
    shape = {"scaling": a.scaling, "pairs_per_rank": pairs_per_rank(a, world)}
    if world == 1:
        print(json.dumps({"probe": True, "n_gpus": 1, "rank_sum": 1, "ranks_expected_sum": 1,
                          **shape}), flush=True)
        return
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"probe": True, "n_gpus": world, "rank_sum": int(t.item()),
                          "ranks_expected_sum": world * (world + 1) // 2, **shape}), flush=True)
    dist.destroy_process_group()


def main():
    a = parse()
    # the process shape, decided before torch is imported (no GPU touched yet):
    # under a launcher WORLD_SIZE must be --gpus; without one, --gpus N > 1
    # starts its own N-rank child run
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    if env_world is not None and int(env_world) != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={env_world} "
                 "ranks; pass --gpus equal to --nproc-per-node")
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if a.launch_probe:
        launch_probe(a, int(env_world or 1), int(os.environ.get("RANK", "0")))
        return
    # stdout carries exactly one JSON line: the libraries' own chatter (RCCL
    # prints its version banner from C on fd 1) goes to stderr until then
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    from gene2vec_amd import _native as N
    if a.library:
        N.use_library(a.library)
    from gene2vec_amd import distributed as Dd
    from gene2vec_amd import engine as E
    from gene2vec_amd import synthetic as S

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.backend == "gloo":
        # rehearsal mode: ranks beyond the visible GPUs share them round-robin
        local %= max(1, torch.cuda.device_count())
    use_dist = world > 1 or a.dist
    if use_dist:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local)
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    n_pairs = pairs_per_rank(a, world)
    V0, D, K = a.vocab, a.dim, a.negative

    # ---- corpus shard + global vocabulary ---------------------------------------
    t = time.time()
    pairs = S.zipf_gene_pairs(n_pairs, V0, a.zipf, seed=20250114, shard=rank)
    flat = pairs.reshape(-1)
    counts, first = E.count_ids(flat, V0)
    counts, first = Dd.global_vocab(counts, first, token_offset=rank * flat.size, device=dev)
    order, remap = S.vocab_order(counts, first)
    V = len(order)
    vcounts = counts[order].astype(np.int64)
    tok = remap[flat]
    del flat, pairs
    t_corpus = time.time() - t

    # ---- device state --------------------------------------------------------------
    eng = E.SGNSEngine(V, D, K, device=local)
    if a.grid:
        eng.set_option(N.OPT_GRID, a.grid)
    if a.stripe:
        sr, sc = (int(x) for x in a.stripe.lower().split("x"))
        eng.set_option(N.OPT_STRIPE_ROWS, sr)
        eng.set_option(N.OPT_STRIPE_COPIES, sc)
    if a.stripe2:
        r2, c2 = (int(x) for x in a.stripe2.lower().split("x"))
        eng.set_option(N.OPT_STRIPE2_ROWS, r2)
        eng.set_option(N.OPT_STRIPE2_COPIES, c2)
    if a.seg_jobs:
        eng.set_option(N.OPT_SEG_JOBS, a.seg_jobs)
    if a.tail_store is not None:
        eng.set_option(N.OPT_TAIL_STORE, a.tail_store)
    if a.sample_overlap is not None:
        eng.set_option(N.OPT_SAMPLE_OVERLAP, a.sample_overlap)
    # a dedicated (non-default) stream: g2v kernels, RCCL all-reduces and the
    # timing events are all ordered on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream != 0
    eng.set_stream(stream.cuda_stream)
    ld = eng.ld
    names = S.gene_names(V0)
    seeds = np.array([zlib.crc32((names[i] + "1").encode()) for i in order], np.uint32)
    syn0_h = E.seeded_vectors(seeds, D)  # [ext] seeded_vector, deterministic hash
    # both tables in one buffer: a replica merge is one collective per quantity
    tables = torch.zeros((2, V, ld), dtype=torch.float32, device=dev)
    syn0, syn1 = tables[0], tables[1]
    syn0[:, :D] = torch.from_numpy(syn0_h).to(dev)
    eng.bind_tables(syn0.data_ptr(), syn1.data_ptr(), ld, keepalive=(tables,))
    eng.set_vocab(vcounts, a.sample)
    tok_d = torch.from_numpy(tok).to(dev)
    eng.set_corpus_device(tok_d.data_ptr(), tok_d.numel(), sent_len=2, keepalive=tok_d)
    js = E.plan_jobs(n_sent=n_pairs, sent_len=2)
    n_jobs = len(js) - 1
    alphas = E.job_alphas(js, n_pairs)
    rs = np.random.RandomState(Dd.rank_seed(1, rank))  # gensim model.random(seed=1) per rank
    step_seeds = [E.job_seeds(rs, n_jobs) for _ in range(a.warmup + a.steps)]
    merge_rule, avg_every = Dd.dp_merge_plan(n_pairs, a.avg_every_jobs or None, a.merge,
                                             jobs_per_rank=n_jobs, world=world)
    merge_beta = Dd.dp_merge_beta(n_pairs, world, a.merge)
    if merge_beta != 1.0:
        eng.set_option(N.OPT_MERGE_BETA_MILLI, int(round(merge_beta * 1000)))
    if not use_dist:
        avg_every = n_jobs
    merge_backend = "torch"
    merge_note = None
    if use_dist and ((a.backend == "nccl" and a.merge_transport == "auto")
                     or a.merge_transport == "rccl"):
        # libg2v's own RCCL communicator: rank 0's unique id over the process group
        box = [eng.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        try:
            eng.comm_init(box[0], world, rank)
            merge_backend = "rccl"
        except N.G2VError as e:  # keep the run measurable: torch merges the bound tables
            merge_note = f"g2v_comm_init failed ({e}); torch.distributed merge used"
        ok = torch.tensor([1 if merge_backend == "rccl" else 0],
                          device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok.item() == 0:  # every rank must merge the same way
            merge_backend = "torch"
    elif use_dist and a.merge_transport == "auto":
        # gloo rehearsal: libg2v's merge, its all-reduce carried through the host
        eng.comm_init_host(Dd.host_collective(), world, rank)
        merge_backend = "libg2v-host"
    trainer = Dd.ReplicaTrainer(eng, (tables,), avg_every, N.MODE_HOGWILD, merge=merge_rule,
                                backend="torch" if merge_backend == "torch" else "libg2v")
    torch.cuda.synchronize(dev)

    def step(i, timing):
        trainer.train_epoch(js, alphas, step_seeds[i], timing=timing)

    for i in range(a.warmup):
        step(i, False)
    torch.cuda.synchronize(dev)
    eng.read_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    # per-step events on the same stream (SURVEY 8(d) asks for the median step
    # as well); value stays whole-job throughput over the bracketed region
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    w0 = time.perf_counter()
    ev0.record(stream)
    for i in range(a.steps):
        marks[i].record(stream)
        step(a.warmup + i, True)
    marks[a.steps].record(stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - w0
    st = eng.read_stats()
    gpu_ms = ev0.elapsed_time(ev1)
    step_ms = [round(marks[i].elapsed_time(marks[i + 1]), 3) for i in range(a.steps)]
    elapsed = max(wall, gpu_ms / 1e3)
    if world > 1:
        el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed = float(el.item())
        ex = torch.tensor([st["examples"]], dtype=torch.int64, device=dev)
        dist.all_reduce(ex)
        total_examples = int(ex.item())
    else:
        total_examples = st["examples"]
    total_pairs = n_pairs * a.steps * world
    value = total_pairs / elapsed

    # ---- roofline of the dominant kernel (k_sgns_atomic) --------------------------------
    bytes_per_example = 2 * (K + 2) * D * 4
    launches = max(1, st["launches"])
    avg_launch_ms = st["sgns_kernel_ms"] / launches
    alg_bytes_launch = st["examples"] * bytes_per_example / launches
    achieved = alg_bytes_launch / (avg_launch_ms / 1e3) / 1e9 if avg_launch_ms > 0 else 0.0
    traffic = None
    traffic_src = None
    # PMC bytes per example of the same workload (vocabulary, shape,
    # downsampling and skew) from a separate rocprofv3 --pmc pass of THIS
    # kernel build (scripts/profile_round.sh -> profiles/traffic_*.json,
    # stamped with the hash of the kernel's sources), scaled to this run's
    # examples per launch; a profile of another build is refused (traffic null)
    from gene2vec_amd.build import kernel_source_hash
    # (an A/B run of another build matches no traffic profile)
    ksha = kernel_source_hash() if not a.library else "library " + os.path.basename(a.library)
    # the layout the timed launches actually used (g2v_stats): the grid and
    # stripe tiers are set_vocab's; the stability cap only holds waves back
    # inside a launch (waves_last_launch below)
    launch = {"grid_workgroups": st["sgns_grid"],
              "stripes": f"{st['stripe_rows']}x{st['stripe_copies']}",
              "stripes_tier2": (f"rows < {st['stripe2_rows']} x{st['stripe2_copies']}"
                                if st["stripe2_copies"] > 1 else "off"),
              # cold rows written by plain stores (G2V_OPT_TAIL_STORE, 0 = off)
              "tail_store": eng.get_option(N.OPT_TAIL_STORE)}
    cands = [a.traffic_json] if a.traffic_json else sorted(
        glob.glob(os.path.join(ROOT, "profiles", "**", "traffic_r*.json"), recursive=True),
        reverse=True)
    stale = []
    for tpath in cands:
        if traffic is not None or not os.path.exists(tpath):
            continue
        try:
            tj = json.load(open(tpath))
        except (OSError, ValueError):
            continue
        if (tj.get("vocab"), tj.get("dim"), tj.get("negative"), tj.get("sample"),
                tj.get("zipf")) != (V0, D, K, a.sample, a.zipf):
            continue
        if tj.get("kernel_src_sha16") != ksha or tj.get("launch") != launch:
            stale.append(os.path.relpath(tpath, ROOT))
            continue
        traffic = round((tj["fetch_bytes_per_example"] + tj["write_bytes_per_example"])
                        * st["examples"] / launches, 1)
        # the same profile's L2 hit rate and VALU busy (scripts/pmc_traffic.py)
        counter_extras = {k: tj[k] for k in ("l2_hit_rate", "valu_busy", "valu_insts_per_cycle_per_simd",
                                              "traffic_over_algorithmic") if k in tj}
        traffic_src = (f"{os.path.relpath(tpath, ROOT)} (kernel build {ksha}, same launch "
                       "layout): PMC bytes "
                       f"per example x this run's {st['examples'] // launches} examples per "
                       "launch (not measured in this process)")
    if traffic is None:
        counter_extras = {}
        traffic_src = (f"no PMC profile of kernel build {ksha} with this launch layout for "
                       "this workload"
                       + (f"; refused profiles of other builds: {', '.join(stale[:3])}"
                          if stale else ""))
    # bound = the resource that binds k_sgns_atomic: its row updates leave the
    # CU as memory-side f32 atomics of the delta (MI355X_MICROARCH.md "Global
    # float atomics": ~1.3 TB/s of added bytes chip-wide, whatever the
    # placement) except the cold syn1neg rows' plain write-through stores of
    # the new value (G2V_OPT_TAIL_STORE; the guide's plain
    # stores of the same shape: 6.0-6.2 TB/s).  Per directed example
    # (K+2)*D*4 algorithmic update bytes; the stored share is the vocabulary's
    # expectation for the rows the launches stored (g2v_stats tail rows: the
    # centre and K negatives of syn1neg from p_tok / p_neg, the syn0 input
    # from p_tok; checked against the lost-update probe's store count).  The
    # roof time is atomic bytes / 1.3 TB/s + stored bytes / 6.1 TB/s;
    # achieved = update bytes / launch time, peak = update bytes / roof time.
    # The HBM view of the same launches (2*(K+2)*D*4 bytes per example: every
    # updated row read and written) stays beside it as hbm_*.
    update_bytes = (K + 2) * D * 4
    t0r, t1r = st["tail_row_syn0"], st["tail_row_syn1neg"]
    stored_rows = stored_rows_per_example(vcounts, a.sample, K, t0r, t1r)
    stored_bytes = stored_rows * D * 4
    atomic_bytes = update_bytes - stored_bytes
    t_ex = st["sgns_kernel_ms"] / 1e3 / max(1, st["examples"])  # s per example
    upd_gbps, peak_gbps, frac = composite_roofline(update_bytes, stored_bytes, t_ex)
    roofline = {"bound": "atomics", "achieved": round(upd_gbps, 1), "peak": round(peak_gbps, 1),
                "unit": "GB/s", "frac": round(frac, 4),
                "traffic": traffic,
                "kernel": "k_sgns_atomic", "avg_launch_ms": round(avg_launch_ms, 4),
                "update_bytes_per_example": update_bytes,
                "atomic_bytes_per_example": round(atomic_bytes, 1),
                "stored_bytes_per_example": round(stored_bytes, 1),
                "stored_rows_per_example": round(float(stored_rows), 4),
                "tail_row_syn1neg": t1r, "tail_row_syn0": t0r,
                "atomic_achieved_GBps": round(atomic_bytes / t_ex / 1e9, 1) if t_ex > 0 else 0.0,
                "atomic_peak_GBps": ATOMIC_PEAK_GBPS, "store_peak_GBps": STORE_PEAK_GBPS,
                "algorithmic_bytes_per_launch": int(alg_bytes_launch),
                "bytes_per_example": bytes_per_example,
                "binding_resource": "memory-side float atomics (MI355X_MICROARCH.md: ~1300 GB/s "
                                    "of added bytes chip-wide) plus the cold rows' plain stores "
                                    "(~6100 GB/s); peak = the update bytes over "
                                    "atomic/1300 + stored/6100",
                # algorithmic bytes (every updated row read + written) against
                # the HBM peak: a view, not measured HBM traffic
                "alg_mem_achieved_GBps": round(achieved, 1), "hbm_peak_GBps": HBM_PEAK_GBPS,
                "alg_mem_frac_of_hbm_peak": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic_unit": ("L2-to-fabric bytes per launch (Infinity Cache + HBM: PMC "
                                 "TCC FETCH_SIZE x2 + WRITE_SIZE, which count the L2's "
                                 "memory-side requests, Infinity-Cache hits included; "
                                 "MI355X_MICROARCH.md 'HBM')"),
                **counter_extras,
                "traffic_source": traffic_src,
                "kernel_src_sha16": ksha,
                # waves that trained in the last timed launch (the stability
                # cap may hold some back)
                "waves_last_launch": st["sgns_waves"],
                **launch}

    # ---- measured gather roof: the same kernel on the same index
    # stream with its table writes compiled out (G2V_OPT_DEBUG_WRITE=2) and a
    # full-occupancy grid, untimed by the contract, tables left unchanged ----------
    if rank == 0 and K == 5 and D <= 256 and not a.no_gather_roof:
        gj = min(n_jobs, 2048)
        eng.set_option(N.OPT_DEBUG_WRITE, 2)
        eng.set_option(N.OPT_GRID, 2048)
        eng.train(js[:gj + 1], alphas[:gj], step_seeds[0][:gj], N.MODE_HOGWILD, timing=True)
        gs = eng.read_stats()
        eng.set_option(N.OPT_DEBUG_WRITE, 0)
        eng.set_option(N.OPT_GRID, a.grid)
        read_bytes = (K + 2) * D * 4
        gather_gbps = read_bytes * gs["examples"] / (gs["sgns_kernel_ms"] / 1e3) / 1e9
        ours = read_bytes * st["examples"] / (st["sgns_kernel_ms"] / 1e3) / 1e9
        roofline.update({"gather_roof_GBps": round(gather_gbps, 1),
                         "gather_achieved_GBps": round(ours, 1),
                         "gather_frac": round(ours / gather_gbps, 4)})

    # ---- quality sanity check: SGNS objective on held-in pairs ------------------------------
    quality = None
    if not a.no_eval and rank == 0:
        s0 = syn0[:, :D].cpu().numpy()
        s1 = syn1[:, :D].cpu().numpy()
        r = np.random.Generator(np.random.PCG64(99))
        idx = r.integers(0, n_pairs, 20000)
        c, j = tok[2 * idx], tok[2 * idx + 1]
        p = vcounts.astype(np.float64) ** 0.75
        negs = r.choice(V, size=(20000, K), p=p / p.sum())
        u = s0[j].astype(np.float64)
        pos = np.einsum("nd,nd->n", u, s1[c].astype(np.float64))
        neg = np.einsum("nd,nkd->nk", u, s1[negs].astype(np.float64))
        loss = float((np.logaddexp(0, -pos) + np.logaddexp(0, neg).sum(1)).mean())
        quality = {"sgns_loss_heldin": round(loss, 4), "init_loss": round((K + 1) * np.log(2), 4)}

    # ---- CPU baseline (C oracle, Hogwild OpenMP) on a bounded sample -------------------------
    cpu = None
    if world == 1 and not a.no_cpu_baseline:
        from oracle import c_oracle as CO
        usable, host_cores, affinity, quota = usable_cpus()
        ncpu = a.cpu_threads or usable
        ns = min(a.cpu_sample_pairs, n_pairs)
        jsc = E.plan_jobs(n_sent=ns, sent_len=2)
        off = np.arange(0, 2 * ns + 1, 2, dtype=np.int64)
        si = CO.sample_int(vcounts, a.sample)
        cum = CO.make_cum_table(vcounts)
        al = E.job_alphas(jsc, ns).astype(np.float32)
        sd = E.job_seeds(np.random.RandomState(1), len(jsc) - 1)
        ld_cpu = (D + 15) // 16 * 16  # rows on 64-B lines of their own (no false sharing)

        def cpu_run(threads, n=ns):
            c0 = syn0_h.copy()
            c1 = np.zeros_like(c0)
            js_n = jsc if n == ns else E.plan_jobs(n_sent=n, sent_len=2)
            al_n = al if n == ns else E.job_alphas(js_n, n).astype(np.float32)
            t = time.perf_counter()
            CO.train(tok[:2 * n], off[:n + 1], js_n, al_n, sd[:len(js_n) - 1], si,
                     a.sample != 0, cum, c0, c1, np.ones(V, np.float32), K, nthreads=threads,
                     ld=ld_cpu)
            return time.perf_counter() - t

        dt = cpu_run(ncpu)
        cpu = {"value": round(ns / dt, 1), "unit": "pairs/s", "cores": ncpu, "kind": "port",
               "host_cores": host_cores, "affinity_cores": affinity, "cgroup_cpu_quota": quota,
               "sample": f"first {ns} pairs of the same corpus, 1 epoch, C oracle "
                         f"(oracle/sgns_oracle.c) Hogwild OpenMP on {ncpu} threads = every "
                         f"CPU this process may use (os.cpu_count() {host_cores}, affinity "
                         f"{affinity}, cgroup quota {quota}), rows padded to {ld_cpu} floats, "
                         f"{dt:.2f} s"}
        if host_cores != ncpu:
            # os.cpu_count() threads as well (SURVEY 8(d) "all host cores"), on a
            # smaller sample: under a CPU quota they time-share `usable` CPUs
            nh = min(ns, 10_000_000)
            dh = cpu_run(host_cores, nh)
            cpu["value_host_cores_threads"] = round(nh / dh, 1)
            cpu["host_cores_sample"] = (f"first {nh} pairs, {host_cores} threads "
                                        f"(os.cpu_count()), {dh:.2f} s")
        if a.cpu_extra:
            for th in sorted({1, host_cores} - {ncpu}):
                d = cpu_run(th)
                cpu[f"value_{th}_threads"] = round(ns / d, 1)

    cfg_name = {(24447, 200, 5): "C2", (60000, 512, 15): "C4"}.get((V0, D, K), "custom")
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "pairs/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": a.scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {
                "workload": (f"{cfg_name}: synthetic Zipf({a.zipf:g}) gene pairs, V={V0}, "
                             f"{n_pairs} pairs, dim {D}, neg {K}, window 1, sample {a.sample:g}, "
                             "1 epoch per step") if world == 1 and a.scaling == "weak" else
                            (f"C3 strong scaling: synthetic Zipf({a.zipf:g}) gene pairs, V={V0}, "
                             f"{n_pairs * world} pairs in all, dim {D}, neg {K}, window 1, sample "
                             f"{a.sample:g}, 1 epoch per step on one GPU") if world == 1 else
                            ((f"C3 strong scaling: synthetic Zipf gene pairs, V={V0}, "
                              f"{n_pairs * world} pairs in all = {n_pairs} per GPU x {world}"
                              if a.scaling == "strong" else
                              f"C3: synthetic Zipf gene pairs, V={V0}, {n_pairs} pairs per GPU x "
                              f"{world}")
                             + f", dim {D}, neg {K}, replica merge ({merge_rule}) every "
                             f"{avg_every} jobs: "
                             + (("libg2v g2v_average (RCCL over xGMI)" if a.backend == "nccl"
                                 else "libg2v RCCL merge path through G2V_RCCL_LIB (rehearsal, "
                                      "ranks sharing a GPU)") if merge_backend == "rccl"
                                else "libg2v merge over gloo (host collective) rehearsal, ranks "
                                     "sharing a GPU" if merge_backend == "libg2v-host"
                                else "torch.distributed gloo rehearsal, ranks sharing a GPU"
                                if a.backend == "gloo" else
                                "torch.distributed merge (libg2v communicator unavailable)")),
                "vocab": V, "vocab_requested": V0, "zipf": a.zipf, "pairs_per_gpu": n_pairs,
                **({"total_pairs": n_pairs * world} if a.scaling == "strong" else {}),
                "dim": D, "negative": K, "sample": a.sample, "window": 1,
                "parallelism": f"dp{world}" + (f" + {merge_backend} {merge_rule} merge"
                                               if world > 1 else "")},
            # per-GPU rate beside the shard it trained: N = 1 trains the C2
            # 100 M pairs without merges, N > 1 a 125 M-pair shard per rank
            # with merges, so compare points of a 1 -> N curve per GPU AND shard
            "value_per_gpu": round(value / world, 1), "pairs_per_gpu": n_pairs,
            "examples_per_s": round(total_examples / elapsed, 1),
            "effective_examples": total_examples,
            "roofline": roofline, "cpu_baseline": cpu, "quality": quality,
            "merge": ({"backend": merge_backend, "rule": merge_rule, "every_jobs": avg_every,
                       "merges": trainer.averages, "note": merge_note} if world > 1 else None),
            "gpu_event_ms": round(gpu_ms, 3), "wall_s": round(wall, 4),
            "step_ms_rank0": step_ms, "step_ms_median_rank0": float(np.median(step_ms)),
            "corpus_gen_s": round(t_corpus, 2),
        }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    eng.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
