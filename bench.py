"""Benchmark: MultiSURF feature scoring on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg4]
                    [--samples 20000 --features 20000]

--config picks a BASELINE.json configuration: cfg4 (default, the headline:
MultiSURF 20000 x 20000), cfg2 (MultiSURF 5000 x 5000), cfg3 (ReliefF k=10,
20000 x 2000), cfg5s (SURF* 10000 x 50000), cfg5m (MultiSURF* 10000 x
50000).  Every line carries the dominant kernel's roofline and, at N=1, a CPU
baseline from the oracle on a bounded sample of the same workload.

For N > 1 launch one process per GPU with torch.distributed.run; the pair
tiles are sharded round-robin over the ranks and the three small exchange
vectors are summed with RCCL all-reduces (fastselect_amd/parallel.py).

Workload (BASELINE.json configs[3], the north-star target "MultiSURF on
20000x20000 fp32"; it fits one GPU, so N=1 runs the same job): make_classification(
n_samples=20000, n_features=20000, n_informative=20, n_redundant=100,
random_state=42), X cast to float32 once on the host, MultiSURF (non-star).
One step = one full scoring pass over the HBM-resident X: quantize, pass 1
(distance tiles), thresholds/neighbour counts, exact refinement of ambiguous
rows, pair weights, pass 2 (score accumulation), all-reduces, / n.

Rank 0 prints ONE JSON line: value = n*p / step time (feature-scores/s, the
whole job across all ranks), a `roofline` object for the dominant kernel
(VALU bound; 4 FMA-equivalent FLOPs per pair-feature evaluation)
measured with HIP events on the stream the kernels run on, and at N=1 a
`cpu_baseline` from the C oracle (oracle/relief_oracle.c, OpenMP) timed on a
bounded sample of focal samples of the same data and extrapolated.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Peak FP32 vector rate, MI355X_MICROARCH.md: 157.3 TFLOP/s = 256 CU x 4 SIMD x
# 64 lanes / 2 cycles per wave64 v_fma_f32 x 2 FLOP x 2.4 GHz.  Both hot
# kernels spend 2 full-rate VALU issue slots per pair-feature evaluation (PFE):
# k_score v_sub_f32 + v_fma_f32, k_dist one half-rate v_sad_u32.  Two issue
# slots are the cost of two FMAs, so one PFE is priced at 4 FMA-equivalent
# FLOPs against that peak ("Kernels").
VALU_PEAK_TFLOPS = 157.3
# float64 vector peak (SURF's float64 distance kernel k_dist_f64: v_add_f64
# sub + v_add_f64 |.| per PFE, each priced as one FMA): AMD's MI355X figure,
# half the FP32 vector rate (16 f64 lanes per SIMD cycle); not re-measured here
VALU_F64_PEAK_TFLOPS = 78.6
FLOP_PER_PFE = 4
HBM_PEAK_GBPS = 8000.0

# BASELINE.json configs (make_classification n_informative=20, n_redundant=R,
# random_state=42)
CONFIGS = {
    "cfg2": dict(algo="multisurf", n=5000, p=5000, red=100, star=False, idx=1),
    "cfg3": dict(algo="relieff", n=20000, p=2000, red=50, k=10, star=False, idx=2),
    "cfg4": dict(algo="multisurf", n=20000, p=20000, red=100, star=False, idx=3),
    "cfg5s": dict(algo="surf", n=10000, p=50000, red=100, star=True, idx=4),
    "cfg5m": dict(algo="multisurf", n=10000, p=50000, red=100, star=True, idx=4),
}
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def pmc_traffic(kernel, n, p, world):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (tools/summarize_prof.py), if it was taken on this workload."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    if t.get("n") != n or t.get("p") != p or t.get("world", 1) != world:
        return None, None
    k = t.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return k["hbm_bytes_per_launch"], t.get("source")


def rank_envs(n, port, base=None):
    """Environment of each of the n ranks bench.py starts for ``--gpus n``
    (one process per GPU, torch.distributed env:// rendezvous on 127.0.0.1),
    as torch.distributed.run would set it."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def launch_ranks(n, argv):
    """``python bench.py --gpus n`` without a launcher: start the n ranks as
    child processes (before this process touches any GPU), wait for all of
    them and exit with the first failure's status.  A rank that fails ends
    the others, so none waits forever at a barrier."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = os.path.abspath(__file__)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=e)
             for e in rank_envs(n, port)]
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 1
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def make_data(n, p, seed, red=100):
    from sklearn.datasets import make_classification
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=red,
                               random_state=seed)
    return X, y


def oracle_threads():
    """Threads of the CPU baseline: this job's CPU share (OMP_NUM_THREADS, 16
    on the GPU box, where nproc counts the whole machine), at most 16."""
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    return min(threads, 16)


def full_host_note(value, threads):
    """The baseline's full-host figure by linear scaling (the oracle is a
    per-focal-sample parallel loop): stated beside the
    measured one, labelled as extrapolated."""
    cores = os.cpu_count() or threads
    return {"machine_cores": cores,
            "value_full_host_extrapolated": value * cores / threads,
            "full_host_note": f"measured on {threads} threads (this job's CPU share); x{cores}/"
                              f"{threads} linear scaling to all {cores} cores of the host, "
                              f"not measured"}


def cpu_baseline_rows(algo, X, y, k, star, budget_s=25.0):
    """Oracle ReliefF / SURF on the first m focal samples, extrapolated to n
    (as cpu_baseline)."""
    from oracle import oracle as O
    O.build()
    threads = oracle_threads()
    n, p = X.shape

    def run(m):
        if algo == "relieff":
            return O.relieff_scores(X, y, n_neighbors=k, i_range=(0, m), n_jobs=threads)
        return O.surf_scores(X, y, use_star=star, i_range=(0, m), n_jobs=threads)
    run(threads)  # warm-up
    m = min(n, 2 * threads)
    t0 = time.perf_counter()
    run(m)
    t = time.perf_counter() - t0
    m = int(min(n, max(threads, threads * round(budget_s / t * m / threads))))
    t0 = time.perf_counter()
    run(m)
    t = time.perf_counter() - t0
    t_full = t * n / m
    name = "ReliefF" if algo == "relieff" else ("SURF*" if star else "SURF")
    out = {"value": n * p / t_full, "unit": "feature-scores/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(),
           "sample": f"oracle {name} (C/OpenMP restatement of the reference backend='cpu') on "
                     f"focal samples [0, {m}) of the same {n}x{p} data: {t:.2f} s, extrapolated "
                     f"x{n / m:.1f} to {t_full:.1f} s"}
    out.update(full_host_note(out["value"], threads))
    return out


def cpu_baseline(x, y, budget_s=25.0):
    """Oracle MultiSURF on the first m focal samples, extrapolated to n: a
    small untimed run (page-in, thread start), a short run to measure the
    per-sample rate, then a ~budget_s sample whose time is reported."""
    from oracle import oracle as O
    O.build()
    threads = oracle_threads()
    n, p = x.shape
    O.multisurf_scores(x, y, i_range=(0, threads), n_jobs=threads)  # warm-up
    m = min(n, 2 * threads)
    t0 = time.perf_counter()
    O.multisurf_scores(x, y, i_range=(0, m), n_jobs=threads)
    t = time.perf_counter() - t0
    m = int(min(n, max(threads, threads * round(budget_s / t * m / threads))))
    t0 = time.perf_counter()
    O.multisurf_scores(x, y, i_range=(0, m), n_jobs=threads)
    t = time.perf_counter() - t0
    t_full = t * n / m
    # the reference's loop evaluates every distance row twice plus the near
    # accumulation: ~(2 + near fraction) * n^2 * p PFE; the
    # published reference CPU rate is ~5e9 PFE/s
    pfe = 2.0 * m * (n - 1) * p
    out = {"value": n * p / t_full, "unit": "feature-scores/s", "cores": threads,
           "kind": "port", "cpu_model": cpu_model(),
           "pfe_per_s_distance_passes": pfe / t, "reference_published_pfe_per_s": 5e9,
           "sample": f"oracle MultiSURF (C/OpenMP restatement of the reference backend='cpu') "
                     f"on focal samples [0, {m}) of the same {n}x{p} data: {t:.2f} s, "
                     f"extrapolated x{n / m:.1f} to {t_full:.1f} s"}
    out.update(full_host_note(out["value"], threads))
    return out


GOLD = os.path.join(ROOT, "tests", "golden")
# FMA-equivalent FLOPs per PFE of the reference-order chains (k_ms_chains):
# v_sub_f32, v_mul_f32 |.| and v_add_f32, three full-rate issue slots
FLOP_PER_PFE_CHAINS = 6


def decisions_vs_fixture(counts, n, p, config):
    """Rows whose near hit / near miss counts differ from the reference's
    (the oracle's multisurf_decisions, committed as
    tests/golden/fullsize_<config>_multisurf_decisions.npz by
    tests/golden/make_fullsize.py --decisions), or None without a fixture
    for this workload."""
    path = os.path.join(GOLD, f"fullsize_{config}_multisurf_decisions.npz")
    if not os.path.exists(path):
        return None
    d = np.load(path, allow_pickle=False)
    if int(d["n"]) != n or int(d["p"]) != p:
        return None
    ref = d["counts"].astype(np.int64).reshape(-1, 2)
    got = np.asarray(counts, dtype=np.float64).reshape(-1, 2).astype(np.int64)
    bad = np.any(got != ref, axis=1)
    return {"flipped_rows": int(bad.sum()), "rows": int(n),
            "near_pairs_differing": int(np.abs(got - ref).sum()),
            "fixture": os.path.relpath(path, ROOT)}


def chain_entries(counts, y, star):
    """Directed (focal, neighbour) entries the reference-order chains walk:
    near hits + near misses, plus every far miss for MultiSURF*."""
    c = np.asarray(counts, dtype=np.float64).reshape(-1, 2)
    if not star:
        return float(c.sum())
    yv = np.asarray(y)
    _, inv, cnt = np.unique(yv, return_inverse=True, return_counts=True)
    misses = len(yv) - cnt[inv]
    return float(c[:, 0].sum() + misses.sum())


def reference_step(make_job, y, star, p, sync, steps=3):
    """The same step in reference-order accumulation (bit-identical to the
    oracle): ms per step and the chain kernel's rate."""
    job = make_job()
    try:
        job.step()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            job.step()
        sync()
        ms = (time.perf_counter() - t0) / steps * 1e3
        d_ms, c_ms = job.kernel_ms(0), job.kernel_ms(1)
        pfe = chain_entries(job.counts.cpu().numpy(), y, star) * p
        rate = pfe / (c_ms * 1e-3)
        return {"ms_per_step": ms, "steps": steps,
                "kernel_ms": {"k_dist": d_ms, "k_ms_chains": c_ms},
                "chain_pfe_per_launch": pfe, "chain_pfe_per_s": rate,
                "chain_valu_frac": FLOP_PER_PFE_CHAINS * rate / 1e12 / VALU_PEAK_TFLOPS,
                "pass1_operands": "32-bit",
                "parity": "bit-identical to the oracle (tests/test_gpu_refacc.py)"}
    finally:
        job.close()


def fit_ms(X, y, star, repeats=5):
    """End-to-end ``MultiSURF(backend='gpu').fit`` (validation + float32
    cast, column statistics, H2D of X, scoring, top-k): median of `repeats`
    after one warm-up fit.  SURVEY.md §8d's end-to-end timing."""
    import fastselect_amd
    est = fastselect_amd.MultiSURF(backend="gpu", n_features_to_select=10, use_star=star)
    est.fit(X, y)
    ts = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        est.fit(X, y)
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts)), ts


def sharded_fit_ms(X, y, star, local, barrier, sync, dist, repeats=3):
    """End-to-end multi-GPU scoring (``parallel.multisurf_scores``: cast,
    X to the GPUs by per-rank rows + all-gather, column statistics, plan,
    one step, all-reduces), max over ranks, median of `repeats` after one
    warm-up."""
    import torch

    from fastselect_amd.parallel import multisurf_scores
    multisurf_scores(X, y, use_star=star, device=local, release_cache=False)
    ts = []
    for _ in range(repeats):
        barrier()
        t0 = time.perf_counter()
        multisurf_scores(X, y, use_star=star, device=local, release_cache=False)
        sync()
        t = torch.tensor([(time.perf_counter() - t0) * 1e3], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ts.append(float(t.item()))
    return float(np.median(ts)), ts


def bench_rows(args, cfg, world, rank, local, on_gpu, dist, sync, barrier, dist_backend):
    """ReliefF (cfg3) / SURF* (cfg5s): a step is one scoring pass of a
    resident row plan (fs_plan_score: pass 1, neighbour selection or mean,
    pass 2 / update) over X in HBM; at N > 1 rank r scores the focal samples
    parallel.shard_rows(n, r, N) and one all-reduce sums the vectors."""
    import torch

    from fastselect_amd import _lib
    from fastselect_amd.parallel import shard_rows
    algo, n, p = cfg["algo"], args.samples, args.features
    t0 = time.perf_counter()
    X, y = make_data(n, p, args.seed, cfg["red"])
    if algo == "relieff":
        from fastselect_amd.ReliefF import relieff_inputs
        xin, ye, recip, isd, pri = relieff_inputs(X, y, 10, "gpu" if on_gpu else "cpu", local)
        kw = dict(k=cfg["k"], class_probs=pri)
    else:
        from fastselect_amd.SURF import surf_inputs
        xin = np.ascontiguousarray(X, dtype=np.float64)
        isd, recip = surf_inputs(xin, 10, "gpu" if on_gpu else "cpu", local)
        ye = np.asarray(y).astype(np.int32)
        kw = dict(use_star=args.star)
    log(f"rank {rank}/{world}: data {n}x{p} ready in {time.perf_counter() - t0:.1f} s")
    rows = shard_rows(n, rank, world)
    tdev = torch.device("cuda", local) if on_gpu else torch.device("cpu")
    stream = torch.cuda.current_stream().cuda_stream if on_gpu else 0
    barrier()
    sync()
    t0 = time.perf_counter()
    if algo != "relieff" and args.accumulation == "reference":
        raise SystemExit("bench.py: reference-order accumulation is MultiSURF / ReliefF only")
    with _lib.accumulation(args.accumulation):
        plan = _lib.RowsPlan(args.backend, algo, xin, ye, recip, isd, rows=rows, device=local,
                             stream=stream, **kw)
    sums = torch.zeros(p, dtype=torch.float64, device=tdev)
    sync()
    setup_ms = (time.perf_counter() - t0) * 1e3

    # reference order over ranks: every rank's float32 temp rows, then the
    # column sums passed rank to rank (parallel._chain_column_sums)
    chain = args.accumulation == "reference" and world > 1 and on_gpu

    def step():
        if chain:
            from fastselect_amd.parallel import _chain_column_sums
            plan.ref_temp()
            _chain_column_sums(plan, p, local)
            return
        if world > 1 and on_gpu:
            # the plan runs on its own stream: last step's all-reduce of sums
            # (on torch's stream) must have finished before it writes them
            torch.cuda.current_stream().synchronize()
        plan.score(sums.data_ptr())
        if world > 1:
            dist.all_reduce(sums, op=dist.ReduceOp.SUM)

    for w in range(args.warmup):
        step()
        sync()
        log(f"warmup {w} done")
    barrier()
    sync()
    t_start = time.perf_counter()
    kms = {0: [], 1: [], 2: []}
    for _ in range(args.steps):
        step()
        if on_gpu:
            for w in kms:
                kms[w].append(plan.kernel_ms(w))
    sync()
    barrier()
    elapsed = time.perf_counter() - t_start
    t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms_per_step = float(t.item()) / args.steps * 1e3
    roofline = None
    q16 = False
    surf_int = False
    if on_gpu:
        nb = (n + 127) // 128
        b0, b1 = rows[0] // 128, (rows[1] + 127) // 128
        # distance pairs this rank computes: every upper-triangle tile that
        # touches its focal blocks (algorithmic count: unique pairs of them)
        tiles = sum(1 for a in range(nb) for b in range(a, nb) if b0 <= a < b1 or b0 <= b < b1)
        pairs = min(tiles * 128.0 * 128.0, n * (n - 1) / 2.0)
        k_ms = float(np.mean(kms[0]))
        # SURF: integer distances resolved to the reference's float32 values
        # (fs_surfint.hip) unless the plan's calibration kept float64 ones
        surf_int = algo == "surf" and not plan.calibration()["surf_f64"]
        name = "k_dist" if algo == "relieff" or surf_int else "k_dist_f64"
        peak = VALU_PEAK_TFLOPS if algo == "relieff" or surf_int else VALU_F64_PEAK_TFLOPS
        # ReliefF's k_dist on 16-bit operands (n >= 4096): one v_sad_u16 per 2
        # PFE, one issue slot per PFE = 2 FMA-equivalent FLOPs (32-bit: 4)
        q16 = algo == "relieff" and bool(plan.calibration()["q16"])
        fpp = FLOP_PER_PFE // 2 if q16 else FLOP_PER_PFE
        achieved = fpp * pairs * p / (k_ms * 1e-3) / 1e12
        roofline = {"bound": "valu", "kernel": name, "achieved": achieved, "peak": peak,
                    "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
                    "flop_per_pfe": fpp, "pfe_per_launch": pairs * p,
                    "pfe_per_s": pairs * p / (k_ms * 1e-3),
                    "kernel_ms": {name: k_ms, "stage2": float(np.mean(kms[1]))}}
        if algo == "relieff":
            # k_rf_select: one float32 key row per focal sample read per launch
            sel_ms = float(np.mean(kms[2]))
            rbytes = (rows[1] - rows[0]) * n * 4.0
            roofline["kernel_ms"]["k_rf_select"] = sel_ms
            roofline["k_rf_select_hbm"] = {"bytes": rbytes, "GBps": rbytes / (sel_ms * 1e-3) / 1e9,
                                           "peak": HBM_PEAK_GBPS,
                                           "frac": rbytes / (sel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}
            roofline["peak_note"] = (
                "k_dist on 16-bit operands: v_sad_u16 takes 2 PFE per issue slot, so 1 slot per "
                "PFE = 2 FMA-equivalent FLOPs against the fp32 vector peak" if q16 else
                "k_dist on 32-bit operands: one half-rate v_sad_u32 per PFE = 4 FMA-equivalent "
                "FLOPs against the fp32 vector peak")
        elif surf_int:
            roofline["kernel_ms"]["surf_resolve"] = float(np.mean(kms[2]))
            roofline["refined_pairs"] = int(plan.info()[2])
            roofline["peak_note"] = (
                "k_dist on 32-bit operands: one half-rate v_sad_u32 per PFE = 4 FMA-equivalent "
                "FLOPs against the fp32 vector peak; surf_resolve: the row means and the pairs "
                "whose float32 distance they or a decision depend on, recomputed exactly")
        else:
            roofline["peak_note"] = ("float64 vector peak (AMD MI355X figure, half the fp32 rate); "
                                     "2 v_add_f64 per PFE, each priced as one FMA")
    plan.close()
    # ReliefF / SURF in reference order beside the default (N = 1): same plan type
    refacc = None
    if on_gpu and world == 1 and not args.no_ref and args.accumulation == "fast":
        with _lib.accumulation("reference"):
            rplan = _lib.RowsPlan(args.backend, algo, xin, ye, recip, isd, rows=rows,
                                  device=local, stream=stream, **kw)
        try:
            rplan.score(sums.data_ptr())
            sync()
            ks = max(1, min(args.steps, 3))
            t_r = time.perf_counter()
            for _ in range(ks):
                rplan.score(sums.data_ptr())
            sync()
            refacc = {"ms_per_step": (time.perf_counter() - t_r) / ks * 1e3, "steps": ks,
                      "kernel_ms": {"k_dist" if algo == "relieff" or surf_int else "k_dist_f64":
                                    rplan.kernel_ms(0),
                                    "selection_to_scores" if algo == "relieff"
                                    else "masks_and_chains": rplan.kernel_ms(1)},
                      "parity": "bit-identical to the oracle (tests/test_gpu_refacc.py)"}
        finally:
            rplan.close()
    out = None
    if rank == 0:
        name = "ReliefF k=%d" % cfg["k"] if algo == "relieff" else ("SURF*" if args.star else "SURF")
        out = {
            "metric": f"feature-scores/sec (n*p/s) {name} fp32",
            "value": n * p / (ms_per_step * 1e-3), "unit": "feature-scores/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None,
            "dtype": (f"{'u16' if q16 else 'u32'} pass 1 (exact keys near the k-th), fp32 / fp64 "
                      "update" if algo == "relieff" else
                      "u32 pass 1 (the reference's fp32 distances resolved exactly: fp64 "
                      "recomputation where a row sum or decision depends on one), fp32 pair sums"
                      if surf_int else "fp64 distances, fp32 pair sums")
                     + (" (SURF* star split: near pairs in pass 2, the far pairs per column from "
                        "its sorted values in fp64)" if algo == "surf" and args.star else ""),
            "data": f"synthetic make_classification(n_informative=20, n_redundant={cfg['red']}, "
                    f"random_state=42)",
            "config": {"workload": f"{name} n={n} p={p} (BASELINE configs[{cfg['idx']}])",
                       "name": args.config, "n_samples": n, "n_features": p,
                       "parallelism": f"focal-row shard x{world}"
                                      + (f", {'RCCL' if dist_backend == 'nccl' else dist_backend}"
                                         f" all-reduce" if world > 1 else "")},
            "roofline": roofline, "setup_ms": setup_ms,
            "accumulation": args.accumulation,
        }
        if refacc is not None:
            out["reference_accumulation"] = refacc
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline (oracle) ...")
            out["cpu_baseline"] = cpu_baseline_rows(algo, X, y, cfg.get("k", 0), args.star)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg4", choices=sorted(CONFIGS),
                    help="BASELINE.json configuration (cfg4: the headline MultiSURF 20000x20000)")
    ap.add_argument("--samples", type=int, default=None)
    ap.add_argument("--features", type=int, default=None)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--star", action="store_true")
    ap.add_argument("--no-q32", action="store_true",
                    help="skip the 32-bit pass-1 comparison step time (MultiSURF at N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--accumulation", default="fast", choices=("fast", "reference"),
                    help="the timed step's accumulation mode (reference: the reference's "
                         "float32 per-sample chains and column sums, bit-identical scores)")
    ap.add_argument("--no-ref", action="store_true",
                    help="skip the reference-order step time beside the default (N=1)")
    ap.add_argument("--no-fit", action="store_true", help="skip the end-to-end fit() timing")
    ap.add_argument("--backend", default="gpu", choices=("gpu", "cpu"),
                    help="cpu: rehearse the multi-rank job on host threads (gloo, tests only)")
    ap.add_argument("--dist-backend", default=None,
                    help="torch.distributed backend for N > 1 (default nccl = RCCL over xGMI "
                         "on the GPU, gloo with --backend cpu)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    cfg = CONFIGS[args.config]
    args.samples = args.samples or cfg["n"]
    args.features = args.features or cfg["p"]
    args.star = args.star or cfg["star"]
    dist_backend = args.dist_backend or ("nccl" if args.backend == "gpu" else "gloo")

    # --gpus N without a launcher: start the N ranks here, before any GPU call
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF, resident_x

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch exactly "
                         f"one rank per GPU")
    on_gpu = args.backend == "gpu"
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if on_gpu:
        ndev = torch.cuda.device_count()
        if dist_backend == "nccl" and ndev < world:
            raise SystemExit(f"bench.py: {world} ranks need {world} visible GPUs, found {ndev}")
        # a gloo rehearsal may put several ranks on one GPU
        local %= max(1, ndev)
        torch.cuda.set_device(local)
    if world > 1:
        if dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(dist_backend)

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    if cfg["algo"] != "multisurf":
        return bench_rows(args, cfg, world, rank, local, on_gpu, dist, sync, barrier,
                          dist_backend)

    t0 = time.perf_counter()
    X, y = make_data(args.samples, args.features, args.seed, cfg["red"])
    x = X.astype(np.float32)
    ranges = (x.max(axis=0) - x.min(axis=0)).astype(np.float32)
    ranges[ranges == 0] = 1
    recip = (1.0 / ranges).astype(np.float32)
    # make_classification columns are continuous; discrete detection is part
    # of fit() (timed separately in fit_ms), not of a step
    is_disc = np.zeros(args.features, dtype=bool)
    log(f"rank {rank}/{world}: data {args.samples}x{args.features} ready in "
        f"{time.perf_counter() - t0:.1f} s")

    # X onto the GPUs: at N > 1 each rank uploads its n/N rows and the rest
    # arrive by an RCCL all-gather (parallel.resident_x); the plan then copies
    # the gathered X device-to-device
    barrier()
    sync()
    t0 = time.perf_counter()
    with resident_x(x, args.backend, local):
        job = ShardedMultiSURF(x, y, recip, is_disc, use_star=args.star, backend=args.backend,
                               device=local, accumulation=args.accumulation)
    sync()
    setup_ms = (time.perf_counter() - t0) * 1e3
    ref_mode = args.accumulation == "reference"
    tiles, _, _ = job.info()
    q16_used = bool(job.plan.calibration()["q16"]) if on_gpu else False

    for w in range(args.warmup):
        job.step()
        sync()
        log(f"warmup {w} done")
    barrier()
    sync()
    t_start = time.perf_counter()
    dist_ms, score_ms = [], []
    for s in range(args.steps):
        job.step()
        if on_gpu:
            dist_ms.append(job.kernel_ms(0))
            score_ms.append(job.kernel_ms(1))
    sync()
    barrier()
    elapsed = time.perf_counter() - t_start
    _, _, refined = job.info()
    weighted = job.weighted_pairs()  # non-zero pass-2 weights (sparse pass 2), -1 if dense
    step_counts = job.counts.cpu().numpy()
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    n, p = args.samples, args.features

    roofline = None
    if on_gpu:
        # dominant kernel roofline (rank-local launch).  Algorithmic count of
        # pass 1: unique pairs x features / world (padding and the duplicated
        # half of diagonal tiles are executed but not counted); of pass 2: the
        # pairs with a non-zero weight x features when pass 2 is sparse (the
        # work the reference's near/far accumulation needs), else every pair.
        d_ms, s_ms = float(np.mean(dist_ms)), float(np.mean(score_ms))
        pairs_dense = n * (n - 1) / 2.0 / world
        pairs_score = weighted if weighted >= 0 else pairs_dense
        score_name = "k_score_sparse" if weighted >= 0 else "k_score"
        if ref_mode:  # the chains walk directed entries (one per focal side)
            score_name, weighted = "k_ms_chains", -1
            # rank-local: each rank walks the chains of its 1/world of the
            # focal rows (ShardedMultiSURF._step_reference)
            pairs_score = chain_entries(step_counts, y, args.star) / world
        pfe = {"k_dist": pairs_dense * p, score_name: pairs_score * p}
        kern = {"k_dist": d_ms, score_name: s_ms}
        dom = max(kern, key=kern.get)
        # FMA-equivalent FLOPs per PFE: k_dist 2 on 16-bit operands (one
        # v_sad_u16 per 2 PFE), 4 on 32-bit (half-rate v_sad_u32); pass 2 4;
        # the reference-order chains 6 (sub, mul, add)
        fpp = {"k_dist": FLOP_PER_PFE // 2 if q16_used else FLOP_PER_PFE,
               score_name: FLOP_PER_PFE_CHAINS if ref_mode else FLOP_PER_PFE}
        achieved = fpp[dom] * pfe[dom] / (kern[dom] * 1e-3) / 1e12
        # bytes the tiles stream from L2/HBM into the CUs (both row panels of
        # every owned tile, + the D write / the pair weights): on-chip reuse
        # traffic, NOT the algorithmic HBM bytes
        w_bytes = weighted * 8 if weighted >= 0 else tiles * 128 * 128 * 4
        panel_bytes = {"k_dist": tiles * (2 * 128 * p * 4 + 2 * 128 * 128 * 8),
                       score_name: tiles * 2 * 128 * p * 4 + w_bytes}
        # algorithmic HBM bytes: X once per kernel, D written
        # by pass 1 (8-byte entries, both halves), the pair weights read by pass 2
        alg_bytes = {"k_dist": n * p * 4 / world + n * n * 8 / world,
                     score_name: n * p * 4 + w_bytes}
        traffic = {k: pmc_traffic(k, n, p, world)[0] for k in kern}
        roofline = {
            "bound": "valu", "kernel": dom, "achieved": achieved,
            "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / VALU_PEAK_TFLOPS,
            "traffic": traffic[dom],
            "traffic_source": pmc_traffic(dom, n, p, world)[1],
            "traffic_per_kernel": traffic,
            "flop_per_pfe": fpp[dom],
            "pfe_per_s": pfe[dom] / (kern[dom] * 1e-3),
            "valu_frac_per_kernel": {k: fpp[k] * pfe[k] / (kern[k] * 1e-3) / 1e12 / VALU_PEAK_TFLOPS
                                     for k in kern},
            "kernel_ms": kern,
            "pfe_per_launch": pfe[dom],
            "pass2_weighted_pairs": weighted,
            "pass2_pair_density": (pairs_score / pairs_dense) if pairs_dense else None,
            "hbm_alg_GBps": {k: alg_bytes[k] / (kern[k] * 1e-3) / 1e9 for k in kern},
            "hbm_alg_frac": {k: alg_bytes[k] / (kern[k] * 1e-3) / 1e9 / HBM_PEAK_GBPS
                             for k in kern},
            "onchip_panel_GBps": {k: panel_bytes[k] / (kern[k] * 1e-3) / 1e9 for k in kern},
            "hbm_peak_GBps": HBM_PEAK_GBPS,
            # the measured traffic of the dominant kernel (rocprofv3 FETCH x2 +
            # WRITE per launch, profiles/pmc_traffic.json) over its launch time
            "hbm_measured_GBps": (traffic[dom] / (kern[dom] * 1e-3) / 1e9
                                  if traffic[dom] else None),
            "hbm_measured_frac": (traffic[dom] / (kern[dom] * 1e-3) / 1e9 / HBM_PEAK_GBPS
                                  if traffic[dom] else None),
        }
    job.close()
    # the decision-finer 32-bit pass 1 beside the default step (VERDICT r2
    # next #6): same job, 32-bit operands forced by the q16 test hook
    q32 = None
    if on_gpu and world == 1 and not args.no_q32 and not ref_mode:
        _lib.set_test_hook("q16", 0)
        try:
            with resident_x(x, args.backend, local):
                job32 = ShardedMultiSURF(x, y, recip, is_disc, use_star=args.star,
                                         backend=args.backend, device=local)
            job32.step()
            sync()
            t_q = time.perf_counter()
            ks = max(1, min(args.steps, 3))
            for _ in range(ks):
                job32.step()
            sync()
            q32 = {"ms_per_step": (time.perf_counter() - t_q) / ks * 1e3,
                   "kernel_ms": {"k_dist": job32.kernel_ms(0), "pass2": job32.kernel_ms(1)},
                   "steps": ks}
            job32.close()
        finally:
            _lib.set_test_hook("reset")
    # the reference-order step beside the default (its
    # cost at cfg2 / cfg4): same job, accumulation='reference'
    refacc = None
    if on_gpu and world == 1 and not args.no_ref and not ref_mode:
        def make_ref():
            with resident_x(x, args.backend, local):
                return ShardedMultiSURF(x, y, recip, is_disc, use_star=args.star,
                                        backend=args.backend, device=local,
                                        accumulation="reference")
        refacc = reference_step(make_ref, y, args.star, p, sync, max(1, min(args.steps, 3)))
    setup = torch.tensor([setup_ms], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
    if world > 1:
        dist.all_reduce(setup, op=dist.ReduceOp.MAX)

    out = None
    if rank == 0:
        out = {
            "metric": "feature-scores/sec (n*p/s) MultiSURF fp32",
            "value": n * p / (ms_per_step * 1e-3),
            "unit": "feature-scores/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": f"{'u16' if q16_used else 'u32'} pass 1, fp32 pass 2 (fp64 accumulation)",
            "arith": "pass 1: integer L1 distances (v_sad_u16 on 16-bit operands for n >= 16384, "
                     "else v_sad_u32), pairs near a threshold recomputed in the reference's "
                     "float32 arithmetic; pass 2 over the pairs with a non-zero weight: f32 diffs x "
                     "f32 pair weights, f64 accumulation"
                     + ("; MultiSURF* star split: pass 2 over the near pairs, the far misses' "
                        "all-pairs part per column from its sorted values (k_star_terms, f64)"
                        if args.star else ""),
            "data": "synthetic make_classification(n_informative=20, n_redundant=100, random_state=42)",
            "config": {"workload": f"MultiSURF{'*' if args.star else ''} n={n} p={p} "
                                   f"(BASELINE configs[{cfg['idx']}])",
                       "name": args.config,
                       "n_samples": n, "n_features": p,
                       "parallelism": f"pair-tile shard x{world}"
                                      + (f", {'RCCL' if dist_backend == 'nccl' else dist_backend}"
                                         f" all-reduce" if world > 1 else "")
                                      + (", decision-mask all-reduce + column sums chained "
                                         "over the ranks" if world > 1 and ref_mode else "")},
            "roofline": roofline,
            "refined_pairs": refined,
            # X to the GPUs (per-rank rows + all-gather at N > 1) + plan
            # creation (device ranges, calibration, layout), max over ranks
            "setup_ms": float(setup.item()),
            "pass1_operands": "16-bit" if q16_used else "32-bit",
            "accumulation": args.accumulation,
            # the timed step's near/far decisions against the reference's
            # (VERDICT r4 next #2), when the oracle's decisions are committed
            "decisions_vs_reference": decisions_vs_fixture(step_counts, n, p, args.config)
            if args.seed == 42 else None,
        }
        if ref_mode:
            out["arith"] = ("pass 1: integer L1 distances on 32-bit operands, pairs near a "
                            "threshold and the thresholds of flagged rows recomputed in the "
                            "reference's arithmetic; pass 2: the reference's float32 per-sample "
                            "hit / miss chains in sample order and float32 sequential column "
                            "sums (bit-identical to the oracle)")
        if q32 is not None:
            out["q32_pass1"] = q32
        if refacc is not None:
            out["reference_accumulation"] = refacc
    if on_gpu and world == 1 and not args.no_fit:
        log("timing end-to-end fit() ...")
        med, ts = fit_ms(X, y, args.star)
        out["fit_ms"] = med
        out["fit_ms_runs"] = ts
        out["fit_feature_scores_per_s"] = n * p / (med * 1e-3)
    elif on_gpu and world > 1 and not args.no_fit:
        log("timing end-to-end multi-GPU scoring ...")
        med, ts = sharded_fit_ms(X, y, args.star, local, barrier, sync, dist)
        if rank == 0:
            out["fit_ms"] = med
            out["fit_ms_runs"] = ts
            out["fit_feature_scores_per_s"] = n * p / (med * 1e-3)
            out["fit_path"] = ("parallel.multisurf_scores: float32 cast, per-rank rows + RCCL "
                               "all-gather of X, column statistics, plan, step, all-reduces; "
                               "max over ranks")
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline (oracle) ...")
            out["cpu_baseline"] = cpu_baseline(x, y)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
