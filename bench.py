"""Benchmark: MultiSURF feature scoring on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--samples 20000 --features 20000]

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
FLOP_PER_PFE = 4
HBM_PEAK_GBPS = 8000.0
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


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def make_data(n, p, seed):
    from sklearn.datasets import make_classification
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=100,
                               random_state=seed)
    return X.astype(np.float32), y


def cpu_baseline(x, y, budget_s=25.0):
    """Oracle MultiSURF on the first m focal samples, extrapolated to n: a
    small untimed run (page-in, thread start), a short run to measure the
    per-sample rate, then a ~budget_s sample whose time is reported."""
    from oracle import oracle as O
    O.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = min(threads, 16)
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
    return {"value": n * p / t_full, "unit": "feature-scores/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle MultiSURF (C/OpenMP restatement of the reference backend='cpu') "
                      f"on focal samples [0, {m}) of the same {n}x{p} data: {t:.2f} s, "
                      f"extrapolated x{n / m:.1f} to {t_full:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--samples", type=int, default=20000)
    ap.add_argument("--features", type=int, default=20000)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--star", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; "
                         "gloo only to rehearse several ranks on one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one GPU per local rank; ranks beyond the visible GPUs share them (only
    # meaningful for a gloo rehearsal)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)

    t0 = time.perf_counter()
    x, y = make_data(args.samples, args.features, args.seed)
    ranges = (x.max(axis=0) - x.min(axis=0)).astype(np.float32)
    ranges[ranges == 0] = 1
    recip = (1.0 / ranges).astype(np.float32)
    # make_classification columns are continuous; the estimator's np.unique
    # discrete detection (host, ~2 s here) is part of fit(), not of a step
    is_disc = np.zeros(args.features, dtype=bool)
    log(f"rank {rank}/{world}: data {args.samples}x{args.features} ready in {time.perf_counter() - t0:.1f} s")

    job = ShardedMultiSURF(x, y, recip, is_disc, use_star=args.star, backend="gpu", device=local)
    tiles, _, _ = job.info()

    def barrier():
        if world > 1:
            dist.barrier()

    for w in range(args.warmup):
        job.step()
        torch.cuda.synchronize()
        log(f"warmup {w} done")
    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    dist_ms, score_ms = [], []
    for s in range(args.steps):
        scores = job.step()
        dist_ms.append(job.kernel_ms(0))
        score_ms.append(job.kernel_ms(1))
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    _, _, refined = job.info()
    weighted = job.weighted_pairs()  # non-zero pass-2 weights (sparse pass 2), -1 if dense
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3

    # dominant kernel roofline (rank-local launch).  Algorithmic count of
    # pass 1: unique pairs x features / world (padding and the duplicated half
    # of diagonal tiles are executed but not counted); of pass 2: the pairs
    # with a non-zero weight x features when pass 2 is sparse (the work the
    # reference's near/far accumulation needs), else every unique pair.
    d_ms, s_ms = float(np.mean(dist_ms)), float(np.mean(score_ms))
    pairs_dense = args.samples * (args.samples - 1) / 2.0 / world
    pairs_score = weighted if weighted >= 0 else pairs_dense
    score_name = "k_score_sparse" if weighted >= 0 else "k_score"
    pfe = {"k_dist": pairs_dense * args.features, score_name: pairs_score * args.features}
    kern = {"k_dist": d_ms, score_name: s_ms}
    dom = max(kern, key=kern.get)
    pfe_launch = pfe[dom]
    achieved = FLOP_PER_PFE * pfe_launch / (kern[dom] * 1e-3) / 1e12
    # algorithmic bytes one launch moves from HBM/L2 into the CUs: both row
    # panels of every owned tile once (+ D write for k_dist; the pair weights
    # for k_score: 8-byte entries when sparse, the dense 128x128 f32 tiles else)
    w_bytes = weighted * 8 if weighted >= 0 else tiles * 128 * 128 * 4
    alg_bytes = {"k_dist": tiles * (2 * 128 * args.features * 4 + 2 * 128 * 128 * 8),
                 score_name: tiles * 2 * 128 * args.features * 4 + w_bytes}
    traffic, traffic_src = pmc_traffic(dom, args.samples, args.features, world)

    if rank == 0:
        out = {
            "metric": "feature-scores/sec (n*p/s) MultiSURF fp32",
            "value": args.samples * args.features / (ms_per_step * 1e-3),
            "unit": "feature-scores/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "arith": "pass 1: integer L1 distances (v_sad_u16 on 16-bit operands for n >= 16384, "
                     "else v_sad_u32), pairs near a threshold recomputed in the reference's "
                     "float32 arithmetic; pass 2 over the pairs with a non-zero weight: f32 diffs x "
                     "f32 pair weights, f64 accumulation",
            "data": "synthetic make_classification(n_informative=20, n_redundant=100, random_state=42)",
            "config": {"workload": f"MultiSURF{'*' if args.star else ''} n={args.samples} "
                                   f"p={args.features} (BASELINE configs[3])",
                       "n_samples": args.samples, "n_features": args.features,
                       "parallelism": f"pair-tile shard x{world}, "
                                      f"{'RCCL' if args.dist_backend == 'nccl' else args.dist_backend}"
                                      f" all-reduce"},
            "roofline": {
                "bound": "valu", "kernel": dom, "achieved": achieved,
                "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / VALU_PEAK_TFLOPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "flop_per_pfe": FLOP_PER_PFE,
                "pfe_per_s": pfe_launch / (kern[dom] * 1e-3),
                "kernel_ms": kern,
                "pfe_per_launch": pfe_launch,
                "pass2_weighted_pairs": weighted,
                "pass2_pair_density": (pairs_score / pairs_dense) if pairs_dense else None,
                "hbm_alg_GBps": {k: alg_bytes[k] / (kern[k] * 1e-3) / 1e9 for k in kern},
                "hbm_peak_GBps": HBM_PEAK_GBPS,
            },
            "refined_pairs": refined,
        }
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline (oracle) ...")
            out["cpu_baseline"] = cpu_baseline(x, y)
        print(json.dumps(out), flush=True)
    job.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
