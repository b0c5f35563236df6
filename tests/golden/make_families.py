"""Generate tests/golden/family_*.npz: oracle MultiSURF / MultiSURF* scores
on data families other than make_classification, at n = 16384, where the
default GPU pass 1 takes 16-bit operands (the pass-1
cut-offs and band were tuned on make_classification only).

    uniform_16k    X ~ U(0, 1) iid, labels independent of X: no signal, so
                   the distance distribution of a row is narrow (sigma /
                   mean ~ 1/sqrt(p)) and many pairs sit near mu - sigma/2
    lognormal_16k  X = exp(3 z), z ~ N(0, 1) plus a class shift on 30
                   features: every column's range is set by a few extreme
                   values, so most samples share a handful of 16-bit levels
                   (the quantisation error is large against typical diffs)
    mixed_16k      make_classification continuous features beside 400
                   integer features with 3-8 levels (is_discrete: the
                   mismatch count of MultiSURF.py:185-190) and 200 columns
                   on a coarse 0.25 grid (continuous, coherent rounding)

p = 2000 in each.  Every fixture holds the C oracle's scores for use_star
False and True (oracle/relief_oracle.c, the restatement of
MultiSURF.py:165-253) and the sha256 of X, which the GPU test regenerates
and checks.

Run (container; ~6 min per case on 8 cores):
    python tests/golden/make_families.py [names...]
    python tests/golden/make_families.py --f64 [names...]        (float64 sums)
    python tests/golden/make_families.py --decisions [names...]  (thresholds, counts)
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

N, P = 16384, 2000
CASES = ("uniform_16k", "lognormal_16k", "mixed_16k")


def make(name):
    """(X float32, y) of one case (deterministic)."""
    if name == "uniform_16k":
        rng = np.random.default_rng(11)
        X = rng.random((N, P), dtype=np.float32)
        y = rng.integers(0, 2, N)
    elif name == "lognormal_16k":
        rng = np.random.default_rng(12)
        y = rng.integers(0, 2, N)
        z = rng.standard_normal((N, P), dtype=np.float32)
        z[:, :30] += 0.5 * y[:, None].astype(np.float32)
        X = np.exp(3.0 * z).astype(np.float32)
    elif name == "mixed_16k":
        from sklearn.datasets import make_classification
        X, y = make_classification(n_samples=N, n_features=P, n_informative=20,
                                   n_redundant=50, random_state=13)
        X = X.astype(np.float32)
        rng = np.random.default_rng(13)
        levels = rng.integers(3, 9, 400)
        X[:, 100:500] = (rng.random((N, 400)) * levels).astype(np.int32).astype(np.float32)
        X[:, 100:110] += y[:, None].astype(np.float32)          # a few informative ones
        X[:, 600:800] = np.round(X[:, 600:800] * 4.0) / 4.0
    else:
        raise KeyError(name)
    return np.ascontiguousarray(X), np.asarray(y)


def digest(x):
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def run(name):
    from oracle import oracle as O
    t0 = time.time()
    X, y = make(name)
    s0 = O.multisurf_scores(X, y, use_star=False)
    s1 = O.multisurf_scores(X, y, use_star=True)
    out = os.path.join(HERE, f"family_{name}.npz")
    np.savez(out, x_sha256=np.array(digest(X)), y_sum=np.array(int(np.sum(y))),
             scores=s0.astype(np.float32), scores_star=s1.astype(np.float32))
    print(f"{name}: {time.time() - t0:.0f} s -> {out}", flush=True)


def run_f64(name):
    """family_<name>_f64.npz: MultiSURF with the oracle's accum='f64' (the
    reference's diffs, distances and near/far decisions, every later sum in
    float64) -- the attribution reference where the scores sit at the
    reference's own float32 rounding level (signal-free data)."""
    from oracle import oracle as O
    t0 = time.time()
    X, y = make(name)
    s0 = O.multisurf_scores(X, y, use_star=False, accum="f64")
    out = os.path.join(HERE, f"family_{name}_f64.npz")
    np.savez(out, x_sha256=np.array(digest(X)), scores=s0.astype(np.float64))
    print(f"{name} f64: {time.time() - t0:.0f} s -> {out}", flush=True)


def run_decisions(name):
    """family_<name>_decisions.npz: the reference's near/far decisions alone
    (oracle_multisurf_decisions: thresholds mu - sigma/2 and every row's near
    hit / near miss counts, MultiSURF.py:175-217) -- a score residual with
    identical counts is accumulation, not decisions."""
    from oracle import oracle as O
    t0 = time.time()
    X, y = make(name)
    thr, counts = O.multisurf_decisions(X, y)
    out = os.path.join(HERE, f"family_{name}_decisions.npz")
    np.savez_compressed(out, x_sha256=np.array(digest(X)), thr=thr, counts=counts.astype(np.int32))
    print(f"{name} decisions: {time.time() - t0:.0f} s -> {out}", flush=True)


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--decisions":
        for nm in args[1:] or list(CASES):
            run_decisions(nm)
    elif args and args[0] == "--f64":
        for nm in args[1:] or list(CASES):
            run_f64(nm)
    else:
        for nm in args or list(CASES):
            run(nm)
