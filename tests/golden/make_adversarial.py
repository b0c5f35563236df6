"""Generate tests/golden/adversarial_*.npz: oracle scores on inputs whose
quantisation errors add up coherently across features.

The pass-1 refinement band of the GPU path was derived for independent
per-feature rounding; these inputs break that assumption on purpose:

    dup        4 base columns, each repeated 4000 times (p = 16000): every
               copy of a column rounds the same way, so a pair's distance
               error is 4000x one column's instead of ~sqrt(16000)x
    intgrid    integer-valued columns 0..30 (31 distinct values, so
               continuous), all with the same range: the rounding error of a
               value depends on the value only, identically in every column
    collinear  8 base columns, p = 8000 affine copies a*x + b (float32), so
               the scaled values agree up to float32 rounding

Each fixture holds the C oracle's MultiSURF scores (oracle/relief_oracle.c,
the restatement of the reference backend='cpu', MultiSURF.py:165-253) for
use_star False and True, the generator's seed and the sha256 of the float32
X, so that a GPU test regenerates X and checks it is the same input.

The *_16k variants (n = 16384, p = 2000) are the same constructions at the
size from which MultiSURF's default pass 1 takes 16-bit operands (MultiSURF*
from 10000), so the default path meets them with the coherence guard.

Run (container; ~2-7 min per case on 8 cores):
    python tests/golden/make_adversarial.py [names...]
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# name: (n, p)
SIZES = {"dup": (3000, 16000), "intgrid": (3000, 6000), "collinear": (3000, 8000),
         "dup_16k": (16384, 2000), "intgrid_16k": (16384, 2000), "collinear_16k": (16384, 2000)}


def make(name):
    """(X float32, y int) of one adversarial case (deterministic)."""
    kind = name.split("_")[0]
    n, p = SIZES[name]
    seed = {"dup": 101, "intgrid": 202, "collinear": 303}[kind]
    rng = np.random.default_rng(seed if n == 3000 else seed + n)
    if kind == "dup":
        base = rng.standard_normal((n, 4)).astype(np.float32)
        X = np.repeat(base, p // 4, axis=1)          # column k = base column k // (p/4)
        y = (base[:, 0] + base[:, 1] > 0).astype(np.int64)
    elif kind == "intgrid":
        X = rng.integers(0, 31, size=(n, p)).astype(np.float32)
        X[0, :] = 0.0                                # every column spans exactly 0..30
        X[1, :] = 30.0
        y = (X[:, 2] + X[:, 3] + rng.integers(0, 8, n) > 33).astype(np.int64)
    elif kind == "collinear":
        base = rng.standard_normal((n, 8)).astype(np.float32)
        a = rng.uniform(0.5, 4.0, p).astype(np.float32)
        b = rng.uniform(-3.0, 3.0, p).astype(np.float32)
        X = (base[:, np.arange(p) % 8] * a + b).astype(np.float32)
        y = (base[:, 0] - base[:, 3] > 0.2).astype(np.int64)
    else:
        raise KeyError(name)
    return np.ascontiguousarray(X), y


def base_of(name, p):
    """Base column of each column (top-k is compared per base column: copies tie)."""
    kind = name.split("_")[0]
    if kind == "dup":
        return np.arange(p) // (p // 4)
    if kind == "collinear":
        return np.arange(p) % 8
    return np.arange(p)


def digest(x):
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def run(name):
    from oracle import oracle as O
    t0 = time.time()
    X, y = make(name)
    s0 = O.multisurf_scores(X, y, use_star=False)
    s1 = O.multisurf_scores(X, y, use_star=True)
    out = os.path.join(HERE, f"adversarial_{name}.npz")
    np.savez(out, x_sha256=np.array(digest(X)), y_sum=np.array(int(y.sum())),
             scores=s0.astype(np.float32), scores_star=s1.astype(np.float32))
    print(f"{name}: {time.time() - t0:.0f} s -> {out}", flush=True)


if __name__ == "__main__":
    for nm in sys.argv[1:] or list(SIZES):
        run(nm)
