"""Generate tests/golden/rowcoherent_*.npz: oracle scores on inputs whose
pass-1 quantisation error is coherent within a few ROWS (VERDICT r2, weak #2
and next #1c), at n = 16384, where MultiSURF's default pass 1 takes 16-bit
operands (MultiSURF* from 10000).

The 16-bit operands are q = trunc(t + 0.5) of t = (x - min) * recip * SC with
SC ~ 65534 (fs_prep.cpp set_integer_scale).  A row whose values all sit 0.6
of a quantum above a grid point rounds every feature the same way (error
eps ~ +0.4 per feature).  When the row also sits below almost every other
sample in every column (at the column minimum), the signs in the pair error
sum_f sign(t_i - t_j)(eps_i - eps_j) agree too, and the distance error of
each of its pairs is ~ -0.4 * pc integer units: 800 at pc = 2000, against the
refinement band's ~220 for independent rounding.  The whole-matrix sampled
calibration (4096 pairs) sees such rows only by chance:

    minrows_16k   40 rows at min + 0.6 quantum in every column (~20 sampled
                  pairs touch them)
    minrow4_16k   4 such rows (~2 sampled pairs; none with probability ~0.14)
    gridrows_16k  1% of the rows (164) moved to the 0.6-quantum grid where
                  they are (coherent rounding, signs mixed)

Base data: make_classification(n=16384, p=2000, n_informative=20,
n_redundant=50, random_state=7) as float32; labels from it.  Each fixture
holds the C oracle's MultiSURF scores (oracle/relief_oracle.c, the
restatement of MultiSURF.py:165-253) for use_star False and True and the
sha256 of X, which the GPU test regenerates and checks.

Run (container; ~6 min per case on 8 cores):
    python tests/golden/make_rowcoherent.py [names...]
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
CASES = {"minrows_16k": 40, "minrow4_16k": 4, "gridrows_16k": 164}
QUANTA = 65534.0


def make(name):
    """(X float32, y) of one case (deterministic)."""
    from sklearn.datasets import make_classification
    rows = CASES[name]
    X, y = make_classification(n_samples=N, n_features=P, n_informative=20, n_redundant=50,
                               random_state=7)
    X = X.astype(np.float32)
    rng = np.random.default_rng(1000 + rows)
    pick = np.sort(rng.choice(np.arange(2, N), size=rows, replace=False))
    mn = X.min(axis=0).astype(np.float64)
    rg = X.max(axis=0).astype(np.float64) - mn
    q = rg / QUANTA
    if name.startswith("grid"):
        k = np.floor((X[pick].astype(np.float64) - mn) / q)
        X[pick] = (mn + (k + 0.6) * q).astype(np.float32)
    else:
        X[pick] = (mn + 0.6 * q).astype(np.float32)
    return np.ascontiguousarray(X), y


def digest(x):
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def run(name):
    from oracle import oracle as O
    t0 = time.time()
    X, y = make(name)
    s0 = O.multisurf_scores(X, y, use_star=False)
    s1 = O.multisurf_scores(X, y, use_star=True)
    out = os.path.join(HERE, f"rowcoherent_{name}.npz")
    np.savez(out, x_sha256=np.array(digest(X)), y_sum=np.array(int(y.sum())),
             scores=s0.astype(np.float32), scores_star=s1.astype(np.float32))
    print(f"{name}: {time.time() - t0:.0f} s -> {out}", flush=True)


if __name__ == "__main__":
    for nm in sys.argv[1:] or list(CASES):
        run(nm)
