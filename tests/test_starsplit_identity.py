"""The star split's algebra on the CPU (fs_starterm.hip; DESIGN.md §Star
split), independent of the GPU code: for MultiSURF* and SURF* the dense sum
sum_ij w_ij d_f(i, j) equals the near-only sum with the split's weights plus
the per-column term U_f computed the way k_star_terms does -- one sort of the
column, S_all(i) = v_k (2k - n) - 2 P_k + T, the same per class from that
class's prefix at i's position (for a sample of any class), equal-value counts
for discrete columns.  Small float64 problems, 3 classes, ties, a discrete
column, focal-row slices (alpha = 0 off the slice)."""
import numpy as np
import pytest


def _problem(seed, n=160, p=12, n_cls=3):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, p))
    X[:, 0] = rng.integers(0, 5, n)            # a value grid: many ties
    X[:, 1] = rng.integers(0, 3, n)            # treated as discrete below
    y = rng.integers(0, n_cls, n)
    disc = np.zeros(p, dtype=bool)
    disc[1] = True
    return X, y, disc


def _diffs(X, disc):
    d = np.abs(X[:, None, :] - X[None, :, :])
    d[:, :, disc] = (X[:, None, disc] != X[None, :, disc]).astype(float)
    return d  # [i, j, f]


def _near(X, disc, algo):
    D = _diffs(X, disc).sum(axis=2)
    n = len(X)
    off = ~np.eye(n, dtype=bool)
    mu = np.array([D[i, off[i]].mean() for i in range(n)])
    if algo == "multisurf":
        sd = np.array([D[i, off[i]].std() for i in range(n)])
        thr = mu - sd / 2
    else:
        thr = mu
    return (D < thr[:, None]) & off


def _dense(X, y, disc, algo, focal):
    near = _near(X, disc, algo)
    hit = y[:, None] == y[None, :]
    n = len(X)
    off = ~np.eye(n, dtype=bool)
    if algo == "multisurf":
        H = (near & hit).sum(1).astype(float)
        M = (near & ~hit).sum(1).astype(float)
        Hs = np.where(H > 0, H, 1.0)[:, None]
        Mp = np.where(M > 0, M, 1.0)[:, None]
        w = np.where(near, np.where(hit, -1.0 / Hs, 1.0 / Mp), np.where(hit, 0.0, -1.0 / Mp))
    else:
        w = np.where(near, np.where(hit, -1.0, 1.0), np.where(hit, 1.0, -1.0))
    w = w * off * focal[:, None]
    return np.einsum("ij,ijf->f", w, _diffs(X, disc)), near, hit, off


def _column_term(v, y, alpha, gamma, discrete, n_cls):
    """U_f as k_star_terms forms it (sorted order, prefix sums / run bounds)."""
    n = len(v)
    order = np.argsort(v, kind="stable")
    vs, cs, al = v[order], y[order], alpha[order]
    k = np.arange(n)
    if discrete:
        lo = np.searchsorted(vs, vs, side="left")
        hi = np.searchsorted(vs, vs, side="right")
        s_all = n - (hi - lo)
    else:
        P = np.concatenate([[0.0], np.cumsum(vs)[:-1]])
        s_all = vs * (2 * k - n) - 2 * P + vs.sum()
    s_same = np.zeros(n)
    for c in range(n_cls):
        m = cs == c
        if discrete:
            cnt = np.concatenate([[0], np.cumsum(m)])  # class-c items before each position
            eq = cnt[hi] - cnt[lo]
            g = m.sum() - eq
        else:
            lc = np.concatenate([[0], np.cumsum(m)[:-1]])
            ls = np.concatenate([[0.0], np.cumsum(np.where(m, vs, 0.0))[:-1]])
            g = vs * (2 * lc - m.sum()) - 2 * ls + vs[m].sum()
        s_same = np.where(m, g, s_same)
    return float(np.sum(al * (gamma * s_same - s_all)))


@pytest.mark.parametrize("algo", ["multisurf", "surf"])
@pytest.mark.parametrize("seed,rows", [(1, None), (2, (40, 120))])
def test_split_identity(algo, seed, rows):
    X, y, disc = _problem(seed)
    n, p = X.shape
    focal = np.zeros(n)
    lo, hi = rows or (0, n)
    focal[lo:hi] = 1.0
    dense, near, hit, off = _dense(X, y, disc, algo, focal)
    # near-only part with the split's weights
    if algo == "multisurf":
        H = (near & hit).sum(1).astype(float)
        M = (near & ~hit).sum(1).astype(float)
        Mp = np.where(M > 0, M, 1.0)
        w = np.where(near, np.where(hit, -1.0 / np.where(H > 0, H, 1.0)[:, None],
                                    2.0 / Mp[:, None]), 0.0)
        alpha, gamma = focal / Mp, 1.0
    else:
        w = np.where(near, np.where(hit, -2.0, 2.0), 0.0)
        alpha, gamma = focal, 2.0
    w = w * off * focal[:, None]
    split = np.einsum("ij,ijf->f", w, _diffs(X, disc))
    split += [_column_term(X[:, f], y, alpha, gamma, disc[f], 3) for f in range(p)]
    np.testing.assert_allclose(split, dense, rtol=1e-9, atol=1e-9 * np.abs(dense).max())
