"""Regenerate the committed fixtures in tests/golden/.

* reference_fixtures.npz -- the input arrays the reference's own tests use
  (tests/test_multisurf.py:19-33, tests/test_relieff.py:21-31,
  tests/test_surf.py:22-32, the discrete-limit array of
  tests/test_multisurf.py:99-100).  Data only.
* cfg1_reference.json -- the reference's MultiSURF output on the README
  quickstart dataset (README.md:79-85, BASELINE cfg1), as recorded by the
  survey run of the reference: top-15 feature set and
  max|score|, plus the sha256 prefix of the generated X.
* oracle_vectors.npz -- outputs of the C oracle (oracle/relief_oracle.c) on
  small seeded datasets, for regression checks.  Oracle-generated (the
  reference itself cannot run in this image: numba is absent).

Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def reference_fixtures():
    ms_x = np.array([
        [1.1, 5.0, 10, 3.0], [1.2, 4.0, 10, 3.0], [2.3, 6.0, 10, 3.0], [2.5, 5.5, 10, 3.0],
        [1.5, 4.5, 20, 3.0], [8.8, 5.0, 20, 3.0], [8.9, 4.0, 20, 3.0], [9.5, 6.0, 20, 3.0],
        [10.5, 4.5, 20, 3.0], [10.5, 4.5, 10, 3.0]], dtype=np.float32)
    ms_y = np.array([0, 0, 0, 0, 0, 1, 1, 1, 1, 1], dtype=np.int32)
    rs_x = np.array([
        [0.1, 5.0, 10, 3.0], [0.2, 4.0, 10, 3.0], [0.3, 6.0, 10, 3.0],
        [10.8, 5.0, 20, 3.0], [10.9, 4.0, 20, 3.0], [11.0, 6.0, 20, 3.0]], dtype=np.float32)
    rs_y = np.array([0, 0, 0, 1, 1, 1], dtype=np.int32)
    dl_x = np.array([[i, i % 3] for i in range(11)] * 2, dtype=np.float32)
    dl_y = np.array([0] * 11 + [1] * 11, dtype=np.int32)
    return dict(ms_x=ms_x, ms_y=ms_y, rs_x=rs_x, rs_y=rs_y, dl_x=dl_x, dl_y=dl_y)


def small_datasets():
    from sklearn.datasets import make_classification
    out = {}
    rng = np.random.default_rng(7)
    for name, (n, p, ncls, seed) in {"a": (150, 40, 2, 0), "b": (120, 60, 3, 1),
                                     "c": (200, 100, 2, 2)}.items():
        X, y = make_classification(n_samples=n, n_features=p, n_informative=8, n_redundant=4,
                                   n_classes=ncls, n_clusters_per_class=1, random_state=seed)
        X[:, 0] = rng.integers(0, 4, n)      # discrete column
        X[:, 1] = 2.5                        # constant column
        out[name] = (X, y)
    return out


def main():
    from oracle import oracle as O
    fx = reference_fixtures()
    np.savez(os.path.join(HERE, "reference_fixtures.npz"), **fx)

    from sklearn.datasets import make_classification
    X, y = make_classification(n_samples=500, n_features=1000, n_informative=20,
                               n_redundant=100, random_state=42)
    cfg1 = {
        "source": "SURVEY.md §8c (reference MultiSURF, backend='cpu', run during the survey)",
        "X_sha256_prefix": hashlib.sha256(X.tobytes()).hexdigest()[:16],
        "y_sum": int(y.sum()),
        "top15": [7, 18, 83, 85, 261, 366, 477, 521, 599, 791, 806, 838, 863, 889, 927],
        "max_abs_score": 3.08e-2,
        "rel_gap_15_16": 0.031,
    }
    with open(os.path.join(HERE, "cfg1_reference.json"), "w") as f:
        json.dump(cfg1, f, indent=1)

    vec = {}
    for name, (X, y) in small_datasets().items():
        vec[f"{name}_X"] = X
        vec[f"{name}_y"] = y
        vec[f"{name}_multisurf"] = O.multisurf_scores(X, y)
        vec[f"{name}_multisurfstar"] = O.multisurf_scores(X, y, use_star=True)
        vec[f"{name}_surf"] = O.surf_scores(X, y)
        vec[f"{name}_surfstar"] = O.surf_scores(X, y, use_star=True)
        for k in (1, 3, 10):
            vec[f"{name}_relieff_k{k}"] = O.relieff_scores(X, y, n_neighbors=k)
    np.savez_compressed(os.path.join(HERE, "oracle_vectors.npz"), **vec)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
