"""Scale-relative error and top-k agreement of the GPU path against every
committed oracle fixture (tests/golden/fullsize_*.npz, adversarial_*.npz).
Prints one line per case; run on the GPU box:

    python tools/parity_report.py > profiles/r02/parity_report.txt
"""
import glob
import hashlib
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")


def rel(a, r):
    a, r = np.asarray(a, np.float64), np.asarray(r, np.float64)
    return float(np.abs(a - r).max() / np.abs(r).max())


def topk(s, k=10):
    return set(np.argsort(np.asarray(s))[::-1][:k].tolist())


def main():
    import fastselect_amd as F
    from fastselect_amd import _lib
    from sklearn.datasets import make_classification
    for path in sorted(glob.glob(os.path.join(GOLD, "fullsize_*.npz"))):
        fx = np.load(path, allow_pickle=False)
        n, p, red, algo = int(fx["n"]), int(fx["p"]), int(fx["n_redundant"]), str(fx["algo"])
        X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=red,
                                   random_state=42)
        lo, hi = (int(v) for v in fx["i_range"])
        star = bool(fx["use_star"])
        if algo == "multisurf" and (lo, hi) == (0, n):
            s = F.MultiSURF(backend="gpu", use_star=star, n_features_to_select=10).fit(X, y)
            s = s.feature_importances_
        elif algo == "relieff":
            s = F.ReliefF(backend="gpu", n_neighbors=int(fx["n_neighbors"]),
                          n_features_to_select=10).fit(X, y).feature_importances_
        else:
            from fastselect_amd.SURF import surf_inputs
            x = np.ascontiguousarray(X, dtype=np.float64)
            isd, recip = surf_inputs(x, 10, "gpu")
            s = (_lib.surf_score("gpu", x, np.asarray(y).astype(np.int32), recip, star, isd,
                                 rows=(lo, hi)) / n).astype(np.float32)
        ref = fx["scores"]
        print(f"{os.path.basename(path):40s} n={n:6d} p={p:6d} rows=[{lo},{hi}) "
              f"scale-rel {rel(s, ref):.2e}  top-10 same: {topk(s) == topk(ref)}", flush=True)
    spec = importlib.util.spec_from_file_location("mk", os.path.join(GOLD, "make_adversarial.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    for path in sorted(glob.glob(os.path.join(GOLD, "adversarial_*.npz"))):
        name = os.path.basename(path)[len("adversarial_"):-4]
        fx = np.load(path, allow_pickle=False)
        X, y = mk.make(name)
        assert hashlib.sha256(X.tobytes()).hexdigest() == str(fx["x_sha256"])
        for star, key in ((False, "scores"), (True, "scores_star")):
            est = F.MultiSURF(backend="gpu", use_star=star, n_features_to_select=1).fit(X, y)
            print(f"adversarial {name:16s} star={int(star)} n={X.shape[0]:6d} p={X.shape[1]:6d} "
                  f"scale-rel {rel(est.feature_importances_, fx[key]):.2e}", flush=True)


if __name__ == "__main__":
    main()
