"""MultiSURF / ReliefF scores with 16-bit (q16 test hook 1) vs 32-bit (0)
pass-1 operands on the BASELINE configs: scale-relative difference and top-k
agreement (the 32-bit path is the one pinned to the oracle at ~1e-7).

    python tools/q16_compare.py [--only cfg2,cfg4]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from sklearn.datasets import make_classification  # noqa: E402

CFG = {
    "cfg2": ("ms", 5000, 5000, 100, False),
    "cfg2s": ("ms", 5000, 5000, 100, True),
    "n8k": ("ms", 8192, 4096, 100, False),
    "cfg4": ("ms", 20000, 20000, 100, False),
    "cfg4s": ("ms", 20000, 20000, 100, True),
    "cfg5m": ("ms", 10000, 50000, 100, True),
    "cfg3": ("rf", 20000, 2000, 50, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=",".join(CFG))
    a = ap.parse_args()
    from fastselect_amd import MultiSURF, ReliefF, _lib
    for name in a.only.split(","):
        algo, n, p, R, star = CFG[name]
        X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=R,
                                   random_state=42)
        X = X.astype(np.float32)
        s = {}
        for flag in ("0", "1"):
            _lib.set_test_hook("q16", int(flag))
            if algo == "ms":
                est = MultiSURF(backend="gpu", use_star=star, n_features_to_select=10)
            else:
                est = ReliefF(backend="gpu", n_neighbors=10, n_features_to_select=10)
            s[flag] = est.fit(X, y).feature_importances_.astype(np.float64)
        d = np.abs(s["1"] - s["0"]).max() / np.abs(s["0"]).max()
        top = set(np.argsort(s["0"])[::-1][:10]) == set(np.argsort(s["1"])[::-1][:10])
        print(json.dumps({"config": name, "scale_rel_diff": d, "top10_equal": bool(top),
                          "max_abs_score": float(np.abs(s["0"]).max())}), flush=True)


if __name__ == "__main__":
    main()
