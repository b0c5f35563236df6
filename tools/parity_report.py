"""Parity of the GPU path against every committed oracle fixture
(tests/golden/fullsize_*.npz, adversarial_*.npz, rowcoherent_*.npz), with the
figures SURVEY.md §8(d) asks for: the scale-relative error (the 1e-5 bar),
per-element relative error on the features with |s_ref| >= 1e-3 and 1e-2 of
max|s_ref|, and top-10 agreement.  Where a float64-accumulation fixture
(*_f64.npz: the oracle with every sum after the diffs in float64) exists,
the line after it attributes the error: |GPU - f64| against |oracle - f64|
(max and rms over all features, and the share of features where the GPU is
at least as close to the float64 sums as the oracle).  Run on the GPU box:

    python tools/parity_report.py > profiles/r03/parity_report.txt
"""
import glob
import hashlib
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLD = os.path.join(ROOT, "tests", "golden")

from parity_metrics import summary, topk_same  # noqa: E402


def attribution(gpu, ref, exact):
    gpu, ref, exact = (np.asarray(v, np.float64) for v in (gpu, ref, exact))
    scale = np.abs(exact).max()
    dg, do = np.abs(gpu - exact), np.abs(ref - exact)
    return (f"  vs f64 sums: GPU max {dg.max() / scale:.2e} rms {np.sqrt((dg ** 2).mean()) / scale:.2e}"
            f" | oracle(ref arithmetic) max {do.max() / scale:.2e} rms "
            f"{np.sqrt((do ** 2).mean()) / scale:.2e} | GPU at least as close on "
            f"{100 * (dg <= do).mean():.1f}% of features")


def gpu_scores(fx, X, y):
    import fastselect_amd as F
    from fastselect_amd import _lib
    n = int(fx["n"])
    lo, hi = (int(v) for v in fx["i_range"])
    star = bool(fx["use_star"])
    algo = str(fx["algo"])
    if algo == "multisurf" and (lo, hi) == (0, n):
        return F.MultiSURF(backend="gpu", use_star=star, n_features_to_select=10).fit(X, y) \
            .feature_importances_
    if algo == "relieff":
        return F.ReliefF(backend="gpu", n_neighbors=int(fx["n_neighbors"]),
                         n_features_to_select=10).fit(X, y).feature_importances_
    from fastselect_amd.SURF import surf_inputs
    x = np.ascontiguousarray(X, dtype=np.float64)
    isd, recip = surf_inputs(x, 10, "gpu")
    return (_lib.surf_score("gpu", x, np.asarray(y).astype(np.int32), recip, star, isd,
                            rows=(lo, hi)) / n).astype(np.float32)


def main():
    from sklearn.datasets import make_classification
    paths = sorted(p for p in glob.glob(os.path.join(GOLD, "fullsize_*.npz"))
                   if not p.endswith("_f64.npz"))
    for path in paths:
        fx = np.load(path, allow_pickle=False)
        n, p, red = int(fx["n"]), int(fx["p"]), int(fx["n_redundant"])
        ncls = int(fx["n_classes"]) if "n_classes" in fx else 2
        X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=red,
                                   n_classes=ncls, random_state=42)
        lo, hi = (int(v) for v in fx["i_range"])
        ref = fx["scores"]
        f64 = path[:-4] + "_f64.npz"
        exact = np.load(f64, allow_pickle=False)["scores"] if os.path.exists(f64) else None
        variants = [("default", {})]
        if str(fx["algo"]) == "surf":  # the whole-fit (dense) pass 2 beside the sparse slice path
            variants.append(("dense", {"sparse": 0}))
        if str(fx["algo"]) == "multisurf" and n >= 16384:  # 32-bit pass 1 beside the 16-bit default
            variants.append(("q32", {"q16": 0}))
        from fastselect_amd import _lib
        for label, hooks in variants:
            try:
                with _lib.test_hooks(**hooks):
                    s = gpu_scores(fx, X, y)
            finally:
                _lib.set_test_hook("reset")
            print(f"{os.path.basename(path):36s} {label:11s} n={n:6d} p={p:6d} rows=[{lo},{hi}) "
                  f"{summary(s, ref)} top-10 same: {topk_same(s, ref, 10)}", flush=True)
            if exact is not None:
                print(attribution(s, ref, exact), flush=True)
    for pattern, modname in (("adversarial_*.npz", "make_adversarial.py"),
                             ("rowcoherent_*.npz", "make_rowcoherent.py")):
        gen = os.path.join(GOLD, modname)
        if not os.path.exists(gen):
            continue
        spec = importlib.util.spec_from_file_location("mk_" + modname[:-3], gen)
        mk = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mk)
        prefix = pattern.split("*")[0]
        for path in sorted(glob.glob(os.path.join(GOLD, pattern))):
            import fastselect_amd as F
            name = os.path.basename(path)[len(prefix):-4]
            fx = np.load(path, allow_pickle=False)
            X, y = mk.make(name)
            assert hashlib.sha256(X.tobytes()).hexdigest() == str(fx["x_sha256"])
            for star, key in ((False, "scores"), (True, "scores_star")):
                est = F.MultiSURF(backend="gpu", use_star=star, n_features_to_select=1).fit(X, y)
                print(f"{prefix[:-1]} {name:16s} star={int(star)} n={X.shape[0]:6d} "
                      f"p={X.shape[1]:6d} {summary(est.feature_importances_, fx[key])}", flush=True)


if __name__ == "__main__":
    main()
