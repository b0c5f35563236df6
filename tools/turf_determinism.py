"""TuRF over a resident ReliefF plan vs refits: repeat both, log every
refit's active set and scores, and report where two runs first differ
(tests/test_gpu.py::test_turf_resident_rows_gpu_equals_refits).

    python tools/turf_determinism.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from sklearn.datasets import make_classification
    import fastselect_amd as fa
    from fastselect_amd import _resident

    log = []
    orig = _resident.ResidentRows.refit

    def refit(self, active):
        est = orig(self, active)
        log.append((np.asarray(active).copy(), est.feature_importances_.copy()))
        return est

    _resident.ResidentRows.refit = refit

    class Refit(fa.ReliefF):
        _resident_scorer = None

    X, y = make_classification(n_samples=700, n_features=300, n_informative=10, n_classes=3,
                               random_state=8)
    X[:, 4] = np.round(X[:, 4])
    kw = dict(n_features_to_select=10, pct_remove=0.3)
    runs = []
    for r in range(6):
        log.clear()
        f = fa.TuRF(fa.ReliefF(backend="gpu", n_neighbors=6), **kw).fit(X, y)
        runs.append((f.top_features_.tolist(), list(log)))
    s = fa.TuRF(Refit(backend="gpu", n_neighbors=6), **kw).fit(X, y)
    print("refit top:", s.top_features_.tolist(), flush=True)
    base = runs[0][1]
    for r, (top, lg) in enumerate(runs):
        first = None
        for it, ((a0, s0), (a1, s1)) in enumerate(zip(base, lg)):
            if not np.array_equal(a0, a1) or not np.array_equal(s0, s1):
                first = (it, np.array_equal(a0, a1), float(np.abs(s0 - s1).max()) if s0.shape == s1.shape else None,
                         int((s0 != s1).sum()) if s0.shape == s1.shape else None)
                break
        print(f"run {r}: top {top}; iterations {len(lg)}; first difference vs run 0: {first}",
              flush=True)
    # replay run 0's active sets on fresh resident scorers and one-shot calls
    from fastselect_amd import _lib
    from fastselect_amd.ReliefF import relieff_inputs
    for it, (act, sc) in enumerate(base):
        xs, ye, rc, isd, pri = relieff_inputs(np.ascontiguousarray(X[:, act]), y, 6, "gpu")
        b = (_lib.relieff_score("gpu", xs, ye, rc, isd, 6, pri)).astype(np.float32)
        print(f"iter {it}: {act.size} features, max |resident - one-shot| {np.abs(sc - b).max():.3e}, "
              f"differing {(sc != b).sum()}", flush=True)


if __name__ == "__main__":
    main()


def replay():
    """Repeat the late TuRF subsets: one-shot calls and a resident plan."""
    import torch
    from sklearn.datasets import make_classification
    from fastselect_amd import _lib
    from fastselect_amd.ReliefF import relieff_inputs
    X, y = make_classification(n_samples=700, n_features=300, n_informative=10, n_classes=3,
                               random_state=8)
    X[:, 4] = np.round(X[:, 4])
    rng = np.random.default_rng(3)
    sets = [np.sort(rng.choice(300, size=k, replace=False)) for k in (26, 19, 14, 10, 10, 19)]
    sets[4] = np.array([0, 4, 63, 78, 95, 111, 166, 172, 243, 248])
    for act in sets:
        xs, ye, rc, isd, pri = relieff_inputs(np.ascontiguousarray(X[:, act]), y, 6, "gpu")
        outs = {tuple(_lib.relieff_score("gpu", xs, ye, rc, isd, 6, pri).tolist()) for _ in range(10)}
        print(f"one-shot {act.size} features: {len(outs)} distinct results in 10", flush=True)
    x, ye, rc, isd, pri = relieff_inputs(X, y, 6, "gpu")
    plan = _lib.RowsPlan("gpu", "relieff", x, ye, rc, isd, k=6, class_probs=pri)
    res = {}
    for rep in range(5):
        for k, act in enumerate(sets):
            plan.set_features(act)
            buf = torch.empty(act.size, dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            plan.score(buf.data_ptr())
            torch.cuda.synchronize()
            res.setdefault(k, set()).add(tuple(buf.cpu().numpy().tolist()))
    print("resident distinct results per subset:", {k: len(v) for k, v in res.items()}, flush=True)
    plan.close()


if __name__ == "__main__" and os.environ.get("REPLAY"):
    replay()
