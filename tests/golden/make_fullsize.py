"""Generate the full-size parity fixtures in tests/golden/fullsize_*.npz.

Each fixture holds the C oracle's scores (oracle/relief_oracle.c, the
restatement of the reference backend='cpu') on one BASELINE.json
configuration, plus what a GPU test needs to be sure it regenerated the same
input on the GPU box (which has no /root/reference and runs no oracle at this
size):

    x_sha256   sha256 of the float32 (or float64 for SURF) X bytes
    y_sum      sum of the labels
    scores     float32 oracle scores (already / n, as the reference returns them)
    i_range    focal samples the oracle scored ([0, n) = the whole fit; a
               slice gives sum_{i in slice} row_i / n, the reference's column
               sum restricted to those rows)
    accum      'f32' (the reference's arithmetic) or 'f64' (*_f64 fixtures:
               the same diffs and decisions, every later sum in float64)

Inputs follow SURVEY.md §8d: make_classification(n, p, n_informative=20,
n_redundant=R, random_state=42), R = 50 for cfg3 and 100 otherwise; the
3-class cfg3 variant passes n_classes=3 (recorded in the fixture).

Run (container, ~45 min on 8 cores for everything):
    python tests/golden/make_fullsize.py [names...]
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# name: (algorithm, n, p, n_redundant, i_range or None, extra)
CONFIGS = {
    "cfg2_multisurf": ("multisurf", 5000, 5000, 100, None, {}),
    "cfg3_relieff_k10": ("relieff", 20000, 2000, 50, None, {"n_neighbors": 10}),
    "cfg5_surfstar_slice": ("surf", 10000, 50000, 100, (0, 384), {"use_star": True}),
    "cfg5_surf_slice": ("surf", 10000, 50000, 100, (4992, 5376), {"use_star": False}),
    "cfg5_multisurfstar": ("multisurf", 10000, 50000, 100, None, {"use_star": True}),
    "cfg4_multisurf": ("multisurf", 20000, 20000, 100, None, {}),
    # "add a 3-class cfg3 variant to exercise prior weights"
    "cfg3_relieff_k10_3class": ("relieff", 20000, 2000, 50, None,
                                {"n_neighbors": 10, "n_classes": 3}),
    # accum='f64': the oracle with every sum after the diffs in float64 (not
    # the reference; the "exact" side of tests/test_parity_attribution.py)
    "cfg2_multisurf_f64": ("multisurf", 5000, 5000, 100, None, {"accum": "f64"}),
    "cfg3_relieff_k10_f64": ("relieff", 20000, 2000, 50, None, {"n_neighbors": 10, "accum": "f64"}),
    "cfg5_surfstar_slice_f64": ("surf", 10000, 50000, 100, (0, 384),
                                {"use_star": True, "accum": "f64"}),
    "cfg5_surf_slice_f64": ("surf", 10000, 50000, 100, (4992, 5376),
                            {"use_star": False, "accum": "f64"}),
    "cfg4_multisurf_f64": ("multisurf", 20000, 20000, 100, None, {"accum": "f64"}),
    "cfg5_multisurfstar_f64": ("multisurf", 10000, 50000, 100, None,
                               {"use_star": True, "accum": "f64"}),
    "cfg3_relieff_k10_3class_f64": ("relieff", 20000, 2000, 50, None,
                                    {"n_neighbors": 10, "n_classes": 3, "accum": "f64"}),
    # round 6 (VERDICT r5 missing #2): whole-fit SURF / SURF* at cfg5, so that
    # k_surf_avg over all 10000 rows and the whole column sum are pinned, not
    # only the 384-sample slices (~1-2 h each on 6 threads)
    "cfg5_surf": ("surf", 10000, 50000, 100, None, {"use_star": False}),
    "cfg5_surfstar": ("surf", 10000, 50000, 100, None, {"use_star": True}),
}


def make_data(n, p, n_redundant, seed=42, n_classes=2):
    from sklearn.datasets import make_classification
    return make_classification(n_samples=n, n_features=p, n_informative=20,
                               n_redundant=n_redundant, n_classes=n_classes, random_state=seed)


def x_digest(x):
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def run(name, n_jobs):
    from oracle import oracle as O
    algo, n, p, red, i_range, extra = CONFIGS[name]
    extra = dict(extra)
    n_classes = extra.pop("n_classes", 2)
    t0 = time.time()
    X, y = make_data(n, p, red, n_classes=n_classes)
    if algo == "multisurf":
        x = X.astype(np.float32)
        s = O.multisurf_scores(x, y, i_range=i_range, n_jobs=n_jobs, **extra)
    elif algo == "relieff":
        x = X.astype(np.float32)   # the estimator's float32 cast (ReliefF.py:400) of float64 X
        s = O.relieff_scores(X, y, i_range=i_range, n_jobs=n_jobs, **extra)
    else:
        x = X                      # SURF validates to float64 (SURF.py:330-332)
        s = O.surf_scores(X, y, i_range=i_range, n_jobs=n_jobs, **extra)
    ir = np.array(i_range if i_range else (0, n), dtype=np.int64)
    out = os.path.join(HERE, f"fullsize_{name}.npz")
    np.savez(out, x_sha256=np.array(x_digest(x)), y_sum=np.array(int(np.asarray(y).sum())),
             scores=s.astype(np.float32), i_range=ir, n=np.array(n), p=np.array(p),
             n_redundant=np.array(red), algo=np.array(algo),
             use_star=np.array(bool(extra.get("use_star", False))),
             n_neighbors=np.array(int(extra.get("n_neighbors", 0))),
             accum=np.array(extra.get("accum", "f32")), n_classes=np.array(n_classes))
    print(f"{name}: {time.time() - t0:.0f} s -> {out}", flush=True)


def run_decisions(name, n_jobs):
    """fullsize_<name>_decisions.npz: the reference's near/far decisions alone
    at a full-size MultiSURF configuration (oracle_multisurf_decisions, pass 1
    only: thresholds mu - sigma/2 and every row's near hit / near miss
    counts, MultiSURF.py:174-217), so the GPU test can assert the default
    path's decisions row by row."""
    from oracle import oracle as O
    algo, n, p, red, _, extra = CONFIGS[name]
    assert algo == "multisurf"
    t0 = time.time()
    X, y = make_data(n, p, red, n_classes=extra.get("n_classes", 2))
    x = X.astype(np.float32)
    thr, counts = O.multisurf_decisions(x, y, n_jobs=n_jobs)
    out = os.path.join(HERE, f"fullsize_{name}_decisions.npz")
    np.savez_compressed(out, x_sha256=np.array(x_digest(x)),
                        y_sum=np.array(int(np.asarray(y).sum())), thr=thr,
                        counts=counts.astype(np.int32), n=np.array(n), p=np.array(p))
    print(f"{name} decisions: {time.time() - t0:.0f} s -> {out}", flush=True)


def main():
    args = sys.argv[1:]
    n_jobs = int(os.environ.get("ORACLE_THREADS", "-1"))
    if args and args[0] == "--decisions":
        for nm in args[1:] or ["cfg4_multisurf"]:
            run_decisions(nm, n_jobs)
        return
    names = args or list(CONFIGS)
    for nm in names:
        run(nm, n_jobs)


if __name__ == "__main__":
    main()
