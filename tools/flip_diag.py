"""Decision flips of the plan path against the oracle's decisions on a
data-family fixture (tests/golden/make_families.py), with the plan's trace:
    FS_TRACE=1 python tools/flip_diag.py lognormal_16k [q16|q32|default]
Prints the rows whose near hit / miss counts differ from the reference's,
the 16-bit decision risk, the scale-relative score error against the
oracle and the float64-sum fixture, and (stderr) the plan trace, which
includes how many rows took exact thresholds (exact_thresholds)."""
import importlib.util
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "lognormal_16k"
    mode = sys.argv[2] if len(sys.argv) > 2 else "default"
    backend = sys.argv[3] if len(sys.argv) > 3 else "gpu"
    if mode == "q16":
        os.environ["FS_Q16"] = "1"
    elif mode == "q32":
        os.environ["FS_Q16"] = "0"
    spec = importlib.util.spec_from_file_location("mk", os.path.join(GOLD, "make_families.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    from fastselect_amd import parallel
    X, y = mk.make(name)
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend=backend)
    job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend=backend, shard=False)
    try:
        s = job.step().cpu().numpy()
        counts = job.counts.cpu().numpy().reshape(-1, 2)
        cal = job.plan.calibration()
        guard = job.last_guard
    finally:
        job.close()
    fx = np.load(os.path.join(GOLD, f"family_{name}.npz"), allow_pickle=False)
    ref = fx["scores"]
    dpath = os.path.join(GOLD, f"family_{name}_decisions.npz")
    epath = os.path.join(GOLD, f"family_{name}_f64.npz")
    ref_counts = np.load(dpath, allow_pickle=False)["counts"] if os.path.exists(dpath) else counts
    ex = np.load(epath, allow_pickle=False)["scores"] if os.path.exists(epath) else ref
    bad = np.flatnonzero(np.any(counts != ref_counts, axis=1))
    print(json.dumps({
        "family": name, "mode": mode, "q16": bool(cal["q16"]), "guard": list(guard),
        "flipped_rows": bad[:20].tolist(), "n_flipped": int(bad.size),
        "count_diff": int(np.abs(counts - ref_counts).sum()),
        "have_decisions": os.path.exists(dpath),
        "err_vs_oracle": float(np.max(np.abs(s - ref)) / np.max(np.abs(ref))),
        "err_vs_f64": float(np.max(np.abs(s - ex)) / np.max(np.abs(ex))),
        "oracle_vs_f64": float(np.max(np.abs(ref - ex)) / np.max(np.abs(ex))),
        "top10_same": set(np.argsort(s)[::-1][:10].tolist()) == set(np.argsort(ref)[::-1][:10].tolist()),
    }), flush=True)


if __name__ == "__main__":
    main()
