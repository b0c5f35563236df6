"""Diagnostic (GPU): scale-relative error of MultiSURF on a data-family
fixture (tests/golden/make_families.py) under operand / correction variants.
Each variant runs in a child process (the env knobs are read once)."""
import importlib.util
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def child(name, star):
    sys.path.insert(0, ROOT)
    spec = importlib.util.spec_from_file_location("mk", os.path.join(GOLD, "make_families.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    import fastselect_amd as F
    fx = np.load(os.path.join(GOLD, f"family_{name}.npz"), allow_pickle=False)
    X, y = mk.make(name)
    s = F.MultiSURF(backend="gpu", use_star=star, n_features_to_select=10).fit(X, y).feature_importances_
    ref = fx["scores_star" if star else "scores"]
    err = float(np.max(np.abs(s - ref)) / np.max(np.abs(ref)))
    top = set(np.argsort(s)[::-1][:10]) == set(np.argsort(ref)[::-1][:10])
    from fastselect_amd import _lib
    risk, rerun = _lib.multisurf_last_guard()
    out = {"err": err, "top10": top, "maxref": float(np.max(np.abs(ref))), "risk": risk, "rerun": rerun}
    f64 = os.path.join(GOLD, f"family_{name}_f64.npz")
    if not star and os.path.exists(f64):
        e = np.load(f64, allow_pickle=False)["scores"]
        sc = float(np.max(np.abs(e)))
        out["gpu_vs_f64"] = float(np.max(np.abs(s - e)) / sc)
        out["oracle_vs_f64"] = float(np.max(np.abs(ref - e)) / sc)
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(sys.argv[2], sys.argv[3] == "1")
        sys.exit(0)
    names = os.environ.get("FAM", "uniform_16k").split(",")
    variants = [("default", {}), ("q32", {"FS_Q16": "0"}), ("q16", {"FS_Q16": "1"})]
    for name in names:
        for star in ("0", "1"):
            for lab, env in variants:
                e = dict(os.environ, **env)
                r = subprocess.run([sys.executable, __file__, "child", name, star], env=e,
                                   capture_output=True, text=True, timeout=240)
                print(name, "star" if star == "1" else "ms", lab,
                      r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:], flush=True)
