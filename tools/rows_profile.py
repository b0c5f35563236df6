"""One rank's share of row-sharded ReliefF (cfg3) and SURF* (cfg5) on one
MI355X: wall time of fs_*_score_rows for rank 0 of world N (whole-block
slices, the slowest rank up to one 128-sample block), N = 1, 2, 4, 8.

    python tools/rows_profile.py [--surf-n 10000 --surf-p 50000]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
from sklearn.datasets import make_classification  # noqa: E402

from fastselect_amd import _lib  # noqa: E402
from fastselect_amd.parallel import shard_rows  # noqa: E402
from fastselect_amd.ReliefF import relieff_inputs  # noqa: E402
from fastselect_amd.SURF import surf_inputs  # noqa: E402


def timed(fn, reps=3):
    fn()
    best = 1e30
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t)
    return best * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--surf-n", type=int, default=10000)
    ap.add_argument("--surf-p", type=int, default=50000)
    a = ap.parse_args()
    out = {}
    X, y = make_classification(n_samples=20000, n_features=2000, n_informative=20,
                               n_redundant=50, random_state=42)
    n = X.shape[0]
    x32, ye, recip, isd, pr = relieff_inputs(X, y, 10, "gpu")
    for w in (1, 2, 4, 8):
        ms = timed(lambda: _lib.relieff_score("gpu", x32, ye, recip, isd, 10, pr,
                                              rows=shard_rows(n, 0, w)))
        out[f"relieff_cfg3_world{w}_rank0_ms"] = round(ms, 2)
        print(f"ReliefF cfg3 world {w}: rank 0 {ms:.1f} ms", flush=True)
    X, y = make_classification(n_samples=a.surf_n, n_features=a.surf_p, n_informative=20,
                               n_redundant=100, random_state=42)
    n = X.shape[0]
    isd, recip = surf_inputs(X, 10, "gpu")
    yi = y.astype(np.int32)
    for w in (1, 2, 4, 8):
        ms = timed(lambda: _lib.surf_score("gpu", X, yi, recip, True, isd,
                                           rows=shard_rows(n, 0, w)), reps=2)
        out[f"surfstar_{a.surf_n}x{a.surf_p}_world{w}_rank0_ms"] = round(ms, 2)
        print(f"SURF* world {w}: rank 0 {ms:.1f} ms", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
