"""Reference-order MultiSURF on 16-bit pass-1 operands (the ref_q16 test
hook) against 32-bit ones, at a BASELINE config: step time and kernel split,
decisions against the oracle's (tests/golden/fullsize_<cfg>_decisions.npz)
and scores against the oracle's bit for bit (a whole fit per mode).

    FS_TRACE=1 python tools/ref_q16_probe.py [--name cfg4_multisurf] [--steps 3]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="cfg4_multisurf")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--modes", default="0,1")
    a = ap.parse_args()
    import torch

    import fastselect_amd as F
    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    from test_gpu_baseline import GOLD, _fixture, _inputs
    fx = _fixture(a.name)
    X, y = _inputs(fx)
    dec = np.load(os.path.join(GOLD, f"fullsize_{a.name}_decisions.npz"), allow_pickle=False)
    ref_counts = dec["counts"].astype(np.int64).reshape(-1, 2)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    for mode in (int(m) for m in a.modes.split(",")):
        _lib.set_test_hook("ref_q16", mode)
        try:
            job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False,
                                   accumulation="reference")
            job.step()
            got = job.counts.cpu().numpy().reshape(-1, 2).astype(np.int64)
            flipped = int(np.sum(np.any(got != ref_counts, axis=1)))
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.steps):
                job.step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / a.steps * 1e3
            k1, k2 = job.kernel_ms(0), job.kernel_ms(1)
            job.close()
            print(f"ref_q16={mode}: {ms:.2f} ms/step (pass 1 {k1:.2f}, chains {k2:.2f} ms), "
                  f"flipped rows {flipped}", flush=True)
            est = F.MultiSURF(backend="gpu", accumulation="reference",
                              n_features_to_select=10).fit(X, y)
            s = np.asarray(est.feature_importances_)
            diff = int(np.sum(s != fx["scores"]))
            print(f"ref_q16={mode}: whole fit {diff} of {s.size} scores differ from the oracle",
                  flush=True)
        finally:
            _lib.set_test_hook("reset", 0)


if __name__ == "__main__":
    main()
