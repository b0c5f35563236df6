"""Resident ReliefF plan (fs_plan_set_features + fs_plan_score) against the
one-shot call on the same feature subsets, repeated and alternated, to find
state that leaks from one score into the next.

    python tools/resident_determinism.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from sklearn.datasets import make_classification
    from fastselect_amd import _lib
    from fastselect_amd.ReliefF import relieff_inputs
    X, y = make_classification(n_samples=700, n_features=300, n_informative=10, n_classes=3,
                               random_state=8)
    X[:, 4] = np.round(X[:, 4])
    x, ye, recip, isd, pri = relieff_inputs(X, y, 6, "gpu")
    plan = _lib.RowsPlan("gpu", "relieff", x, ye, recip, isd, k=6, class_probs=pri)
    subsets = [np.arange(300), np.arange(0, 300, 2), np.arange(1, 300, 3), np.arange(0, 300, 2),
               np.arange(300), np.arange(1, 300, 3)]
    for rep in range(2):
        for k, act in enumerate(subsets):
            plan.set_features(act)
            sums = torch.zeros(act.size, dtype=torch.float64, device="cuda")
            plan.score(sums.data_ptr())
            torch.cuda.synchronize()
            a = sums.cpu().numpy()
            one = _lib.relieff_score("gpu", x, ye, recip, isd, 6, pri, feat_idx=act) \
                if "feat_idx" in _lib.relieff_score.__code__.co_varnames else None
            xs, ye2, rc2, isd2, pri2 = relieff_inputs(np.ascontiguousarray(X[:, act]), y, 6, "gpu")
            b = _lib.relieff_score("gpu", xs, ye2, rc2, isd2, 6, pri2).astype(np.float64)
            a32 = (a / 700).astype(np.float32).astype(np.float64)
            print(f"rep {rep} subset {k} ({act.size}): max |resident - one-shot| "
                  f"{np.abs(a32 - b).max():.3e} (scale {np.abs(b).max():.3e})", flush=True)
    plan.close()


if __name__ == "__main__":
    main()
