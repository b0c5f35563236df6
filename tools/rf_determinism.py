"""ReliefF determinism probe: the same one-shot call repeated must give
bit-identical scores; run under several switches (and with FS_TRACE's
refined-pair / tie-row counts) to locate a source of run-to-run variation.

    python tools/rf_determinism.py
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os
import sys
import numpy as np
sys.path.insert(0, {root!r})
from sklearn.datasets import make_classification
from fastselect_amd import _lib
from fastselect_amd.ReliefF import relieff_inputs
X, y = make_classification(n_samples=700, n_features=300, n_informative=10, n_classes=3,
                           random_state=8)
X[:, 4] = np.round(X[:, 4])
out = []
for act in (np.arange(300), np.array([0, 4, 63, 78, 95, 111, 166, 172, 243, 248]),
            np.array([0, 63, 78, 95, 111, 166, 172, 243, 248, 261])):
    Xs = np.ascontiguousarray(X[:, act])
    _lib.set_test_hook("ksplit", int(os.environ.get("RF_DET_KSPLIT", "0")))
    _lib.set_test_hook("q16", int(os.environ.get("RF_DET_Q16", "-1")))
    x, ye, recip, isd, pri = relieff_inputs(Xs, y, 6, "gpu")
    res = {{tuple(_lib.relieff_score("gpu", x, ye, recip, isd, 6, pri).tolist()) for r in range(12)}}
    out.append(len(res))
print("distinct results in 12 (full, 10 with the discrete column, 10 continuous):", out)
"""


def main():
    for label, env in (("default", {}), ("ksplit=1", {"RF_DET_KSPLIT": "1"}),
                       ("q16=1", {"RF_DET_Q16": "1"}), ("trace", {"FS_TRACE": "1"})):
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=e,
                           capture_output=True, text=True, timeout=300)
        print(label, r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-1500:],
              flush=True)
        if label == "trace":
            lines = [l for l in r.stderr.splitlines() if "relieff:" in l]
            print("  trace lines (distinct):", sorted(set(lines))[:12], flush=True)


if __name__ == "__main__":
    main()
