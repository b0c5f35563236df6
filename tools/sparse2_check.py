"""Quick GPU check of the sparse pass-2 variants against the oracle (small
shapes covering: 512-feature blocks, the 256-feature tail, a tail longer than
256 features (one more, partial, 512-feature block), p = 64 (a single
partial block), discrete / mixed blocks, n not a multiple of 128).  Each
configuration runs with FS_SPARSE_V=1 (round-2 streams) and 2 (half tiles x 8
features), the latter with the generated loop and with the plain-HIP walk
(FS_SPARSE_ASM=0); one subprocess per variant because the library reads the
switches once.

    python tools/sparse2_check.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [  # (n, p, discrete columns, seed)
    (1024, 64, 0, 1), (700, 600, 0, 2), (1500, 1100, 0, 3), (900, 520, 40, 4), (640, 300, 300, 5),
    (2100, 2048, 0, 6), (900, 800, 0, 7), (600, 1400, 30, 8),
]

CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, {root!r})
from sklearn.datasets import make_classification
import fastselect_amd as F
from oracle import oracle as O
out = []
for n, p, nd, seed in {cases!r}:
    X, y = make_classification(n_samples=n, n_features=p, n_informative=min(10, p // 2),
                               n_redundant=min(20, p // 4), random_state=seed)
    if nd:
        X[:, :nd] = np.round(X[:, :nd])
    for star in (False,):
        s = F.MultiSURF(backend="gpu", use_star=star).fit(X, y).feature_importances_
        r = O.multisurf_scores(X, y, use_star=star)
        out.append([n, p, nd, float(np.abs(s - r).max() / np.abs(r).max())])
print(json.dumps(out))
"""


def main():
    res = {}
    for label, env in (("v1", {"FS_SPARSE_V": "1"}), ("v2", {"FS_SPARSE_V": "2"}),
                       ("v2-hip", {"FS_SPARSE_V": "2", "FS_SPARSE_ASM": "0"})):
        e = dict(os.environ, **env)
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, cases=CASES)], env=e,
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(label, "FAILED rc", r.returncode, r.stderr[-2000:], flush=True)
            sys.exit(1)
        res[label] = json.loads(r.stdout.strip().splitlines()[-1])
        print(label, res[label], flush=True)
    bad = [(k, c) for k, v in res.items() for c in v if c[3] > 1e-5]
    print("ALL OK" if not bad else f"OVER 1e-5: {bad}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
