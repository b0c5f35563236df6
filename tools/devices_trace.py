"""FS_TRACE phase log of a devices= MultiSURF fit: X
crosses the host link once (each device thread uploads its 1/N of the rows,
the rest arrives by peer copies) and the three exchanges are summed on the
devices.  Runs one configuration per child process (FS_TRACE is read once):

    python tools/devices_trace.py [n p] > log   (default: cfg4, 20000 x 20000)

Each child prints its [fs_trace] lines (stderr) and one JSON line with the
fit time and the scores' gap to devices=[0]."""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(n, p, devs):
    sys.path.insert(0, ROOT)
    from sklearn.datasets import make_classification
    import fastselect_amd as F
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=100,
                               random_state=42)
    X = X.astype(np.float32)
    t = time.perf_counter()
    s = F.MultiSURF(backend="gpu", devices=devs, n_features_to_select=10).fit(X, y).feature_importances_
    dt = time.perf_counter() - t
    out = os.path.join(ROOT, "gpurun_out", "devtrace_%s.npy" % "_".join(map(str, devs)))
    np.save(out, s)
    print(json.dumps({"devices": devs, "fit_s": dt}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(int(sys.argv[2]), int(sys.argv[3]), [int(d) for d in sys.argv[4].split(",")])
        sys.exit(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for devs in ("0", "0,0"):
        env = dict(os.environ, FS_TRACE="1")
        r = subprocess.run([sys.executable, __file__, "child", str(n), str(p), devs], env=env,
                           capture_output=True, text=True, timeout=900)
        print(f"== devices=[{devs}] rc={r.returncode}", flush=True)
        print(r.stderr.strip()[-6000:], flush=True)
        print(r.stdout.strip(), flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)
    a = np.load(os.path.join(ROOT, "gpurun_out", "devtrace_0.npy"))
    b = np.load(os.path.join(ROOT, "gpurun_out", "devtrace_0_0.npy"))
    print(json.dumps({"scale_rel_gap_[0,0]_vs_[0]": float(np.max(np.abs(a - b)) / np.max(np.abs(a))),
                      "top10_same": set(np.argsort(a)[::-1][:10]) == set(np.argsort(b)[::-1][:10])}))
