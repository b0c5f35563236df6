"""16-bit vs 32-bit pass-1 operands for MultiSURF now that the row means are
exact (fs_colsort.hip): per configuration, the rows whose near hit / miss
counts differ between the two (decision flips; the 32-bit decisions are the
reference's, tests/test_gpu_meancorr.py), the scale-relative score gap, the
16-bit decision risk the plan's guard would estimate (fs_plan.hip
q16_decision_risk, restated), and for cfg2 the gap to the oracle fixture.

    python tools/q16_parity.py [cfg2 n8k cfg4 ...]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG = {
    "cfg2": (5000, 5000, 100),
    "n3k": (3000, 2000, 100),
    "n8k": (8192, 4096, 100),
    "n12k": (12000, 8000, 100),
    "cfg4": (20000, 20000, 100),
}


def risk(rs, cnt, sums, n, pc, sc, nfeat):
    rs = rs.reshape(-1, 3)
    cnt = cnt.reshape(-1, 2)
    smax = np.max(np.abs((sums / n).astype(np.float32)))
    thr_err = np.sqrt(pc / 6.0 + 1.0) / np.sqrt(n)
    mu_sum = np.sum((rs[:, 0] - rs[:, 2]) / (n - 1))
    dbar = 2.0 * mu_sum / n / (sc * nfeat)
    mu = rs[:, 0] / (n - 1)
    var = rs[:, 1] / (n - 1) - mu * mu
    ok = var > 0
    flips = n * 0.352 * thr_err / np.sqrt(var[ok])
    m = np.maximum(1.0, np.minimum(cnt[ok, 0], cnt[ok, 1]))
    eff = dbar / (n * m)
    return float(np.sqrt(np.sum(flips * eff * eff)) / smax)


def main():
    from sklearn.datasets import make_classification

    from fastselect_amd import parallel
    names = sys.argv[1:] or ["cfg2", "n8k"]
    for name in names:
        n, p, R = CFG[name]
        X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=R,
                                   random_state=42)
        X = X.astype(np.float32)
        out = {}
        for flag in ("0", "1"):
            os.environ["FS_Q16"] = flag
            x, yv, recip, isd = parallel.prepare_inputs(X, y, backend="gpu")
            job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False)
            s = job.step().cpu().numpy()
            cal = job.plan.calibration()
            out[flag] = (s, job.counts.cpu().numpy().copy(), job.rowstats.cpu().numpy().copy(),
                         job.scores.cpu().numpy().copy(), cal)
            job.close()
        del os.environ["FS_Q16"]
        s0, c0, _, _, cal0 = out["0"]
        s1, c1, rs1, sums1, cal1 = out["1"]
        flips = int(np.sum(np.any(c0.reshape(-1, 2) != c1.reshape(-1, 2), axis=1)))
        scale = np.max(np.abs(s0))
        line = {"config": name, "n": n, "p": p, "q16_used": cal1["q16"],
                "rows_flipped_vs_32bit": flips,
                "count_diff_total": int(np.abs(c0 - c1).sum()),
                "scale_rel_gap_vs_32bit": float(np.max(np.abs(s1 - s0)) / scale),
                "risk_estimate": risk(rs1, c1, sums1, n, p, cal1["SC"], p),
                "top10_same": set(np.argsort(s0)[::-1][:10]) == set(np.argsort(s1)[::-1][:10])}
        if name == "cfg2":
            ref = np.load(os.path.join(ROOT, "tests", "golden", "fullsize_cfg2_multisurf.npz"))["scores"]
            ex = np.load(os.path.join(ROOT, "tests", "golden", "fullsize_cfg2_multisurf_f64.npz"))["scores"]
            line["q16_vs_oracle"] = float(np.max(np.abs(s1 - ref)) / np.max(np.abs(ref)))
            line["q32_vs_oracle"] = float(np.max(np.abs(s0 - ref)) / np.max(np.abs(ref)))
            line["q16_vs_f64"] = float(np.max(np.abs(s1 - ex)) / np.max(np.abs(ex)))
            line["q32_vs_f64"] = float(np.max(np.abs(s0 - ex)) / np.max(np.abs(ex)))
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
