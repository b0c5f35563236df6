"""Probe the row-coherent fixture failures on the GPU (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "tests/golden")
import make_rowcoherent as mk
from fastselect_amd import _lib
from fastselect_amd.parallel import prepare_inputs, ShardedMultiSURF
from oracle import oracle as O
from parity_metrics import scale_rel_err

name = sys.argv[1] if len(sys.argv) > 1 else "minrow4_16k"
X, y = mk.make(name)
fx = np.load(f"tests/golden/rowcoherent_{name}.npz")
x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
n = x.shape[0]
job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False)
s = job.step().cpu().numpy()
print("calibration", job.plan.calibration(), "info", job.info())
print("whole fit scale-rel", scale_rel_err(s, fx["scores"]))
rng = np.random.default_rng(1000 + mk.CASES[name])
pick = np.sort(rng.choice(np.arange(2, n), size=mk.CASES[name], replace=False))
tot_g = np.zeros(x.shape[1]); tot_o = np.zeros(x.shape[1])
for r in pick[:6]:
    g = _lib.multisurf_score("gpu", x, yv, recip, None, False, isd, rows=(int(r), int(r) + 1)) / n
    o = O.multisurf_scores(X, y, i_range=(int(r), int(r) + 1)).astype(np.float64)
    print(f"row {r}: |gpu-oracle| max {np.abs(g - o).max():.3e}  |oracle| max {np.abs(o).max():.3e}")
# a normal row
for r in (0, 1, 5, 100):
    g = _lib.multisurf_score("gpu", x, yv, recip, None, False, isd, rows=(r, r + 1)) / n
    o = O.multisurf_scores(X, y, i_range=(r, r + 1)).astype(np.float64)
    print(f"normal row {r}: |gpu-oracle| max {np.abs(g - o).max():.3e}  |oracle| max {np.abs(o).max():.3e}")
job.close()
