"""Large-n route of the column sort (fs_colsort.hip) against the CPU
backend's exact correction: per-row corrections of a GPU plan and a CPU plan
on the same lognormal data, LDS route or (third argument "global") the
large-n route forced by the colsort_global test hook.
Run on the GPU box:  python tools/colsort_debug.py [n p [global]]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_meancorr import lognormal  # noqa: E402

from fastselect_amd import _lib, parallel  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
p = int(sys.argv[2]) if len(sys.argv) > 2 else 64
glob_route = len(sys.argv) > 3 and sys.argv[3] == "global"
if glob_route:
    _lib.set_test_hook("colsort_global", 1)
X, y = lognormal(n, p, seed=7)
out = {}
for be in ("cpu", "gpu"):
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend=be)
    job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend=be, shard=False)
    job.step()
    rs = job.rowstats.cpu().numpy().reshape(-1, 3)
    out[be] = (rs, job.plan.calibration())
    job.close()
(rc, cc), (rg, cg) = out["cpu"], out["gpu"]
print("route", "global" if glob_route else "auto",
      "n", n, "p", p, "q16 gpu", cg["q16"], "SC cpu/gpu", cc["SC"], cg["SC"])
print("corr cpu", rc[:4, 2], "gpu", rg[:4, 2])
print("s1 cpu", rc[:4, 0], "gpu", rg[:4, 0])
if cc["SC"] == cg["SC"]:
    print("max |corr diff| / s1", np.max(np.abs(rc[:, 2] - rg[:, 2]) / rc[:, 0]))
