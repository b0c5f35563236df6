"""Localise the 16-bit vs 32-bit pass-1 difference on a row-coherent fixture:
per-focal-slice score sums of both (diagnostic)."""
import os
import subprocess
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests/golden")
name = sys.argv[1] if len(sys.argv) > 1 else "minrow4_16k"
mode = sys.argv[2] if len(sys.argv) > 2 else "parent"
if mode == "parent":
    outs = {}
    for q in ("1", "0"):
        env = dict(os.environ, FS_Q16=q)
        subprocess.run([sys.executable, __file__, name, "child" + q], env=env, check=True)
    a = np.load("gpurun_out/probe2_child1.npy"); b = np.load("gpurun_out/probe2_child0.npy")
    scale = np.abs(b.sum(0)).max()
    d = np.abs(a - b).max(1) / scale
    print("slice max |q16 - q32| / max|total|:")
    for k, v in enumerate(d):
        print(k, f"{v:.3e}")
    sys.exit(0)
import make_rowcoherent as mk
from fastselect_amd import _lib
from fastselect_amd.parallel import prepare_inputs
X, y = mk.make(name)
x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
n = x.shape[0]
W = 512
parts = [_lib.multisurf_score("gpu", x, yv, recip, None, False, isd, rows=(k, min(n, k + W)))
         for k in range(0, n, W)]
np.save(f"gpurun_out/probe2_{mode}.npy", np.array(parts))
