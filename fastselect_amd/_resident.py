"""Device-resident re-scoring of column subsets for ReliefF and SURF (the
TuRF caller, TuRF.py:93-115): X is uploaded once into a ReliefF / SURF plan
(``fs_plan_create_relieff`` / ``_surf``) and every ``refit(active)`` re-targets
it with ``fs_plan_set_features`` instead of refitting on ``X[:, active]``.
Per-column preprocessing (discreteness, ranges) does not depend on the other
columns, so the subset's inputs are the full ones restricted to ``active``.
"""
from __future__ import annotations

import numpy as np

from . import _base, _lib


class ResidentRows:
    """``refit(active)`` leaves ``est`` exactly as ``est.fit(X[:, active], y)``
    would (fitted attributes included), scoring on the resident plan."""

    def __init__(self, est, name: str, plan: _lib.RowsPlan, n: int, is_discrete, backend: str,
                 before_score=None):
        self.est = est
        self.name = name
        self.plan = plan
        self.n = n
        self.is_discrete = is_discrete
        self.backend = backend
        self.before_score = before_score
        self.active = None
        self._buf = None

    def _sums(self, n_kept: int) -> np.ndarray:
        if self.backend == "gpu":
            import torch
            if self._buf is None or self._buf.numel() != n_kept:
                # no fill kernel: the plan clears the sums on its own stream.
                # That stream is non-blocking, so nothing torch queued on its
                # stream is ordered before the plan's kernels -- a torch.zeros
                # here could land after the plan's k_reduce and wipe the
                # sums (TuRF over ReliefF varied run to run that way)
                self._buf = torch.empty(n_kept, dtype=torch.float64, device="cuda")
            torch.cuda.current_stream().synchronize()
            self.plan.score(self._buf.data_ptr())  # synchronises the plan's stream
            return self._buf.cpu().numpy()
        out = np.zeros(n_kept, dtype=np.float64)
        self.plan.score(out.ctypes.data)
        return out

    def refit(self, active):
        est = self.est
        active = np.asarray(active, dtype=np.int64)
        n_select = est._validate_parameters(self.n, active.size)
        est.n_features_in_ = active.size
        if self.before_score is not None:
            self.before_score()
        if est.verbose:
            print(f"Running {self.name} on the {self.backend.upper()} now...")
        if self.active is None or not np.array_equal(active, self.active):
            self.plan.set_features(active)
            self.active = active
        scores = (self._sums(active.size) / self.n).astype(np.float32)
        est.is_discrete_ = self.is_discrete[active]
        est.feature_importances_ = scores
        est.top_features_ = _base.top_features(scores, n_select)
        return est

    def close(self):
        self.plan.close()
