"""SURF / SURF* estimator (reference: src/fast_select/SURF.py:220-425).

``fit`` validates and preprocesses exactly as the reference (SURF.py:330-355)
and makes one call to ``fs_surf_score``, which replaces
``_surf_{cpu,gpu}_host_caller``.
"""
from __future__ import annotations

import numpy as np
from sklearn.base import BaseEstimator, TransformerMixin
from sklearn.utils.validation import check_is_fitted, validate_data

from . import _base, _lib

# reference wording (SURF.py:342, matched by tests/test_surf.py:130) kept as a
# substring
SURF_GPU_MISSING = ("backend='gpu', but no CUDA-enabled GPU is available. In this build: no "
                    "HIP-enabled GPU is available (it targets AMD MI355X / gfx950).")


def surf_inputs(X, discrete_limit, where, device=0):
    """SURF.fit's preprocessing after validation (SURF.py:347-355): discrete
    detection and reciprocal ranges (discrete and constant columns -> 1),
    computed on ``where``.  Returns (is_discrete, recip f32)."""
    is_discrete, col_min, col_max = _base.column_preprocess(X, discrete_limit, where, device)
    feature_ranges = col_max - col_min
    feature_ranges[is_discrete] = 1.0
    feature_ranges[feature_ranges == 0] = 1.0
    return is_discrete, (1.0 / feature_ranges).astype(np.float32)


class SURF(TransformerMixin, BaseEstimator):
    """MI355X-accelerated feature selection with SURF / SURF*.

    Parameters
    ----------
    n_features_to_select : int or float, default=0.2
        Number (int) or fraction (float in (0, 1]) of top features to select.
    backend : {'auto', 'gpu', 'cpu'}, default='auto'
        Compute backend (see ``MultiSURF``).
    use_star : bool, default=False
        Run SURF* (far hits add, far misses subtract).
    discrete_limit : int, default=10
        Features with at most this many distinct values are discrete.
    n_jobs : int, default=-1
        CPU threads for backend='cpu' (-1 = all).
    verbose : bool, default=False
        Print progress messages.
    devices : None, 'all', int or sequence of int, default=None
        GPU ordinals the GPU backend scores on, one host thread each (whole
        128-sample blocks of the focal samples per thread, X moved over the
        host link once and shared by peer copies, the score sums added on
        the host).  None: device 0, as the reference; 'all': every visible
        device the job has work for (one per 4096 samples).  Not a reference
        parameter; ignored by backend='cpu'.
    accumulation : {'fast', 'reference'}, default='fast'
        'reference': the reference's float32 arithmetic in its n_jobs=1
        order -- per sample the four float32 sums over neighbours in
        ascending order (near hits, near misses, far hits, far misses), the
        float32 score update and one sequential float32 sum over the samples
        (SURF.py:139-218) -- its scores bit for bit.  'fast': each pair's two
        directions folded into one weight, float64 partial sums.  Not a
        reference parameter; 'reference' runs on one device.
    """

    def __init__(
        self,
        n_features_to_select: int | float = 0.2,
        backend: str = "auto",
        use_star: bool = False,
        discrete_limit: int = 10,
        n_jobs: int = -1,
        verbose: bool = False,
        devices=None,
        accumulation: str = "fast",
    ):
        self.n_features_to_select = n_features_to_select
        self.backend = backend
        self.use_star = use_star
        self.discrete_limit = discrete_limit
        self.n_jobs = n_jobs
        self.verbose = verbose
        self.devices = devices
        self.accumulation = accumulation

    def _validate_parameters(self, n_samples, n_features):
        _lib.accumulation_code(self.accumulation)
        return _base.resolve_n_select("SURF", self.backend, self.n_features_to_select,
                                      n_samples, n_features)

    def fit(self, X: np.ndarray, y: np.ndarray):
        """Score every feature with SURF (or SURF*)."""
        X, y = _base.validate_xy(self, X, y, np.float64, self.n_jobs)
        self.n_features_in_ = X.shape[1]
        n_samples = X.shape[0]
        n_select = self._validate_parameters(n_samples, self.n_features_in_)

        if self.backend == "auto":
            self.effective_backend_ = "gpu" if _lib.gpu_available() else "cpu"
        elif self.backend == "gpu" and not _lib.gpu_available():
            raise RuntimeError(SURF_GPU_MISSING)
        else:
            self.effective_backend_ = self.backend

        self.devices_ = _base.fit_devices(self.devices, self.effective_backend_, n_samples)
        _base.check_accumulation_devices(self.accumulation, self.devices_)
        dev0 = self.devices_[0] if self.devices_ else 0
        X = np.ascontiguousarray(X)
        # one upload of X for the whole fit (a multi-device fit uploads per device)
        multi = self.devices_ is not None and len(self.devices_) > 1
        with _lib.staged_x("cpu" if multi else self.effective_backend_, X, dev0):
            self.is_discrete_, recip_full = surf_inputs(X, self.discrete_limit,
                                                        self.effective_backend_, dev0)

            algo_name = "SURF*" if self.use_star else "SURF"
            if self.verbose:
                print(f"Running {algo_name} on the {self.effective_backend_.upper()} now...")
            with _lib.accumulation(self.accumulation):
                scores = _lib.surf_score(self.effective_backend_, X, y.astype(np.int32),
                                         recip_full, self.use_star, self.is_discrete_,
                                         self.n_jobs, devices=self.devices_)
        self.feature_importances_ = scores
        self.top_features_ = _base.top_features(scores, n_select)
        if self.verbose:
            print("Feature scoring completed.")
        return self

    def _resident_scorer(self, X, y):
        """A scorer for TuRF that keeps X resident and re-scores column
        subsets (``ResidentRows``)."""
        from ._resident import ResidentRows
        X, y = _base.validate_xy(self, X, y, np.float64, self.n_jobs)
        n = X.shape[0]
        self._validate_parameters(n, X.shape[1])
        if self.backend == "auto":
            self.effective_backend_ = "gpu" if _lib.gpu_available() else "cpu"
        elif self.backend == "gpu" and not _lib.gpu_available():
            raise RuntimeError(SURF_GPU_MISSING)
        else:
            self.effective_backend_ = self.backend
        is_discrete, recip = surf_inputs(X, self.discrete_limit, self.effective_backend_)
        with _lib.accumulation(self.accumulation):  # the plan keeps its creation mode
            plan = _lib.RowsPlan(self.effective_backend_, "surf", X, y.astype(np.int32), recip,
                                 is_discrete, use_star=self.use_star, n_jobs=self.n_jobs)
        return ResidentRows(self, "SURF*" if self.use_star else "SURF", plan, n, is_discrete,
                            self.effective_backend_)

    def transform(self, x: np.ndarray) -> np.ndarray:
        """Reduce x to the selected features."""
        check_is_fitted(self)
        x = validate_data(self, x, reset=False, dtype=[np.float64, np.float32])
        return x[:, self.top_features_]

    def fit_transform(self, X: np.ndarray, y: np.ndarray) -> np.ndarray:
        """Fit to data, then transform it."""
        self.fit(X, y)
        return self.transform(X)
