"""MultiSURF / MultiSURF* estimator (reference: src/fast_select/MultiSURF.py).

Same scikit-learn surface as the reference class (MultiSURF.py:273-489):
constructor parameters, ``fit`` / ``transform`` / ``fit_transform``, fitted
attributes ``n_features_in_``, ``feature_importances_``, ``top_features_``,
``is_discrete_``, ``effective_backend_``.  ``fit`` validates and preprocesses
exactly as the reference (MultiSURF.py:384-420) and then makes ONE call into
the native library (``fs_multisurf_score``), which replaces the reference's
host callers.
"""
from __future__ import annotations

import contextlib

import numpy as np
from sklearn.base import BaseEstimator, TransformerMixin
from sklearn.utils.validation import check_is_fitted, validate_data

from . import _base, _lib


class MultiSURF(TransformerMixin, BaseEstimator):
    """MI355X-accelerated feature selection with the MultiSURF algorithm.

    Parameters
    ----------
    n_features_to_select : int or float, default=0.2
        Number (int) or fraction (float in (0, 1]) of top features to select.
    backend : {'auto', 'gpu', 'cpu'}, default='auto'
        'gpu' runs the HIP kernels on an AMD Instinct GPU (raises RuntimeError
        when none is visible), 'cpu' the native multithreaded CPU backend,
        'auto' the GPU when one is visible.
    use_star : bool, default=False
        Run MultiSURF* (far misses are subtracted).
    discrete_limit : int, default=10
        Features with at most this many distinct values are discrete.
    n_jobs : int, default=-1
        CPU threads for backend='cpu' (-1 = all).
    verbose : bool, default=False
        Print progress messages.
    devices : None, 'all', int or sequence of int, default=None
        GPU ordinals the GPU backend scores on, one host thread each (the
        pair tiles dealt round-robin; X crosses the host link once, 1/N of
        the rows per device and the rest by peer copies; the exchange
        vectors are summed device-side).  None: device 0, as the reference;
        'all': every visible device the job has work for (one per 4096
        samples).  Not a reference parameter (the reference is
        single-device); ignored by backend='cpu'.
    accumulation : {'fast', 'reference'}, default='fast'
        'reference' replays the reference's float32 arithmetic: each focal
        sample's near-hit / near-miss diffs summed in float32 in sample
        order, then each feature's float32 sequential column sum
        (MultiSURF.py:198-253), on 32-bit pass-1 operands with exact
        thresholds -- the reference's scores bit for bit, at roughly the
        cost of a second pass 2 (DESIGN.md §Reference-order accumulation).
        'fast' (the default) sums each pair once in float32 streams and
        float64 partials: closer to the exact sums than the reference's own
        float32 sums, not equal to them.  Not a reference parameter;
        'reference' runs on one device.
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
        return _base.resolve_n_select("MultiSURF", self.backend, self.n_features_to_select,
                                      n_samples, n_features)

    def fit(self, x: np.ndarray, y: np.ndarray):
        """Score every feature with MultiSURF (or MultiSURF*)."""
        # float64 X: cast, finiteness scan and upload in one native pass
        sd = _base.stage_device(self.backend, self.devices, _base.rows_hint(x))
        x, y, staged = _base.validate_xy_staged(self, x, y, np.float32, self.n_jobs, sd)
        with _lib.unstaged(staged):
            self.n_features_in_ = x.shape[1]
            n_samples = x.shape[0]
            n_select = self._validate_parameters(n_samples, self.n_features_in_)
            self.effective_backend_ = _base.effective_backend(self.backend)
            self.devices_ = _base.fit_devices(self.devices, self.effective_backend_, n_samples)
            _base.check_accumulation_devices(self.accumulation, self.devices_)
            x = np.ascontiguousarray(x)
            # one upload of X for the whole fit (already done when staged);
            # a multi-device fit uploads X per device
            multi = self.devices_ is not None and len(self.devices_) > 1
            with contextlib.nullcontext() if staged or multi else _lib.staged_x(
                    self.effective_backend_, x, self.devices_[0] if self.devices_ else 0):
                scores = self._score(x, y)
        self.feature_importances_ = scores
        self.top_features_ = _base.top_features(scores, n_select)
        return self

    def _score(self, x, y):
        dev0 = self.devices_[0] if self.devices_ else 0
        is_discrete, col_min, col_max = _base.column_preprocess(x, self.discrete_limit,
                                                                self.effective_backend_, dev0)
        feature_ranges = (col_max - col_min).astype(np.float32)  # _compute_ranges
        feature_ranges[feature_ranges == 0] = 1
        recip_full = (1.0 / feature_ranges).astype(np.float32)
        all_feature_indices = np.arange(self.n_features_in_, dtype=np.int64)
        self.is_discrete_ = is_discrete

        if self.verbose:
            name = "MultiSURF*" if self.use_star else "MultiSURF"
            where = "GPU" if self.effective_backend_ == "gpu" else "CPU"
            print(f"Running {name} on the {where} now...")
        with _lib.accumulation(self.accumulation):
            return _lib.multisurf_score(self.effective_backend_, x, y, recip_full,
                                        all_feature_indices, self.use_star, is_discrete,
                                        self.n_jobs, devices=self.devices_)

    def _resident_scorer(self, x, y):
        """A scorer for TuRF that keeps X resident (on the GPU for the GPU
        backend) and re-scores column subsets through feat_idx, which the
        reference's kernels support for exactly this (MultiSURF.py:147,256):
        ``refit(active)`` leaves this estimator as ``fit(X[:, active], y)``
        would, without copying or re-uploading X."""
        return _ResidentMultiSURF(self, x, y)

    def transform(self, x: np.ndarray) -> np.ndarray:
        """Reduce x to the selected features."""
        check_is_fitted(self)
        x = validate_data(self, x, reset=False, dtype=[np.float64, np.float32])
        return x[:, self.top_features_]

    def fit_transform(self, x: np.ndarray, y: np.ndarray) -> np.ndarray:
        """Fit to data, then transform it."""
        self.fit(x, y)
        return self.transform(x)


class _ResidentMultiSURF:
    """See ``MultiSURF._resident_scorer``."""

    def __init__(self, est: MultiSURF, x, y):
        self.est = est
        _lib.accumulation_code(est.accumulation)
        x, y = _base.validate_xy(est, x, y, np.float32, est.n_jobs,
                                 pinned=_base.stage_device(est.backend) is not None)
        est.effective_backend_ = _base.effective_backend(est.backend)
        self.n = x.shape[0]
        self.is_discrete, col_min, col_max = _base.column_preprocess(
            x, est.discrete_limit, est.effective_backend_)
        ranges = (col_max - col_min).astype(np.float32)
        ranges[ranges == 0] = 1
        recip = (1.0 / ranges).astype(np.float32)
        from .parallel import ShardedMultiSURF
        self.job = ShardedMultiSURF(x, y, recip, self.is_discrete, use_star=est.use_star,
                                    backend=est.effective_backend_, shard=False,
                                    accumulation=est.accumulation)
        self.active = None

    def refit(self, active: np.ndarray):
        est = self.est
        active = np.asarray(active, dtype=np.int64)
        n_select = est._validate_parameters(self.n, active.size)
        est.n_features_in_ = active.size
        if est.verbose:
            name = "MultiSURF*" if est.use_star else "MultiSURF"
            where = "GPU" if est.effective_backend_ == "gpu" else "CPU"
            print(f"Running {name} on the {where} now...")
        if self.active is None or not np.array_equal(active, self.active):
            self.job.set_features(active)
            self.active = active
        scores = self.job.step().cpu().numpy()
        est.is_discrete_ = self.is_discrete[active]
        est.feature_importances_ = scores
        est.top_features_ = _base.top_features(scores, n_select)
        return est

    def close(self):
        self.job.close()
