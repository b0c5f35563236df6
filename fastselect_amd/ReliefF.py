"""ReliefF estimator (reference: src/fast_select/ReliefF.py:239-453).

``fit`` validates and preprocesses exactly as the reference
(ReliefF.py:343-380: float64 validation, single-class shortcut, neighbour
warning, discrete detection, class priors, ranges) and then makes one call to
``fs_relieff_score``, which replaces ``_relieff_{cpu,gpu}_host_caller``.
"""
from __future__ import annotations

import warnings

import numpy as np
from sklearn.base import BaseEstimator, TransformerMixin
from sklearn.utils.validation import check_is_fitted, validate_data

from . import _base, _lib


def relieff_inputs(x, y, discrete_limit, where, device=0, n_jobs=-1):
    """ReliefF.fit's preprocessing after validation (ReliefF.py:366-380, 400):
    discrete detection and column ranges (computed on ``where``), class priors,
    class codes, reciprocal ranges (discrete and constant columns -> 1) and the
    float32 cast.  Returns (x32, y_enc int32, recip f32, is_discrete, priors f32)."""
    is_discrete, col_min, col_max = _base.column_preprocess(x, discrete_limit, where, device)
    class_labels, class_counts = np.unique(y, return_counts=True)
    class_probs = class_counts / len(y)
    y_enc = np.searchsorted(class_labels, y)
    feature_ranges = col_max - col_min
    feature_ranges[is_discrete] = 1.0
    feature_ranges[feature_ranges == 0] = 1.0
    recip = (1.0 / feature_ranges).astype(np.float32)
    return (_base.to_float32(x, n_jobs, pinned=where == "gpu"), y_enc.astype(np.int32), recip, is_discrete,
            class_probs.astype(np.float32))


class ReliefF(TransformerMixin, BaseEstimator):
    """MI355X-accelerated feature selection with the ReliefF algorithm.

    Parameters
    ----------
    n_features_to_select : int or float, default=0.2
        Number (int) or fraction (float in (0, 1]) of top features to select.
    discrete_limit : int, default=10
        Features with at most this many distinct values are discrete.
    n_neighbors : int, default=3
        Nearest hits, and nearest misses per other class, used per sample.
    backend : {'auto', 'gpu', 'cpu'}, default='auto'
        Compute backend (see ``MultiSURF``).
    verbose : bool, default=False
        Print progress messages.
    n_jobs : int, default=-1
        CPU threads for backend='cpu' (-1 = all).
    devices : None, 'all', int or sequence of int, default=None
        GPU ordinals the GPU backend scores on, one host thread each (whole
        128-sample blocks of the focal samples per thread, X moved over the
        host link once and shared by peer copies, the score sums added on
        the host).  None: device 0, as the reference; 'all': every visible
        device the job has work for (one per 4096 samples).  Not a reference
        parameter; ignored by backend='cpu'.
    accumulation : {'fast', 'reference'}, default='fast'
        'reference': each sample's neighbours in the reference's argsort
        order, its float64 update rounded to a float32 row, and each
        feature's float32 sequential column sum (ReliefF.py:181-220) -- the
        reference's scores bit for bit.  'fast': the update summed in
        float64 throughout.  Not a reference parameter; 'reference' runs on
        one device.
    """

    def __init__(
        self,
        n_features_to_select: int | float = 0.2,
        discrete_limit: int = 10,
        n_neighbors: int = 3,
        backend: str = "auto",
        verbose: bool = False,
        n_jobs: int = -1,
        devices=None,
        accumulation: str = "fast",
    ):
        self.n_features_to_select = n_features_to_select
        self.discrete_limit = discrete_limit
        self.n_neighbors = n_neighbors
        self.backend = backend
        self.verbose = verbose
        self.n_jobs = n_jobs
        self.devices = devices
        self.accumulation = accumulation

    def _validate_parameters(self, n_samples, n_features):
        _lib.accumulation_code(self.accumulation)
        if self.backend not in ["auto", "gpu", "cpu"]:
            raise ValueError("backend must be one of 'auto', 'gpu', or 'cpu'")
        if n_samples < 2:
            raise ValueError(
                f"ReliefF requires at least 2 samples, but got n_samples = {n_samples}")
        if not (0 < self.n_neighbors < n_samples):
            raise ValueError(
                f"n_neighbors ({self.n_neighbors}) must be an integer "
                f"between 1 and n_samples - 1 ({n_samples - 1}).")
        return _base.n_select_from(self.n_features_to_select, n_features)

    def fit(self, x: np.ndarray, y: np.ndarray):
        """Score every feature with ReliefF."""
        x, y = _base.validate_xy(self, x, y, np.float64, self.n_jobs)
        self.n_features_in_ = x.shape[1]
        n_samples = x.shape[0]
        n_select = self._validate_parameters(n_samples, self.n_features_in_)

        self.classes_, y_encoded = np.unique(y, return_inverse=True)
        if len(self.classes_) < 2:
            self.feature_importances_ = np.zeros(self.n_features_in_, dtype=np.float32)
            self.top_features_ = np.arange(n_select)
            self.effective_backend_ = "cpu" if self.backend != "gpu" else "gpu"
            return self

        min_class_size = np.min(np.bincount(y_encoded))
        if self.n_neighbors >= min_class_size:
            warnings.warn(
                f"n_neighbors ({self.n_neighbors}) is greater than or equal to the "
                f"smallest class size ({min_class_size}).",
                UserWarning,
            )

        # preprocessing runs where the scoring will (the backend itself is
        # resolved below, after these steps, as in the reference)
        where = "gpu" if self.backend != "cpu" and _lib.gpu_available() else "cpu"
        sd = _base.stage_device(self.backend, self.devices, n_samples)
        x32, y_enc, recip_full, is_discrete, class_probs = relieff_inputs(
            x, y, self.discrete_limit, where, 0 if sd is None else sd, n_jobs=self.n_jobs)
        self.is_discrete_ = is_discrete

        self.effective_backend_ = _base.effective_backend(self.backend)
        self.devices_ = _base.fit_devices(self.devices, self.effective_backend_, n_samples)
        _base.check_accumulation_devices(self.accumulation, self.devices_)
        if self.verbose:
            where = "GPU" if self.effective_backend_ == "gpu" else "CPU"
            print(f"Running ReliefF on the {where} now...")
        with _lib.accumulation(self.accumulation):
            scores = _lib.relieff_score(self.effective_backend_, x32, y_enc, recip_full,
                                        is_discrete, self.n_neighbors, class_probs, self.n_jobs,
                                        devices=self.devices_)
        self.feature_importances_ = scores
        self.top_features_ = _base.top_features(scores, n_select)
        return self

    def _resident_scorer(self, x, y):
        """A scorer for TuRF that keeps X resident and re-scores column
        subsets (``ResidentRows``); None when there is nothing to score
        (a single class: TuRF then refits, which yields zeros)."""
        from ._resident import ResidentRows
        x, y = _base.validate_xy(self, x, y, np.float64, self.n_jobs)
        n = x.shape[0]
        self._validate_parameters(n, x.shape[1])
        classes, y_encoded = np.unique(y, return_inverse=True)
        if len(classes) < 2:
            return None
        self.classes_ = classes
        min_class_size = np.min(np.bincount(y_encoded))

        def warn_small_class():
            if self.n_neighbors >= min_class_size:
                warnings.warn(
                    f"n_neighbors ({self.n_neighbors}) is greater than or equal to the "
                    f"smallest class size ({min_class_size}).",
                    UserWarning,
                )

        where = "gpu" if self.backend != "cpu" and _lib.gpu_available() else "cpu"
        x32, y_enc, recip, is_discrete, class_probs = relieff_inputs(
            x, y, self.discrete_limit, where, n_jobs=self.n_jobs)
        self.effective_backend_ = _base.effective_backend(self.backend)
        with _lib.accumulation(self.accumulation):  # the plan keeps its creation mode
            plan = _lib.RowsPlan(self.effective_backend_, "relieff", x32, y_enc, recip,
                                 is_discrete, k=self.n_neighbors, class_probs=class_probs,
                                 n_jobs=self.n_jobs)
        return ResidentRows(self, "ReliefF", plan, n, is_discrete, self.effective_backend_,
                            before_score=warn_small_class)

    def transform(self, x: np.ndarray) -> np.ndarray:
        """Reduce x to the selected features."""
        check_is_fitted(self)
        x = validate_data(self, x, reset=False, dtype=[np.float64, np.float32])
        return x[:, self.top_features_]

    def fit_transform(self, x: np.ndarray, y: np.ndarray) -> np.ndarray:
        """Fit to data, then transform it."""
        self.fit(x, y)
        return self.transform(x)
