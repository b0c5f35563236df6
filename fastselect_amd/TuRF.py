"""TuRF meta-estimator (reference: src/fast_select/TuRF.py:7-136).

Iterative Relief: score with a base estimator, drop the lowest-scoring
``pct_remove`` fraction of the remaining features (at least one, never going
below ``n_features_to_select``), re-score on the survivors, repeat.  It works
with any estimator exposing ``feature_importances_``; the MI355X ``ReliefF``
/ ``SURF`` / ``MultiSURF`` of this package keep X resident across rounds.
"""
from __future__ import annotations

import numpy as np
from sklearn.base import BaseEstimator, TransformerMixin, clone
from sklearn.utils.validation import check_is_fitted, validate_data


class TuRF(TransformerMixin, BaseEstimator):
    """Iterative Relief feature elimination.

    Parameters
    ----------
    estimator : estimator object
        Base scorer (cloned, never modified).
    n_features_to_select : int, default=10
        Number of features to keep.
    pct_remove : float, default=0.1
        Fraction of the remaining features removed per iteration, in (0, 1).
    n_iterations : int or None, default=None
        Maximum number of elimination rounds (None: until
        ``n_features_to_select`` remain).
    verbose : bool, default=False
        Print one line per iteration.
    """

    def __init__(self, estimator, n_features_to_select: int = 10, pct_remove: float = 0.1,
                 n_iterations: int | None = None, verbose: bool = False):
        self.estimator = estimator
        self.n_features_to_select = n_features_to_select
        self.pct_remove = pct_remove
        self.n_iterations = n_iterations
        self.verbose = verbose

    def fit(self, X: np.ndarray, y: np.ndarray):
        """Run the elimination loop (TuRF.py:61-120)."""
        X, y = validate_data(self, X, y, y_numeric=True, dtype=np.float64, ensure_2d=True)
        self.n_features_in_ = X.shape[1]
        if not 0 < self.pct_remove < 1:
            raise ValueError("pct_remove must be between 0 and 1.")

        scorer = clone(self.estimator)
        active = np.arange(self.n_features_in_)
        # Estimators that can keep X resident re-score column subsets in place
        # (MultiSURF, ReliefF, SURF: a device-resident plan re-targeted with
        # fs_plan_set_features); any other estimator --
        # or one that declines (None) -- is refit on X[:, active] as the
        # reference does.
        resident = getattr(scorer, "_resident_scorer", None)
        runner = resident(X, y) if resident is not None else None
        try:
            if runner is not None:
                runner.refit(active)
            else:
                scorer.fit(X, y)
            self.feature_importances_ = scorer.feature_importances_.copy()

            scores = self.feature_importances_.copy()
            rounds = 0
            while len(active) > self.n_features_to_select:
                if self.n_iterations is not None and rounds >= self.n_iterations:
                    break
                drop = max(1, int(len(active) * self.pct_remove))
                drop = min(drop, len(active) - self.n_features_to_select)
                worst = np.argsort(scores)[:drop]
                active = np.delete(active, worst)
                if self.verbose:
                    print(f"Iteration {rounds}: {len(active)} features remaining.")
                if runner is not None:
                    runner.refit(active)
                else:
                    scorer.fit(X[:, active], y)
                scores = scorer.feature_importances_
                rounds += 1
        finally:
            if runner is not None:
                runner.close()

        ranked = active[np.argsort(scores)[::-1]]
        self.top_features_ = np.sort(ranked)
        return self

    def transform(self, X: np.ndarray) -> np.ndarray:
        """Reduce X to the selected features."""
        check_is_fitted(self)
        X = validate_data(self, X, reset=False, dtype=[np.float64, np.float32])
        return X[:, self.top_features_]

    def fit_transform(self, X: np.ndarray, y: np.ndarray) -> np.ndarray:
        """Fit to data, then transform it."""
        self.fit(X, y)
        return self.transform(X)
