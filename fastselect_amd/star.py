"""``SURFstar`` and ``MultiSURFstar``: the star variants as classes of their
own, the names scikit-rebate uses and the reference's benchmark compares
against (benchmarking.py:12-13,34-36).  The reference
exposes them only as ``use_star=True``; these classes are exactly
``SURF(use_star=True)`` / ``MultiSURF(use_star=True)`` with ``use_star``
fixed (it is not a constructor parameter, so ``get_params``/``clone`` never
turn it off).
"""
from __future__ import annotations

from .MultiSURF import MultiSURF
from .SURF import SURF


class SURFstar(SURF):
    """SURF* (far hits add, far misses subtract); parameters as ``SURF``."""

    use_star = True

    def __init__(self, n_features_to_select=0.2, backend="auto", discrete_limit=10, n_jobs=-1,
                 verbose=False, devices=None, accumulation="fast"):
        self.n_features_to_select = n_features_to_select
        self.backend = backend
        self.discrete_limit = discrete_limit
        self.n_jobs = n_jobs
        self.verbose = verbose
        self.devices = devices
        self.accumulation = accumulation


class MultiSURFstar(MultiSURF):
    """MultiSURF* (far misses subtract); parameters as ``MultiSURF``."""

    use_star = True

    def __init__(self, n_features_to_select=0.2, backend="auto", discrete_limit=10, n_jobs=-1,
                 verbose=False, devices=None, accumulation="fast"):
        self.n_features_to_select = n_features_to_select
        self.backend = backend
        self.discrete_limit = discrete_limit
        self.n_jobs = n_jobs
        self.verbose = verbose
        self.devices = devices
        self.accumulation = accumulation
