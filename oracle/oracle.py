"""Parity oracle -- TEST INFRASTRUCTURE ONLY.

Python driver for ``relief_oracle.c`` (the C restatement of the reference's
``backend='cpu'`` kernels).  It restates the preprocessing each reference
``fit`` performs before calling its CPU host caller, then runs the C kernel:

* ``multisurf_scores``  <- ``MultiSURF.fit``  (src/fast_select/MultiSURF.py:384-440)
* ``relieff_scores``    <- ``ReliefF.fit``    (src/fast_select/ReliefF.py:343-403)
* ``surf_scores``       <- ``SURF.fit``       (src/fast_select/SURF.py:330-372)
* ``top_features``      <- ``np.argsort(scores)[::-1][:n_select]`` (MultiSURF.py:443)

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module; the product (``fastselect_amd``) never does.

Parity status: pinned by the reference's own known-answer tests (see
``tests/test_oracle.py``) and cross-checked against the independent numpy
restatement in ``oracle/relief_np.py``.  No reference golden score vectors
exist, and the reference cannot run here (numba is not installed).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "librelief_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_i64 = ctypes.c_int64


def build() -> str:
    """Compile the oracle with its Makefile (gcc + OpenMP)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    lib = ctypes.CDLL(_LIB_PATH)
    lib.oracle_multisurf.argtypes = [_f32p, _i64, _i64, _f64p, _f32p, _i64p, _i64, ctypes.c_int,
                                     _u8p, _i64, _i64, ctypes.c_int, _f32p]
    lib.oracle_relieff.argtypes = [_f32p, _i64, _i64, _i32p, _f32p, _u8p, _i64, _f32p, _i64,
                                   _i64, _i64, ctypes.c_int, _f32p]
    lib.oracle_surf.argtypes = [_f64p, _i64, _i64, _i32p, _f32p, ctypes.c_int, _u8p, _i64, _i64,
                                ctypes.c_int, _f32p]
    lib.oracle_multisurf_acc.argtypes = lib.oracle_multisurf.argtypes[:-1] + [ctypes.c_int, _f32p]
    lib.oracle_relieff_acc.argtypes = lib.oracle_relieff.argtypes[:-1] + [ctypes.c_int, _f32p]
    lib.oracle_surf_acc.argtypes = lib.oracle_surf.argtypes[:-1] + [ctypes.c_int, _f32p]
    lib.numba_argsort_f32.argtypes = [_f32p, _i64, _i64p]
    lib.oracle_multisurf_decisions.argtypes = [_f32p, _i64, _i64, _f64p, _f32p, _i64p, _i64, _u8p,
                                               _i64, _i64, ctypes.c_int, _f64p, _i64p]
    lib.oracle_multisurf_decisions.restype = ctypes.c_int
    lib.oracle_max_threads.restype = ctypes.c_int
    for fn in (lib.oracle_multisurf, lib.oracle_relieff, lib.oracle_surf, lib.oracle_multisurf_acc,
               lib.oracle_relieff_acc, lib.oracle_surf_acc):
        fn.restype = ctypes.c_int
    _lib = lib
    return lib


def _ptr(a, t):
    return a.ctypes.data_as(t)


def _acc(accum) -> int:
    if accum not in ("f32", "f64"):
        raise ValueError("accum must be 'f32' (the reference) or 'f64'")
    return 1 if accum == "f64" else 0


def max_threads() -> int:
    return int(_load().oracle_max_threads())


def is_discrete_mask(x: np.ndarray, discrete_limit: int) -> np.ndarray:
    """MultiSURF.py:416-420 / ReliefF.py:366-368 / SURF.py:347-350."""
    return np.array([np.unique(x[:, f]).size <= discrete_limit for f in range(x.shape[1])],
                    dtype=bool)


def multisurf_scores(X, y, use_star=False, discrete_limit=10, i_range=None, n_jobs=-1,
                     feat_idx=None, accum="f32"):
    """Reference ``MultiSURF(backend='cpu').fit(X, y).feature_importances_``.
    accum='f64' (parity attribution only, not the reference): the same diffs,
    distances and near/far decisions with every later sum in float64
    (oracle_multisurf_acc)."""
    x = np.ascontiguousarray(X, dtype=np.float32)           # validate_data dtype=float32 (:384-386)
    yv = np.ascontiguousarray(np.asarray(y), dtype=np.float64)  # y kept numeric; compared by value (:216)
    n, p = x.shape
    ranges = (x.max(axis=0) - x.min(axis=0)).astype(np.float32)   # _compute_ranges (:141-144)
    ranges[ranges == 0] = 1                                       # :411
    recip = np.ascontiguousarray((1.0 / ranges).astype(np.float32))  # :412
    is_disc = np.ascontiguousarray(is_discrete_mask(x, discrete_limit).astype(np.uint8))
    fidx = np.arange(p, dtype=np.int64) if feat_idx is None else np.ascontiguousarray(feat_idx, dtype=np.int64)
    i0, i1 = (0, n) if i_range is None else i_range
    out = np.zeros(fidx.size, dtype=np.float32)
    rc = _load().oracle_multisurf_acc(_ptr(x, _f32p), n, p, _ptr(yv, _f64p), _ptr(recip, _f32p),
                                      _ptr(fidx, _i64p), fidx.size, int(bool(use_star)),
                                      _ptr(is_disc, _u8p), i0, i1, int(n_jobs), _acc(accum),
                                      _ptr(out, _f32p))
    if rc != 0:
        raise RuntimeError(f"oracle_multisurf failed: {rc}")
    return out


def multisurf_decisions(X, y, discrete_limit=10, i_range=None, n_jobs=-1, feat_idx=None):
    """(thresholds float64[m], counts int64[m, 2]) of MultiSURF.py:175-217 for
    the focal samples i_range (default all): mu - sigma/2 and the near hit /
    near miss counts in the reference's arithmetic (parity attribution: a
    score difference is flipped decisions or accumulation)."""
    x = np.ascontiguousarray(X, dtype=np.float32)
    yv = np.ascontiguousarray(np.asarray(y), dtype=np.float64)
    n, p = x.shape
    ranges = (x.max(axis=0) - x.min(axis=0)).astype(np.float32)
    ranges[ranges == 0] = 1
    recip = np.ascontiguousarray((1.0 / ranges).astype(np.float32))
    is_disc = np.ascontiguousarray(is_discrete_mask(x, discrete_limit).astype(np.uint8))
    fidx = np.arange(p, dtype=np.int64) if feat_idx is None else np.ascontiguousarray(feat_idx, dtype=np.int64)
    i0, i1 = (0, n) if i_range is None else i_range
    thr = np.zeros(i1 - i0, dtype=np.float64)
    cnt = np.zeros((i1 - i0, 2), dtype=np.int64)
    rc = _load().oracle_multisurf_decisions(_ptr(x, _f32p), n, p, _ptr(yv, _f64p),
                                            _ptr(recip, _f32p), _ptr(fidx, _i64p), fidx.size,
                                            _ptr(is_disc, _u8p), i0, i1, int(n_jobs),
                                            _ptr(thr, _f64p), _ptr(cnt, _i64p))
    if rc != 0:
        raise RuntimeError(f"oracle_multisurf_decisions failed: {rc}")
    return thr, cnt


def relieff_scores(X, y, n_neighbors=3, discrete_limit=10, i_range=None, n_jobs=-1, accum="f32"):
    """Reference ``ReliefF(backend='cpu').fit(X, y).feature_importances_``
    (accum as ``multisurf_scores``)."""
    x64 = np.ascontiguousarray(X, dtype=np.float64)          # validate_data dtype=float64 (:343-345)
    y = np.asarray(y)
    n, p = x64.shape
    classes, y_encoded = np.unique(y, return_inverse=True)   # :351
    if len(classes) < 2:                                      # :352-356
        return np.zeros(p, dtype=np.float32)
    is_disc = is_discrete_mask(x64, discrete_limit)           # :366-368
    class_labels, class_counts = np.unique(y, return_counts=True)   # :373
    class_probs = class_counts / len(y)                       # :374
    y_enc = np.ascontiguousarray(np.searchsorted(class_labels, y).astype(np.int32))  # :375
    ranges = x64.max(axis=0) - x64.min(axis=0)                # :377
    ranges[is_disc] = 1.0                                     # :378
    ranges[ranges == 0] = 1.0                                 # :379
    recip = np.ascontiguousarray((1.0 / ranges).astype(np.float32))   # :380
    x32 = np.ascontiguousarray(x64.astype(np.float32))        # :400
    cp = np.ascontiguousarray(class_probs.astype(np.float32))  # :401
    isd = np.ascontiguousarray(is_disc.astype(np.uint8))
    i0, i1 = (0, n) if i_range is None else i_range
    out = np.zeros(p, dtype=np.float32)
    rc = _load().oracle_relieff_acc(_ptr(x32, _f32p), n, p, _ptr(y_enc, _i32p), _ptr(recip, _f32p),
                                    _ptr(isd, _u8p), int(n_neighbors), _ptr(cp, _f32p), cp.size, i0,
                                    i1, int(n_jobs), _acc(accum), _ptr(out, _f32p))
    if rc != 0:
        raise RuntimeError(f"oracle_relieff failed: {rc}")
    return out


def surf_scores(X, y, use_star=False, discrete_limit=10, i_range=None, n_jobs=-1, accum="f32"):
    """Reference ``SURF(backend='cpu').fit(X, y).feature_importances_``
    (accum as ``multisurf_scores``)."""
    x = np.ascontiguousarray(X, dtype=np.float64)            # validate_data dtype=float64 (:330-332)
    n, p = x.shape
    is_disc = is_discrete_mask(x, discrete_limit)             # :347-350
    ranges = x.max(axis=0) - x.min(axis=0)                    # :352
    ranges[is_disc] = 1.0                                     # :353
    ranges[ranges == 0] = 1.0                                 # :354
    recip = np.ascontiguousarray((1.0 / ranges).astype(np.float32))   # :355
    yi = np.ascontiguousarray(np.asarray(y).astype(np.int32))  # :371
    isd = np.ascontiguousarray(is_disc.astype(np.uint8))
    i0, i1 = (0, n) if i_range is None else i_range
    out = np.zeros(p, dtype=np.float32)
    rc = _load().oracle_surf_acc(_ptr(x, _f64p), n, p, _ptr(yi, _i32p), _ptr(recip, _f32p),
                                 int(bool(use_star)), _ptr(isd, _u8p), i0, i1, int(n_jobs),
                                 _acc(accum), _ptr(out, _f32p))
    if rc != 0:
        raise RuntimeError(f"oracle_surf failed: {rc}")
    return out


def top_features(scores: np.ndarray, n_select: int) -> np.ndarray:
    """MultiSURF.py:443 / ReliefF.py:406 / SURF.py:375."""
    return np.argsort(scores)[::-1][:n_select]


def numba_argsort(a: np.ndarray) -> np.ndarray:
    """numba's quicksort argsort on a float32 vector (ReliefF.py:157)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    r = np.empty(a.size, dtype=np.int64)
    _load().numba_argsort_f32(_ptr(a, _f32p), a.size, _ptr(r, _i64p))
    return r
