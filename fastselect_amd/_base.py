"""Shared pieces of the Relief estimators (parameter checks, backend choice,
feature preprocessing), restating the reference's per-estimator code:
``_validate_parameters`` (MultiSURF.py:337-366, ReliefF.py:299-335,
SURF.py:283-312) and the ``backend`` dispatch in each ``fit``.
"""
from __future__ import annotations

import numpy as np

from . import _lib

# The reference's wording is kept as a substring (MultiSURF.py:400-403;
# callers match it, tests/test_multisurf.py:176), followed by what it means here.
GPU_MISSING = ("backend='gpu' was selected, but no compatible NVIDIA GPU was found or CUDA "
               "toolkit is not installed -- in this build: no compatible GPU was found (no HIP "
               "device is visible; it targets AMD MI355X / gfx950).")


def resolve_n_select(name: str, backend: str, n_features_to_select, n_samples: int,
                     n_features: int) -> int:
    """Backend name, sample count and ``n_features_to_select`` checks."""
    if backend not in ["auto", "gpu", "cpu"]:
        raise ValueError("backend must be one of 'auto', 'gpu', or 'cpu'")
    if n_samples < 2:
        raise ValueError(f"{name} requires at least 2 samples, but got n_samples = {n_samples}")
    return n_select_from(n_features_to_select, n_features)


def n_select_from(n_features_to_select, n_features: int) -> int:
    if isinstance(n_features_to_select, float):
        if not 0.0 < n_features_to_select <= 1.0:
            raise ValueError("If n_features_to_select is a float, it must be in (0, 1].")
        return max(1, int(n_features_to_select * n_features))
    if isinstance(n_features_to_select, int):
        if not 0 < n_features_to_select <= n_features:
            raise ValueError(
                f"If n_features_to_select is an int ({n_features_to_select}), "
                f"it must be > 0 and <= n_features ({n_features}).")
        return int(n_features_to_select)
    raise TypeError("n_features_to_select must be an int or a float.")


def validate_xy(est, x, y, dtype, n_jobs=-1, pinned=False):
    """``validate_data(est, x, y, y_numeric=True, dtype=dtype, ensure_2d=True)``
    as the reference's fit calls it, with scikit-learn's single-threaded
    element-wise finiteness scan of X (~56 ms at cfg4) replaced by
    ``fs_all_finite`` on host threads.  When X holds a NaN or an infinity the
    plain call runs again and raises scikit-learn's own error, so behaviour and
    messages are unchanged.  A float64 ndarray bound for float32 is cast by
    ``to_float32`` (the same rounding, over host threads: scikit-learn's cast
    is one thread, ~0.2 s at cfg4); ``pinned`` (a GPU fit) puts the cast in
    pinned host memory.  Returns C-contiguous X."""
    from sklearn.utils.validation import validate_data
    xc = x
    if (dtype == np.float32 and isinstance(x, np.ndarray) and type(x) is np.ndarray
            and x.dtype == np.float64 and x.ndim == 2):
        xc = to_float32(x, n_jobs, pinned)
    xv, yv = validate_data(est, xc, y, y_numeric=True, dtype=dtype, ensure_2d=True,
                           ensure_all_finite=False)
    xv = np.ascontiguousarray(xv)
    if xv.dtype in (np.float32, np.float64) and not _lib.all_finite(xv, n_jobs):
        validate_data(est, x, y, y_numeric=True, dtype=dtype, ensure_2d=True)
    return xv, yv


AUTO_ROWS_PER_DEVICE = 4096


def _device_list(devices, count: int):
    """devices as a list of ordinals, or None when it is not a valid value.
    None -> [0] (one device, as the reference); 'all' -> every visible one."""
    if devices is None:
        return [0] if count > 0 else None
    if isinstance(devices, str) and devices == "all":
        return list(range(count)) or None
    def ordinal(d):
        return isinstance(d, (int, np.integer)) and not isinstance(d, (bool, np.bool_))

    if ordinal(devices):
        devs = [int(devices)]
    elif isinstance(devices, (str, bytes)) or not hasattr(devices, "__iter__"):
        return None
    else:
        devs = list(devices)
        if not all(ordinal(d) for d in devs):
            return None
        devs = [int(d) for d in devs]
    if not devs or any(d < 0 or d >= count for d in devs):
        return None
    return devs


def fit_devices(devices, backend: str, n_samples: int):
    """The GPU ordinals a fit scores on (SURVEY.md §5 "Config / flags", §8(b)
    "one host thread per device"), or None for backend 'cpu'.

    devices=None: device 0, as the reference (fanning out by
    default changed the code path, and the last bits of the scores, with the
    number of visible GPUs); 'all': every visible device, as many as the job
    has work for (one per AUTO_ROWS_PER_DEVICE samples, at least one); an
    int: that device; a sequence: those ordinals, repeats allowed (several
    plans share a device).  Raises ValueError for anything else."""
    if backend != "gpu":
        return None
    count = _lib.device_count()
    devs = _device_list(devices, count)
    if devs is None:
        raise ValueError(f"devices must be None, 'all', a device ordinal or a non-empty "
                         f"sequence of ordinals in [0, {count}); got {devices!r}")
    if isinstance(devices, str):
        devs = devs[:max(1, min(len(devs), int(n_samples) // AUTO_ROWS_PER_DEVICE))]
    return devs


def check_accumulation_devices(accumulation: str, devices) -> None:
    """accumulation='reference' replays one sequential float32 column sum
    per feature, so it scores on one device (ValueError for several)."""
    if accumulation == "reference" and devices is not None and len(devices) > 1:
        raise ValueError("accumulation='reference' runs on one device; got devices="
                         f"{list(devices)!r}")


def stage_device(backend: str, devices=None, n_samples=None):
    """The device a fit may stage X on while validating it: the fit's one
    device when backend is 'auto' or 'gpu', a HIP device is visible and the
    fit will run on a single device; else None (multi-device fits upload
    per device).  Raises nothing: backend and device errors keep their place
    after validation."""
    if backend not in ("auto", "gpu") or not _lib.gpu_available():
        return None
    devs = _device_list(devices, _lib.device_count())
    if devs is None:
        return None
    if isinstance(devices, str) and n_samples is not None:
        devs = devs[:max(1, min(len(devs), int(n_samples) // AUTO_ROWS_PER_DEVICE))]
    return devs[0] if len(devs) == 1 else None


def rows_hint(x):
    """Sample count of an array-like before validation (None if unknown)."""
    try:
        return int(np.shape(x)[0])
    except (TypeError, ValueError, IndexError):
        return None


def validate_xy_staged(est, x, y, dtype, n_jobs=-1, device=None):
    """``validate_xy`` that, for a C-contiguous float64 or float32 ndarray
    bound for float32 and a ``device`` (stage_device), casts (or copies into
    pinned memory), scans and uploads X in one native pass (fs_stage_x_cast:
    the upload of each row block overlaps the casting of later ones).
    Returns (x, y, handle): handle != 0 names the device copy of x, to be
    released with ``_lib.unstaged(handle)``; 0 means x was not staged (other
    inputs take validate_xy)."""
    if (device is None or dtype != np.float32 or type(x) is not np.ndarray
            or x.dtype not in (np.float64, np.float32) or x.ndim != 2
            or not x.flags.c_contiguous
            or x.size < (1 << 20)):
        xv, yv = validate_xy(est, x, y, dtype, n_jobs, pinned=device is not None)
        return xv, yv, 0
    from sklearn.utils.validation import validate_data
    x32, finite, h = _lib.stage_x_cast(x, n_jobs, device)
    try:
        xv, yv = validate_data(est, x32, y, y_numeric=True, dtype=dtype, ensure_2d=True,
                               ensure_all_finite=False)
        xv = np.ascontiguousarray(xv)
        if not finite:  # scikit-learn's own error for the NaN / infinity
            validate_data(est, x, y, y_numeric=True, dtype=dtype, ensure_2d=True)
    except BaseException:
        if h:
            _lib.lib().fs_unstage_x(h)
        raise
    return xv, yv, h


def to_float32(x: np.ndarray, n_jobs: int = -1, pinned: bool = False) -> np.ndarray:
    """``np.ascontiguousarray(x, dtype=np.float32)`` (the reference's cast,
    round to nearest) with the conversion of large arrays split over threads
    by row blocks (numpy releases the GIL in the copy): 15.8 ms on one thread
    for ReliefF's cfg3 matrix.  ``pinned`` (only for fits that score on the
    GPU: it initialises the HIP runtime) puts the result in pinned host
    memory (_lib.pinned_empty), so that its upload is a DMA."""
    if x.dtype == np.float32 and x.flags.c_contiguous:
        return x
    n = x.shape[0] if x.ndim else 0
    nt = _lib.host_threads(n_jobs)
    if x.ndim != 2 or x.size < (1 << 22) or nt <= 1:
        return np.ascontiguousarray(x, dtype=np.float32)
    from concurrent.futures import ThreadPoolExecutor
    # pinned pages (GPU visible): the cast lands in mapped memory and the
    # upload of X is a DMA from it
    out = _lib.pinned_empty(x.shape, np.float32) if pinned else None
    if out is None:
        out = np.empty(x.shape, dtype=np.float32)
    edges = np.linspace(0, n, min(n, 4 * nt) + 1).astype(np.int64)
    with ThreadPoolExecutor(max_workers=nt) as ex:
        list(ex.map(lambda k: np.copyto(out[edges[k]:edges[k + 1]], x[edges[k]:edges[k + 1]],
                                        casting="same_kind"), range(len(edges) - 1)))
    return out


def effective_backend(backend: str) -> str:
    """'auto' -> 'gpu' when a HIP device is visible, else 'cpu'.  An explicit
    'gpu' without a device raises instead of falling back."""
    if backend == "auto":
        return "gpu" if _lib.gpu_available() else "cpu"
    if backend == "gpu" and not _lib.gpu_available():
        raise RuntimeError(GPU_MISSING)
    return backend


def column_preprocess(x: np.ndarray, discrete_limit, backend: str, device: int = 0):
    """The per-column preprocessing of the reference's fit(): returns
    (is_discrete, colmin, colmax) with is_discrete[f] =
    ``np.unique(x[:, f]).size <= discrete_limit`` (MultiSURF.py:416-420,
    ReliefF.py:366-368, SURF.py:347-350) and colmin / colmax = x.min(0) /
    x.max(0) in x's dtype.  Computed by ``fs_column_stats`` on the device the
    estimator scores on ('gpu': HIP kernels on ``device``; 'cpu': native
    threads)."""
    cap = max(0, int(np.floor(discrete_limit)))
    where = backend
    if where == "gpu" and cap > _lib.GPU_STATS_MAX_CAP:
        where = "cpu"  # hash set beyond the GPU kernel's LDS table
    mn, mx, nd = _lib.column_stats(where, x, cap, device=device)
    return nd <= discrete_limit, mn, mx


def discrete_mask(x: np.ndarray, discrete_limit: int, backend: str = "cpu") -> np.ndarray:
    """``np.unique(x[:, f]).size <= discrete_limit`` per column."""
    return column_preprocess(x, discrete_limit, backend)[0]


def top_features(scores: np.ndarray, n_select: int) -> np.ndarray:
    """``np.argsort(scores)[::-1][:n_select]`` (MultiSURF.py:443): numpy's own
    argsort on the float32 scores, so ties order exactly as the reference."""
    return np.argsort(scores)[::-1][:n_select]
