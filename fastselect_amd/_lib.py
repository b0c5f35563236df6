"""ctypes binding of ``libfastselect_amd.so`` (C ABI: ``include/fastselect_amd.h``).

The shared library holds both the hand-written HIP kernels (gfx950) and the
native CPU backend.  It is loaded eagerly when the package is imported: if it
is missing, importing ``fastselect_amd`` fails loudly -- there is no Python or
PyTorch fallback for the scoring path.

Each ``*_score`` function here replaces one reference host caller
(``_multisurf_{cpu,gpu}_host_caller`` MultiSURF.py:147-162/256-270,
``_relieff_{cpu,gpu}_host_caller`` ReliefF.py:127-134/222-236,
``_surf_{cpu,gpu}_host_caller`` SURF.py:117-128/198-218): plain numpy arrays
in, float32 scores already divided by n out.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfastselect_amd.so")

FS_OK, FS_EINVAL, FS_ENODEV, FS_EOOM, FS_EHIP, FS_ENOTSUP = 0, -1, -2, -3, -4, -5
BACKEND_CPU, BACKEND_GPU = 0, 1

_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_i64 = ctypes.c_int64
_int = ctypes.c_int
_vp = ctypes.c_void_p

# every symbol include/fastselect_amd.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "fs_version", "fs_last_error", "fs_device_count", "fs_device_cache_release",
    "fs_stage_x", "fs_stage_x_device", "fs_stage_x_cast", "fs_unstage_x", "fs_all_finite",
    "fs_host_alloc", "fs_host_free",
    "fs_column_stats", "fs_multisurf_score", "fs_multisurf_last_guard", "fs_multisurf_score_rows",
    "fs_relieff_score", "fs_surf_score", "fs_relieff_score_rows", "fs_surf_score_rows",
    "fs_plan_create", "fs_plan_create_relieff", "fs_plan_create_surf", "fs_plan_score", "fs_plan_set_features",
    "fs_plan_pass1", "fs_plan_select", "fs_plan_pass2", "fs_plan_decision_guard", "fs_plan_set_rows",
    "fs_plan_ref_mask_words", "fs_plan_ref_masks", "fs_plan_ref_pass2", "fs_plan_ref_sums",
    "fs_plan_ref_temp",
    "fs_plan_info", "fs_plan_set_shard", "fs_multisurf_shards", "fs_plan_calibration", "fs_plan_calibration_ex", "fs_plan_weighted_pairs", "fs_plan_kernel_ms",
    "fs_plan_destroy", "fs_multisurf_score_devices", "fs_relieff_score_devices",
    "fs_surf_score_devices", "fs_set_accumulation", "fs_get_accumulation", "fs_test_hook",
    "fs_multisurf_score_ex", "fs_relieff_score_ex", "fs_surf_score_ex",
)


def _share_hip_runtime_with_torch() -> None:
    """Load PyTorch's HIP runtime before ours when PyTorch is installed.

    PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7, the
    same SONAME as /opt/rocm's).  Whichever copy is mapped first is the one
    both libraries bind to; if ours came first, torch would map a second HIP
    runtime and fail with "No HIP GPUs are available".  Importing torch first
    gives the process exactly one HIP runtime shared by torch (device memory,
    streams, RCCL via torch.distributed) and the Relief kernels.
    """
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load() -> ctypes.CDLL:
    _share_hip_runtime_with_torch()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"fastselect_amd native library not found at {LIB_PATH}; build it with "
            "`make -C fastselect_amd/csrc` (or __graft_entry__.build()).")
    lib = ctypes.CDLL(LIB_PATH)
    lib.fs_version.restype = ctypes.c_char_p
    lib.fs_last_error.restype = ctypes.c_char_p
    lib.fs_device_count.restype = _int
    lib.fs_device_cache_release.restype = _int
    lib.fs_multisurf_last_guard.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_int)]
    lib.fs_multisurf_last_guard.restype = _int
    lib.fs_stage_x.argtypes = [_int, _vp, _int, _i64, _i64, ctypes.POINTER(ctypes.c_uint64)]
    lib.fs_stage_x.restype = _int
    lib.fs_host_alloc.argtypes = [ctypes.c_uint64, ctypes.POINTER(_vp)]
    lib.fs_host_alloc.restype = _int
    lib.fs_host_free.argtypes = [_vp]
    lib.fs_host_free.restype = _int
    lib.fs_stage_x_device.argtypes = [_int, _vp, _vp, _int, _i64, _i64,
                                      ctypes.POINTER(ctypes.c_uint64)]
    lib.fs_stage_x_device.restype = _int
    lib.fs_stage_x_cast.argtypes = [_int, _vp, _int, _i64, _i64, _int, _vp, ctypes.POINTER(_int),
                                    ctypes.POINTER(ctypes.c_uint64)]
    lib.fs_stage_x_cast.restype = _int
    lib.fs_unstage_x.argtypes = [ctypes.c_uint64]
    lib.fs_unstage_x.restype = _int
    lib.fs_all_finite.argtypes = [_vp, _int, _i64, _i64, _int, ctypes.POINTER(_int)]
    lib.fs_all_finite.restype = _int
    lib.fs_column_stats.argtypes = [_int, _int, _vp, _int, _i64, _i64, _i64, _vp, _vp, _i64p]
    lib.fs_multisurf_score.argtypes = [_int, _int, _f32p, _i64, _i64, _f64p, _f32p, _i64p, _i64,
                                       _int, _u8p, _int, _f32p]
    lib.fs_multisurf_score_rows.argtypes = [_int, _int, _f32p, _i64, _i64, _f64p, _f32p, _i64p,
                                            _i64, _int, _u8p, _int, _i64, _i64, _f64p]
    lib.fs_plan_set_rows.argtypes = [_vp, _i64, _i64]
    lib.fs_relieff_score.argtypes = [_int, _int, _f32p, _i64, _i64, _i32p, _f32p, _u8p, _i64,
                                     _f32p, _i64, _int, _f32p]
    lib.fs_surf_score.argtypes = [_int, _int, _f64p, _i64, _i64, _i32p, _f32p, _int, _u8p, _int,
                                  _f32p]
    # the _ex calls: the same arguments plus the accumulation mode before the output
    lib.fs_multisurf_score_ex.argtypes = list(lib.fs_multisurf_score.argtypes[:-1]) + [_int, _f32p]
    lib.fs_relieff_score_ex.argtypes = list(lib.fs_relieff_score.argtypes[:-1]) + [_int, _f32p]
    lib.fs_surf_score_ex.argtypes = list(lib.fs_surf_score.argtypes[:-1]) + [_int, _f32p]
    lib.fs_relieff_score_rows.argtypes = [_int, _int, _f32p, _i64, _i64, _i32p, _f32p, _u8p,
                                          _i64, _f32p, _i64, _int, _i64, _i64, _f64p]
    lib.fs_surf_score_rows.argtypes = [_int, _int, _f64p, _i64, _i64, _i32p, _f32p, _int, _u8p,
                                       _int, _i64, _i64, _f64p]
    _ip = ctypes.POINTER(_int)
    lib.fs_multisurf_score_devices.argtypes = [_ip, _int, _f32p, _i64, _i64, _f64p, _f32p, _i64p,
                                               _i64, _int, _u8p, _int, _i64, _i64, _f64p]
    lib.fs_relieff_score_devices.argtypes = [_ip, _int, _f32p, _i64, _i64, _i32p, _f32p, _u8p,
                                             _i64, _f32p, _i64, _int, _i64, _i64, _f64p]
    lib.fs_surf_score_devices.argtypes = [_ip, _int, _f64p, _i64, _i64, _i32p, _f32p, _int, _u8p,
                                          _int, _i64, _i64, _f64p]
    lib.fs_plan_create.argtypes = [ctypes.POINTER(_vp), _int, _int, _f32p, _i64, _i64, _f64p,
                                   _f32p, _i64p, _i64, _int, _u8p, _int, _int, _int,
                                   ctypes.c_uint64]
    lib.fs_plan_create_relieff.argtypes = [ctypes.POINTER(_vp), _int, _int, _f32p, _i64, _i64,
                                           _i32p, _f32p, _u8p, _i64, _f32p, _i64, _i64, _i64,
                                           _int, ctypes.c_uint64]
    lib.fs_plan_create_surf.argtypes = [ctypes.POINTER(_vp), _int, _int, _f64p, _i64, _i64,
                                        _i32p, _f32p, _int, _u8p, _i64, _i64, _int,
                                        ctypes.c_uint64]
    lib.fs_plan_score.argtypes = [_vp, _vp]
    lib.fs_plan_set_features.argtypes = [_vp, _i64p, _i64]
    lib.fs_plan_pass1.argtypes = [_vp, _vp]
    lib.fs_plan_select.argtypes = [_vp, _vp, _vp]
    lib.fs_plan_pass2.argtypes = [_vp, _vp, _vp]
    lib.fs_plan_decision_guard.argtypes = [_vp, _vp, _vp, _vp, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(_int)]
    lib.fs_plan_ref_mask_words.argtypes = [_vp, _i64p]
    lib.fs_plan_ref_masks.argtypes = [_vp, _vp, _i64]
    lib.fs_plan_ref_pass2.argtypes = [_vp, _vp, _vp, _i64, _i64]
    lib.fs_plan_ref_sums.argtypes = [_vp, _vp, _vp]
    lib.fs_plan_ref_temp.argtypes = [_vp]
    lib.fs_plan_info.argtypes = [_vp, _i64p, _f64p, _i64p]
    lib.fs_plan_calibration.argtypes = [_vp, _f64p]
    lib.fs_plan_calibration_ex.argtypes = [_vp, _f64p, _int]
    lib.fs_plan_calibration_ex.restype = _int
    lib.fs_plan_set_shard.argtypes = [_vp, _int, _int]
    lib.fs_multisurf_shards.argtypes = [_int, _i64, _i64, _int, ctypes.POINTER(_int)]
    lib.fs_plan_weighted_pairs.argtypes = [_vp, _i64p]
    lib.fs_plan_kernel_ms.argtypes = [_vp, _int]
    lib.fs_plan_kernel_ms.restype = ctypes.c_double
    lib.fs_plan_destroy.argtypes = [_vp]
    lib.fs_set_accumulation.argtypes = [_int, ctypes.POINTER(_int)]
    lib.fs_set_accumulation.restype = _int
    lib.fs_get_accumulation.argtypes = []
    lib.fs_get_accumulation.restype = _int
    lib.fs_test_hook.argtypes = [ctypes.c_char_p, _i64]
    lib.fs_test_hook.restype = _int
    for name in ("fs_column_stats", "fs_multisurf_score", "fs_multisurf_score_rows",
                 "fs_plan_set_rows", "fs_relieff_score", "fs_surf_score",
                 "fs_relieff_score_rows", "fs_surf_score_rows", "fs_plan_create",
                 "fs_plan_create_relieff", "fs_plan_create_surf", "fs_plan_score", "fs_plan_set_features", "fs_plan_pass1", "fs_plan_select",
                 "fs_plan_pass2", "fs_plan_decision_guard", "fs_plan_ref_mask_words", "fs_plan_ref_masks",
                 "fs_plan_ref_pass2", "fs_plan_ref_sums", "fs_plan_ref_temp", "fs_plan_info", "fs_plan_set_shard", "fs_multisurf_shards", "fs_plan_calibration", "fs_plan_weighted_pairs",
                 "fs_plan_destroy", "fs_multisurf_score_devices", "fs_relieff_score_devices",
                 "fs_surf_score_devices", "fs_multisurf_score_ex", "fs_relieff_score_ex",
                 "fs_surf_score_ex"):
        getattr(lib, name).restype = _int
    return lib


_lib = _load()


def lib() -> ctypes.CDLL:
    return _lib


def version() -> str:
    return _lib.fs_version().decode()


@contextlib.contextmanager
def staged_x(backend, x, device=0):
    """One upload of X for a whole fit on the GPU backend (fs_stage_x): the
    column statistics and the scoring call that receive this same array read
    the device copy.  ``x`` must be C-contiguous float32 / float64 and stay
    unchanged inside the block; other backends pass through."""
    if backend != "gpu" or x.dtype not in (np.float32, np.float64) or \
            not x.flags.c_contiguous or x.ndim != 2 or x.size == 0:
        yield
        return
    h = ctypes.c_uint64(0)
    if _lib.fs_stage_x(int(device), x.ctypes.data, int(x.dtype == np.float64), x.shape[0],
                       x.shape[1], ctypes.byref(h)) != 0:
        # staging is only an optimisation: without device room for the extra
        # copy the calls upload X themselves (and report their own errors)
        yield
        return
    try:
        yield
    finally:
        _lib.fs_unstage_x(h)


def stage_x_cast(x, n_jobs=-1, device=0):
    """``x`` (C-contiguous float64 or float32 matrix) cast / copied to
    float32 by fs_stage_x_cast: returns (x32, finite, handle) -- the cast
    array (pinned host memory when possible), whether every value of it is finite, and the handle of its
    device copy on ``device`` (0: not staged; release with ``unstaged``)."""
    out = pinned_empty(x.shape, np.float32)
    if out is None:
        out = np.empty(x.shape, dtype=np.float32)
    fin = _int(0)
    h = ctypes.c_uint64(0)
    check(_lib.fs_stage_x_cast(int(device), x.ctypes.data, int(x.dtype == np.float64),
                               x.shape[0], x.shape[1], int(n_jobs), out.ctypes.data,
                               ctypes.byref(fin), ctypes.byref(h)))
    return out, bool(fin.value), int(h.value)


@contextlib.contextmanager
def unstaged(handle):
    """Release a device copy staged by stage_x_cast (handle 0: nothing) when
    the block ends."""
    try:
        yield
    finally:
        if handle:
            _lib.fs_unstage_x(ctypes.c_uint64(handle))


def pinned_empty(shape, dtype):
    """An uninitialised C-contiguous array in pinned host memory from the
    library's block cache (fs_host_alloc), returned to the cache when the
    array is collected; None when no GPU is visible or pinning fails."""
    import weakref
    dtype = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dtype.itemsize
    if nbytes == 0 or not gpu_available():
        return None
    p = _vp()
    if _lib.fs_host_alloc(ctypes.c_uint64(nbytes), ctypes.byref(p)) != 0 or not p.value:
        return None
    buf = (ctypes.c_char * nbytes).from_address(p.value)
    arr = np.frombuffer(buf, dtype=dtype).reshape(shape)
    fin = weakref.finalize(buf, _lib.fs_host_free, _vp(p.value))
    fin.atexit = False  # at exit the block goes with the process (no HIP call then)
    return arr


def multisurf_shards(n: int, p: int, world: int = 1, device: int = 0) -> int:
    """Tile shards per device that fit a MultiSURF job (fs_multisurf_shards)."""
    v = _int(1)
    check(_lib.fs_multisurf_shards(int(device), int(n), int(p), int(world), ctypes.byref(v)))
    return int(v.value)


@contextlib.contextmanager
def staged_device_x(x, x_device_ptr, device=0):
    """Register a device copy of the host array ``x`` that the caller holds
    (``x_device_ptr``: n x p, same dtype, row-major) for the calls inside the
    block (fs_stage_x_device): the column statistics and the plans given
    ``x`` read it instead of uploading X."""
    h = ctypes.c_uint64(0)
    check(_lib.fs_stage_x_device(int(device), x.ctypes.data, _vp(int(x_device_ptr)),
                                 int(x.dtype == np.float64), x.shape[0], x.shape[1],
                                 ctypes.byref(h)))
    try:
        yield
    finally:
        _lib.fs_unstage_x(h)


def all_finite(x, n_jobs=-1) -> bool:
    """No NaN and no infinity in a C-contiguous float32 / float64 matrix
    (fs_all_finite, host threads)."""
    f = _int(0)
    check(_lib.fs_all_finite(x.ctypes.data, int(x.dtype == np.float64), x.shape[0],
                             int(np.prod(x.shape[1:])), int(n_jobs), ctypes.byref(f)))
    return bool(f.value)


def host_threads(n_jobs=-1) -> int:
    """The native library's thread count for ``n_jobs`` (fs_prep.cpp
    hardware_threads): n_jobs > 0 as given, else the CPUs of this process's
    affinity mask, capped by OMP_NUM_THREADS when set."""
    if n_jobs is not None and n_jobs > 0:
        return int(n_jobs)
    try:
        hw = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        hw = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS", "")
    if cap.isdigit() and 0 < int(cap) < hw:
        hw = int(cap)
    return max(1, hw)


def release_device_cache() -> None:
    """Free the device blocks kept between fits (fs_device_cache_release)."""
    _lib.fs_device_cache_release()


def multisurf_last_guard():
    """(risk, rerun) of this thread's last GPU MultiSURF one-shot call
    (fs_multisurf_last_guard): the 16-bit decision risk (-1 when not
    evaluated) and whether the call scored again on 32-bit operands."""
    risk = ctypes.c_double(-1.0)
    rerun = _int(0)
    _lib.fs_multisurf_last_guard(ctypes.byref(risk), ctypes.byref(rerun))
    return float(risk.value), bool(rerun.value)


def device_count() -> int:
    """Number of visible HIP devices (0 when none)."""
    return int(_lib.fs_device_count())


def gpu_available() -> bool:
    return device_count() > 0


def check(rc: int) -> None:
    """Map a C return code to the Python exception the estimators raise."""
    if rc == FS_OK:
        return
    msg = _lib.fs_last_error().decode(errors="replace")
    if rc == FS_EINVAL:
        raise ValueError(msg)
    if rc == FS_EOOM:
        raise MemoryError(msg)
    raise RuntimeError(msg)


ACCUM_MODES = {"fast": 0, "reference": 1}


def accumulation_code(mode: str) -> int:
    """FS_ACCUM_FAST / FS_ACCUM_REFERENCE for the estimators' ``accumulation``
    parameter ('fast' or 'reference'); ValueError for anything else."""
    if not isinstance(mode, str) or mode not in ACCUM_MODES:
        raise ValueError(f"accumulation must be 'fast' or 'reference'; got {mode!r}")
    return ACCUM_MODES[mode]


@contextlib.contextmanager
def accumulation(mode: str = "fast"):
    """The calling thread's accumulation mode for the native calls (and plan
    creations) inside the block (fs_set_accumulation), restored afterwards.
    'reference' replays the reference's float32 per-sample sums and column
    sums (MultiSURF.py:198-253, ReliefF.py:181-220) bit for bit."""
    code = accumulation_code(mode)
    prev = _int(0)
    check(_lib.fs_set_accumulation(code, ctypes.byref(prev)))
    try:
        yield
    finally:
        _lib.fs_set_accumulation(prev.value, None)


def set_test_hook(name: str, value: int = 1) -> None:
    """TEST-ONLY (fs_test_hook): override one internal choice of the library
    process-wide; ``set_test_hook("reset")`` restores every default."""
    check(_lib.fs_test_hook(name.encode(), int(value)))


@contextlib.contextmanager
def test_hooks(**hooks):
    """TEST-ONLY: the given fs_test_hook overrides inside the block, every
    default restored afterwards."""
    try:
        for k, v in hooks.items():
            set_test_hook(k, int(v))
        yield
    finally:
        set_test_hook("reset")


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


def _backend_code(backend: str) -> int:
    if backend == "gpu":
        return BACKEND_GPU
    if backend == "cpu":
        return BACKEND_CPU
    raise ValueError("backend must be 'cpu' or 'gpu' at the native boundary")


GPU_STATS_MAX_CAP = 8191


def column_stats(backend, x, count_cap, device=0):
    """Column minima, maxima and distinct-value counts (capped at
    ``count_cap + 1``) of a float32 / float64 matrix (``fs_column_stats``):
    the ``x.min(0)``, ``x.max(0)`` and ``np.unique(x[:, f]).size`` of the
    reference's fit() (MultiSURF.py:141-144, 409-420)."""
    x = np.ascontiguousarray(x)
    if x.dtype not in (np.float32, np.float64):
        x = x.astype(np.float64)
    n, p = x.shape
    mn = np.empty(p, dtype=x.dtype)
    mx = np.empty(p, dtype=x.dtype)
    nd = np.empty(p, dtype=np.int64)
    check(_lib.fs_column_stats(_backend_code(backend), int(device), x.ctypes.data,
                               int(x.dtype == np.float64), n, p, int(count_cap), mn.ctypes.data,
                               mx.ctypes.data, _p(nd, _i64p)))
    return mn, mx, nd


def _devices_arg(devices):
    d = np.ascontiguousarray(devices, dtype=np.int32)
    return d, _p(d, ctypes.POINTER(_int)), int(d.size)


def _multi(backend, devices):
    """The *_devices entry point applies: GPU backend and more than one
    device ordinal (one ordinal is the plain call on that device)."""
    return backend == "gpu" and devices is not None and len(devices) > 1


def multisurf_score(backend, x, y, recip, feat_idx, use_star, is_discrete, n_jobs=-1, device=0,
                    rows=None, devices=None):
    """Drop-in for ``_multisurf_{cpu,gpu}_host_caller`` (MultiSURF.py:147-162, 256-270).

    rows=(begin, end): float64 score sums of those focal samples only
    (``fs_multisurf_score_rows``) instead of float32 scores / n.
    devices=[d0, d1, ...] (GPU backend): one host thread per entry
    (``fs_multisurf_score_devices``); one entry = ``device``.
    """
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, p = x.shape
    yv = np.ascontiguousarray(y, dtype=np.float64)
    rc_ = np.ascontiguousarray(recip, dtype=np.float32)
    isd = np.ascontiguousarray(is_discrete, dtype=np.uint8)
    fidx = None if feat_idx is None else np.ascontiguousarray(feat_idx, dtype=np.int64)
    n_kept = p if fidx is None else fidx.size
    if devices is not None and not _multi(backend, devices):
        device = int(devices[0])
    if _multi(backend, devices):
        _keep, dp, nd = _devices_arg(devices)
        lo, hi = (0, n) if rows is None else (int(rows[0]), int(rows[1]))
        sums = np.zeros(n_kept, dtype=np.float64)
        check(_lib.fs_multisurf_score_devices(dp, nd, _p(x, _f32p), n, p, _p(yv, _f64p),
                                              _p(rc_, _f32p),
                                              None if fidx is None else _p(fidx, _i64p), n_kept,
                                              int(bool(use_star)), _p(isd, _u8p), int(n_jobs),
                                              lo, hi, _p(sums, _f64p)))
        return sums if rows is not None else (sums / n).astype(np.float32)
    if rows is not None:
        sums = np.zeros(n_kept, dtype=np.float64)
        check(_lib.fs_multisurf_score_rows(_backend_code(backend), int(device), _p(x, _f32p), n, p,
                                           _p(yv, _f64p), _p(rc_, _f32p),
                                           None if fidx is None else _p(fidx, _i64p), n_kept,
                                           int(bool(use_star)), _p(isd, _u8p), int(n_jobs),
                                           int(rows[0]), int(rows[1]), _p(sums, _f64p)))
        return sums
    out = np.zeros(n_kept, dtype=np.float32)
    check(_lib.fs_multisurf_score(_backend_code(backend), int(device), _p(x, _f32p), n, p,
                                  _p(yv, _f64p), _p(rc_, _f32p),
                                  None if fidx is None else _p(fidx, _i64p), n_kept,
                                  int(bool(use_star)), _p(isd, _u8p), int(n_jobs),
                                  _p(out, _f32p)))
    return out


def relieff_score(backend, x, y_enc, recip, is_discrete, k, class_probs, n_jobs=-1, device=0,
                  rows=None, devices=None):
    """Drop-in for ``_relieff_{cpu,gpu}_host_caller`` (ReliefF.py:127-134, 222-236).

    rows=(begin, end): float64 score sums of those focal samples only
    (``fs_relieff_score_rows``, row sharding) instead of float32 scores / n.
    devices: as ``multisurf_score`` (``fs_relieff_score_devices``).
    """
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, p = x.shape
    ye = np.ascontiguousarray(y_enc, dtype=np.int32)
    rc_ = np.ascontiguousarray(recip, dtype=np.float32)
    isd = np.ascontiguousarray(is_discrete, dtype=np.uint8)
    cp = np.ascontiguousarray(class_probs, dtype=np.float32)
    if devices is not None and not _multi(backend, devices):
        device = int(devices[0])
    if _multi(backend, devices):
        _keep, dp, nd = _devices_arg(devices)
        lo, hi = (0, n) if rows is None else (int(rows[0]), int(rows[1]))
        sums = np.zeros(p, dtype=np.float64)
        check(_lib.fs_relieff_score_devices(dp, nd, _p(x, _f32p), n, p, _p(ye, _i32p),
                                            _p(rc_, _f32p), _p(isd, _u8p), int(k), _p(cp, _f32p),
                                            cp.size, int(n_jobs), lo, hi, _p(sums, _f64p)))
        return sums if rows is not None else (sums / n).astype(np.float32)
    args = (_backend_code(backend), int(device), _p(x, _f32p), n, p, _p(ye, _i32p),
            _p(rc_, _f32p), _p(isd, _u8p), int(k), _p(cp, _f32p), cp.size, int(n_jobs))
    if rows is not None:
        out = np.zeros(p, dtype=np.float64)
        check(_lib.fs_relieff_score_rows(*args, int(rows[0]), int(rows[1]), _p(out, _f64p)))
        return out
    out = np.zeros(p, dtype=np.float32)
    check(_lib.fs_relieff_score(*args, _p(out, _f32p)))
    return out


def surf_score(backend, x, y, recip, use_star, is_discrete, n_jobs=-1, device=0, rows=None,
               devices=None):
    """Drop-in for ``_surf_{cpu,gpu}_host_caller`` (SURF.py:117-128, 198-218).

    rows=(begin, end): float64 score sums of those focal samples only
    (``fs_surf_score_rows``, row sharding) instead of float32 scores / n.
    devices: as ``multisurf_score`` (``fs_surf_score_devices``).
    """
    x = np.ascontiguousarray(x, dtype=np.float64)
    n, p = x.shape
    yi = np.ascontiguousarray(y, dtype=np.int32)
    rc_ = np.ascontiguousarray(recip, dtype=np.float32)
    isd = np.ascontiguousarray(is_discrete, dtype=np.uint8)
    if devices is not None and not _multi(backend, devices):
        device = int(devices[0])
    if _multi(backend, devices):
        _keep, dp, nd = _devices_arg(devices)
        lo, hi = (0, n) if rows is None else (int(rows[0]), int(rows[1]))
        sums = np.zeros(p, dtype=np.float64)
        check(_lib.fs_surf_score_devices(dp, nd, _p(x, _f64p), n, p, _p(yi, _i32p),
                                         _p(rc_, _f32p), int(bool(use_star)), _p(isd, _u8p),
                                         int(n_jobs), lo, hi, _p(sums, _f64p)))
        return sums if rows is not None else (sums / n).astype(np.float32)
    args = (_backend_code(backend), int(device), _p(x, _f64p), n, p, _p(yi, _i32p),
            _p(rc_, _f32p), int(bool(use_star)), _p(isd, _u8p), int(n_jobs))
    if rows is not None:
        out = np.zeros(p, dtype=np.float64)
        check(_lib.fs_surf_score_rows(*args, int(rows[0]), int(rows[1]), _p(out, _f64p)))
        return out
    out = np.zeros(p, dtype=np.float32)
    check(_lib.fs_surf_score(*args, _p(out, _f32p)))
    return out


class Plan:
    """A sharded MultiSURF plan (``fs_plan_*``) for one rank.

    Exchange buffers (rowstats[3n], counts[2n], scores[n_kept], float64) are
    passed by address: device pointers for the GPU backend, host pointers for
    the CPU backend (see ``fastselect_amd.parallel``).
    """

    def __init__(self, backend, x, y, recip, is_discrete, use_star=False, feat_idx=None,
                 rank=0, world=1, n_jobs=-1, device=0, stream=0, _handle=None):
        if _handle is not None:  # built by RowsPlan
            return
        x = np.ascontiguousarray(x, dtype=np.float32)
        self.n, self.p = x.shape
        yv = np.ascontiguousarray(y, dtype=np.float64)
        rc_ = np.ascontiguousarray(recip, dtype=np.float32)
        isd = np.ascontiguousarray(is_discrete, dtype=np.uint8)
        fidx = None if feat_idx is None else np.ascontiguousarray(feat_idx, dtype=np.int64)
        self.n_kept = self.p if fidx is None else fidx.size
        self.backend = backend
        self._h = _vp()
        check(_lib.fs_plan_create(ctypes.byref(self._h), _backend_code(backend), int(device),
                                  _p(x, _f32p), self.n, self.p, _p(yv, _f64p), _p(rc_, _f32p),
                                  None if fidx is None else _p(fidx, _i64p), self.n_kept,
                                  int(bool(use_star)), _p(isd, _u8p), int(rank), int(world),
                                  int(n_jobs), ctypes.c_uint64(int(stream))))

    def set_features(self, feat_idx) -> None:
        """Score another feature subset of the resident samples next
        (``fs_plan_set_features``); pass2 then returns len(feat_idx) sums."""
        fidx = None if feat_idx is None else np.ascontiguousarray(feat_idx, dtype=np.int64)
        self.n_kept = self.p if fidx is None else fidx.size
        check(_lib.fs_plan_set_features(self._h, None if fidx is None else _p(fidx, _i64p),
                                        self.n_kept))

    def pass1(self, rowstats_ptr: int) -> None:
        check(_lib.fs_plan_pass1(self._h, _vp(rowstats_ptr)))

    def select(self, rowstats_ptr: int, counts_ptr: int) -> None:
        check(_lib.fs_plan_select(self._h, _vp(rowstats_ptr), _vp(counts_ptr)))

    def pass2(self, counts_ptr: int, scores_ptr: int) -> None:
        check(_lib.fs_plan_pass2(self._h, _vp(counts_ptr), _vp(scores_ptr)))

    def ref_mask_words(self) -> int:
        """int64 words of the reference-order decision masks (``fs_plan_ref_mask_words``)."""
        w = _i64(0)
        check(_lib.fs_plan_ref_mask_words(self._h, ctypes.byref(w)))
        return int(w.value)

    def ref_masks(self, masks_ptr: int, words: int) -> None:
        """This rank's tile decisions into the zeroed masks (``fs_plan_ref_masks``)."""
        check(_lib.fs_plan_ref_masks(self._h, _vp(masks_ptr), _i64(words)))

    def ref_pass2(self, masks_ptr: int, counts_ptr: int, row_begin: int, row_end: int) -> None:
        """Reference-order chains of the focal rows [row_begin, row_end) into
        the plan's temp rows (``fs_plan_ref_pass2``)."""
        check(_lib.fs_plan_ref_pass2(self._h, _vp(masks_ptr), _vp(counts_ptr), _i64(row_begin),
                                     _i64(row_end)))

    def ref_sums(self, init_ptr: int, sums_ptr: int) -> None:
        """float32 column sums of the temp rows continuing init (0 = none)
        into sums (``fs_plan_ref_sums``)."""
        check(_lib.fs_plan_ref_sums(self._h, _vp(init_ptr or None), _vp(sums_ptr)))

    def decision_guard(self, rowstats_ptr: int, counts_ptr: int, scores_ptr: int):
        """(risk, switched) of the 16-bit decision check after a step whose
        exchange vectors are all-reduced (``fs_plan_decision_guard``);
        switched: the plan now runs on 32-bit operands -- run the step again."""
        risk = ctypes.c_double(-1.0)
        sw = _int(0)
        check(_lib.fs_plan_decision_guard(self._h, _vp(rowstats_ptr), _vp(counts_ptr),
                                          _vp(scores_ptr), ctypes.byref(risk), ctypes.byref(sw)))
        return float(risk.value), bool(sw.value)

    def set_rows(self, begin: int, end: int) -> None:
        """Score only the focal samples [begin, end) in the next pass2
        (``fs_plan_set_rows``; MultiSURF plans)."""
        check(_lib.fs_plan_set_rows(self._h, int(begin), int(end)))

    def info(self):
        """(owned tiles, pair-feature evaluations per step, pairs refined last step)."""
        tiles = ctypes.c_int64(0)
        pfe = ctypes.c_double(0.0)
        ref = ctypes.c_int64(0)
        check(_lib.fs_plan_info(self._h, ctypes.byref(tiles), ctypes.byref(pfe),
                                ctypes.byref(ref)))
        return int(tiles.value), float(pfe.value), int(ref.value)

    def set_shard(self, rank: int, world: int) -> None:
        """Re-target to the pair tiles of shard (rank, world) (fs_plan_set_shard)."""
        check(_lib.fs_plan_set_shard(self._h, int(rank), int(world)))

    def calibration(self) -> dict:
        """Refinement-band calibration of the current layout (fs_plan_calibration)."""
        v = (ctypes.c_double * 8)()
        m = _lib.fs_plan_calibration_ex(self._h, v, 8)
        check(min(m, 0))
        return {"q16": bool(v[0]), "rms": v[1], "max": v[2], "model_sigma": v[3],
                "band_vs_model": v[4], "guard": v[5] in (1.0, 2.0), "row_guard": v[5] == 2.0,
                "surf_f64": v[5] == 3.0, "row_bias_vs_limit": v[6], "SC": v[7]}

    def weighted_pairs(self) -> int:
        """Owned pairs with a non-zero weight in the last pass 2 (-1: not counted)."""
        v = ctypes.c_int64(-1)
        check(_lib.fs_plan_weighted_pairs(self._h, ctypes.byref(v)))
        return int(v.value)

    def kernel_ms(self, which: int) -> float:
        return float(_lib.fs_plan_kernel_ms(self._h, int(which)))

    def close(self) -> None:
        if self._h:
            _lib.fs_plan_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RowsPlan(Plan):
    """A ReliefF or SURF plan (``fs_plan_create_relieff`` / ``_surf``): X
    resident, focal samples ``rows``; ``score(ptr)`` writes the float64 score
    sums of those samples for the current feature subset (``set_features``)."""

    def __init__(self, backend, algo, x, y, recip, is_discrete, k=3, class_probs=None,
                 use_star=False, rows=None, n_jobs=-1, device=0, stream=0):
        super().__init__(None, None, None, None, None, _handle=True)
        self.backend = backend
        self._h = _vp()
        rc_ = np.ascontiguousarray(recip, dtype=np.float32)
        isd = np.ascontiguousarray(is_discrete, dtype=np.uint8)
        yi = np.ascontiguousarray(y, dtype=np.int32)
        if algo == "relieff":
            x = np.ascontiguousarray(x, dtype=np.float32)
            self.n, self.p = x.shape
            lo, hi = (0, self.n) if rows is None else rows
            cp = np.ascontiguousarray(class_probs, dtype=np.float32)
            check(_lib.fs_plan_create_relieff(
                ctypes.byref(self._h), _backend_code(backend), int(device), _p(x, _f32p), self.n,
                self.p, _p(yi, _i32p), _p(rc_, _f32p), _p(isd, _u8p), int(k), _p(cp, _f32p),
                cp.size, int(lo), int(hi), int(n_jobs), ctypes.c_uint64(int(stream))))
        elif algo == "surf":
            x = np.ascontiguousarray(x, dtype=np.float64)
            self.n, self.p = x.shape
            lo, hi = (0, self.n) if rows is None else rows
            check(_lib.fs_plan_create_surf(
                ctypes.byref(self._h), _backend_code(backend), int(device), _p(x, _f64p), self.n,
                self.p, _p(yi, _i32p), _p(rc_, _f32p), int(bool(use_star)), _p(isd, _u8p),
                int(lo), int(hi), int(n_jobs), ctypes.c_uint64(int(stream))))
        else:
            raise ValueError(f"unknown algorithm {algo!r}")
        self.n_kept = self.p

    def score(self, sums_ptr: int) -> None:
        check(_lib.fs_plan_score(self._h, _vp(sums_ptr)))

    def ref_temp(self) -> None:
        """Reference order: the score up to the float32 temp rows, whose column
        sums ``ref_sums`` continues (``fs_plan_ref_temp``; ReliefF, SURF)."""
        check(_lib.fs_plan_ref_temp(self._h))
