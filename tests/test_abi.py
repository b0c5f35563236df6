"""The C ABI (include/fastselect_amd.h): the in-tree library loads, exports
every declared symbol, and reports errors the documented way.  No GPU compute
here (the container has no GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fastselect_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"FS_API\s+[\w\s\*]+?\b(fs_\w+)\s*\(", text)))


def test_header_declares_expected_api():
    from fastselect_amd import _lib
    assert declared_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    from fastselect_amd import _lib
    assert os.path.dirname(_lib.LIB_PATH) == os.path.join(ROOT, "fastselect_amd")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), f"{name} not exported"


def test_version_and_device_count():
    from fastselect_amd import _lib
    assert "fastselect_amd" in _lib.version()
    assert _lib.device_count() >= 0
    _lib.release_device_cache()  # nothing cached (or no device): a no-op


def test_gpu_backend_without_device_is_an_error():
    from fastselect_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    x = np.random.default_rng(0).standard_normal((10, 3)).astype(np.float32)
    with pytest.raises(RuntimeError, match="no HIP device"):
        _lib.multisurf_score("gpu", x, np.arange(10) % 2, np.ones(3, np.float32), None, False,
                             np.zeros(3, bool))


def test_invalid_arguments_raise_value_error():
    from fastselect_amd import _lib
    x = np.zeros((1, 3), np.float32)  # n < 2
    with pytest.raises(ValueError):
        _lib.multisurf_score("cpu", x, [0], np.ones(3, np.float32), None, False,
                             np.zeros(3, bool))
    x = np.random.default_rng(0).standard_normal((5, 3)).astype(np.float32)
    with pytest.raises(ValueError):  # feat_idx out of range
        _lib.multisurf_score("cpu", x, np.arange(5) % 2, np.ones(3, np.float32),
                             np.array([0, 7]), False, np.zeros(3, bool))
    with pytest.raises(ValueError):  # y_enc outside [0, n_classes)
        _lib.relieff_score("cpu", x, np.array([0, 1, 2, 0, 1]), np.ones(3, np.float32),
                           np.zeros(3, bool), 1, np.array([0.5, 0.5], np.float32))
    lib = _lib.lib()
    rc = lib.fs_multisurf_score(7, 0, None, 0, 0, None, None, None, 0, 0, None, -1,
                                (ctypes.c_float * 1)())
    assert rc == _lib.FS_EINVAL
    assert b"backend" in lib.fs_last_error()


def test_plan_lifecycle_cpu():
    """fs_plan_* on the CPU backend: stages compose to fs_multisurf_score."""
    from fastselect_amd import _lib
    rng = np.random.default_rng(1)
    x = rng.standard_normal((150, 9)).astype(np.float32)
    y = (x[:, 0] + 0.3 * rng.standard_normal(150) > 0).astype(float)
    r = (x.max(0) - x.min(0)).astype(np.float32)
    recip = (1 / r).astype(np.float32)
    isd = np.zeros(9, bool)
    pl = _lib.Plan("cpu", x, y, recip, isd)
    rs, cn, sc = np.zeros(450), np.zeros(300), np.zeros(9)
    pl.pass1(rs.ctypes.data)
    pl.select(rs.ctypes.data, cn.ctypes.data)
    pl.pass2(cn.ctypes.data, sc.ctypes.data)
    tiles, pfe, refined = pl.info()
    assert tiles == 3 and pfe == 2 * 3 * 128 * 128 * 9 and refined >= 0
    assert pl.kernel_ms(0) == -1.0
    pl.close()
    one = _lib.multisurf_score("cpu", x, y, recip, None, False, isd)
    np.testing.assert_allclose((sc / 150).astype(np.float32), one, rtol=0, atol=1e-7)


def _np_stats(x, cap):
    nd = np.array([min(np.unique(x[:, f]).size, cap + 1) for f in range(x.shape[1])])
    return x.min(axis=0), x.max(axis=0), nd


def column_stats_cases():
    rng = np.random.default_rng(5)
    x = rng.standard_normal((300, 70))
    x[:, 0] = rng.integers(0, 3, 300)               # 3 levels
    x[:, 1] = 7.5                                   # constant
    x[:, 2] = rng.choice([-0.0, 0.0, 1.0], 300)     # signed zeros are one value
    x[:, 3] = rng.integers(0, 11, 300)              # exactly 11 levels
    x[:, 4] = rng.integers(0, 40, 300)              # many levels (> 32: hash path)
    x[:5, 5] = 1e30                                 # huge values
    return x


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("cap", [0, 2, 10, 11, 50])
def test_column_stats_cpu_matches_numpy(dtype, cap):
    from fastselect_amd import _lib
    x = column_stats_cases().astype(dtype)
    mn, mx, nd = _lib.column_stats("cpu", x, cap)
    emn, emx, end = _np_stats(x, cap)
    assert mn.dtype == dtype and mx.dtype == dtype
    np.testing.assert_array_equal(mn, emn)
    np.testing.assert_array_equal(mx, emx)
    np.testing.assert_array_equal(nd, end)


def test_column_preprocess_is_reference_discrete_mask():
    from fastselect_amd import _base
    x = column_stats_cases()
    for limit in (-1, 0, 3, 10, 11, 12.5, 40):
        isd, _, _ = _base.column_preprocess(x, limit, "cpu")
        ref = np.array([np.unique(x[:, f]).size <= limit for f in range(x.shape[1])])
        np.testing.assert_array_equal(isd, ref)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_all_finite(dtype):
    """fs_all_finite: the estimators' replacement for scikit-learn's scan."""
    from fastselect_amd import _lib
    x = np.random.default_rng(0).normal(size=(3001, 37)).astype(dtype)
    assert _lib.all_finite(x)
    for bad in (np.nan, np.inf, -np.inf):
        y = x.copy()
        y[2999, 36] = bad
        assert not _lib.all_finite(y)
        assert not _lib.all_finite(y, n_jobs=1)
    assert _lib.all_finite(np.zeros((0, 5), dtype=dtype))


def test_estimators_keep_sklearn_finiteness_errors():
    """Non-finite X raises scikit-learn's own ValueError (message included),
    also for float64 values that overflow the float32 cast of MultiSURF."""
    from fastselect_amd import MultiSURF, ReliefF, SURF
    rng = np.random.default_rng(1)
    X = rng.normal(size=(40, 6))
    y = np.arange(40) % 2
    for est in (MultiSURF(backend="cpu"), ReliefF(backend="cpu"), SURF(backend="cpu")):
        Xi = X.copy()
        Xi[3, 2] = np.inf
        with pytest.raises(ValueError, match="Input X contains infinity"):
            est.fit(Xi, y)
    Xo = X.copy()
    Xo[5, 1] = 1e300
    with pytest.raises(ValueError, match="Input X contains infinity or a value too large"):
        MultiSURF(backend="cpu").fit(Xo, y)
    SURF(backend="cpu").fit(Xo, y)  # float64 estimators accept it, as the reference


def test_threaded_float32_cast_equals_numpy():
    """_base.to_float32 (row blocks over threads) is numpy's float32 cast."""
    from fastselect_amd import _base
    rng = np.random.default_rng(3)
    x = rng.normal(size=(4800, 1800)) * 10.0 ** rng.integers(-30, 30, size=(4800, 1800))
    # the strided view holds 2400 x 1799 > 1 << 22 elements: the threaded path
    assert x[::2, 1:].size > (1 << 22)
    for arr in (x, np.asfortranarray(x), x[::2, 1:]):
        got = _base.to_float32(arr, n_jobs=4)
        assert got.flags.c_contiguous and got.dtype == np.float32
        np.testing.assert_array_equal(got, np.ascontiguousarray(arr, dtype=np.float32))


def test_cpu_preprocessing_does_not_pin_host_memory(monkeypatch):
    """a backend='cpu' fit must not touch the HIP runtime
    -- the threaded float32 cast uses plain host memory unless the fit scores
    on the GPU (pinned=True)."""
    from fastselect_amd import _base, _lib
    from fastselect_amd.ReliefF import relieff_inputs

    def boom(*a, **k):
        raise AssertionError("pinned host memory requested by a CPU fit")

    monkeypatch.setattr(_lib, "pinned_empty", boom)
    rng = np.random.default_rng(5)
    x = rng.normal(size=(2100, 2000))
    y = np.arange(2100) % 2
    assert x.size >= (1 << 22)
    got = _base.to_float32(x, n_jobs=4)
    np.testing.assert_array_equal(got, x.astype(np.float32))
    from fastselect_amd import ReliefF
    xv, _ = _base.validate_xy(ReliefF(backend="cpu"), x, y, np.float32, 4)
    np.testing.assert_array_equal(xv, x.astype(np.float32))
    x32 = relieff_inputs(x, y, 10, "cpu", n_jobs=4)[0]
    np.testing.assert_array_equal(x32, x.astype(np.float32))
