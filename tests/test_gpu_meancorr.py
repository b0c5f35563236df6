"""Exact MultiSURF thresholds on the GPU (VERDICT r3 missing #1 and #2).

k_colsort (fs_colsort.hip) orders every continuous column exactly and gives
the mean correction that makes the pass-1 row means exact; before it, a
4096-bin histogram treated samples sharing a bin as tied and heavy-tailed
columns moved the thresholds (lognormal MultiSURF 2.7e-4 of max |s| at
n = 16384).  Checked here on the device:

* corrected row means vs exact means from sorted columns and float64 prefix
  sums (tests/meancorr.py), on the LDS route (n <= 24576: 32-bit operands at
  n = 1500 / 3000, 16-bit ones at n = 16384) and the large-n route (device
  segmented sort, n = 25000), to 1e-10 relative;
* GPU and CPU backends give the same correction (same keys, same order,
  integer eps sums; only k_rowcorr's summation order differs);
* every row's near hit / near miss count against the oracle's decisions in
  the reference's arithmetic (no flipped decision), and the scores as in
  tests/test_meancorr.py;
* the 16-bit decision check now runs in the plan path (ShardedMultiSURF,
  i.e. bench.py, TuRF's resident scorer and the multi-process RCCL path):
  on the signal-free uniform family it re-runs on 32-bit operands and gives
  exactly the one-shot call's scores.
"""
import importlib.util
import os

import numpy as np
import pytest

from conftest import assert_parity_attributed
from meancorr import assert_means_exact, exact_row_means, plan_row_means
from test_meancorr import TOL, gaussian, lognormal, pareto_spikes

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location("mk_families",
                                               os.path.join(HERE, "golden", "make_families.py"))
mk = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mk)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from fastselect_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")


def _job(X, y, backend="gpu"):
    from fastselect_amd import parallel
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend=backend)
    job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend=backend, shard=False)
    s = job.step().cpu().numpy()
    return job, s, x, recip, isd


MEAN_CASES = {
    "pareto_spikes_1500x300": lambda: pareto_spikes(1500, 300),
    "lognormal_3000x2000": lambda: lognormal(3000, 2000),
    "lognormal_16384x2000": lambda: mk.make("lognormal_16k"),
    "uniform_16384x2000": lambda: mk.make("uniform_16k"),
    "mixed_16384x2000": lambda: mk.make("mixed_16k"),
    "lognormal_25000x64_large_n_route": lambda: lognormal(25000, 64, seed=7),
}


@pytest.mark.parametrize("case", sorted(MEAN_CASES))
def test_gpu_row_means_exact(case):
    X, y = MEAN_CASES[case]()
    job, _, x, recip, isd = _job(X, y)
    try:
        mu = plan_row_means(job)
        q16 = job.plan.calibration()["q16"]
        sc = job.plan.calibration()["SC"]
    finally:
        job.close()
    ex = exact_row_means(x, recip, isd)
    assert_means_exact(mu, ex, sc, q16)


def _grid_columns(n, p, seed=9):
    """Integer levels (bins of one key: no within-bin work at any size) with
    2% of the samples nudged off their level (mixed bins of a few samples)."""
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 40, (n, p)).astype(np.float32) * 25.0
    X += (rng.random((n, p)) < 0.02) * rng.random((n, p)).astype(np.float32)
    return X.astype(np.float32), rng.integers(0, 2, n)


CORR_CASES = {
    "lognormal_3000x2000_crowded": lambda: lognormal(3000, 2000),
    "gaussian_3000x500_binned": lambda: gaussian(3000, 500),
    "grid_3000x300_pure_and_mixed_bins": lambda: _grid_columns(3000, 300),
    # 12288 < n <= 20480: 8192 bins (colsort_bin_bits), the cursor in the
    # bin counters; cfg4's route
    "gaussian_13000x48_8192_bins": lambda: gaussian(13000, 48),
    "grid_13000x32_8192_bins_pure_and_mixed": lambda: _grid_columns(13000, 32),
    "lognormal_13000x32_8192_bins_crowded": lambda: lognormal(13000, 32),
    # the edges of colsort_bin_bits / the instantiated items per thread:
    # 12289 (16 per thread, 8192 bins), 20480 (20, 8192), 20481 (24, 4096)
    "gaussian_12289x32_edge": lambda: gaussian(12289, 32),
    "gaussian_20480x32_edge": lambda: gaussian(20480, 32),
    "grid_20481x16_edge": lambda: _grid_columns(20481, 16),
}


@pytest.mark.parametrize("case", sorted(CORR_CASES))
def test_gpu_and_cpu_corrections_agree(case):
    """Same keys, same order, integer eps sums on both backends, on the
    crowded (full sort) and binned routes (k_colsort's within-bin pass by
    sorted position): the per-row corrections differ only by k_rowcorr's
    float64 summation order."""
    X, y = CORR_CASES[case]()
    jg, *_ = _job(X, y, "gpu")
    jc, *_ = _job(X, y, "cpu")
    try:
        assert jg.plan.calibration()["q16"] == jc.plan.calibration()["q16"]
        cg = jg.rowstats.cpu().numpy()[2::3]
        cc = jc.rowstats.numpy()[2::3]
        s1 = jc.rowstats.numpy()[0::3]
    finally:
        jg.close()
        jc.close()
    assert np.max(np.abs(cg - cc) / s1) < 1e-14


DECISION_CASES = {
    "pareto_spikes_1500x300": lambda: pareto_spikes(1500, 300),
    "lognormal_3000x2000": lambda: lognormal(3000, 2000),
    "lognormal_1200x600_a4": lambda: lognormal(1200, 600, seed=5, a=4.0),
}


@pytest.mark.parametrize("case", sorted(DECISION_CASES))
def test_gpu_decisions_and_scores(case, oracle):
    X, y = DECISION_CASES[case]()
    job, s, *_ = _job(X, y)
    try:
        counts = job.counts.cpu().numpy().reshape(-1, 2).astype(np.int64)
    finally:
        job.close()
    _, ref_counts = oracle.multisurf_decisions(X, y)
    assert_parity_attributed(s, oracle.multisurf_scores(X, y),
                             oracle.multisurf_scores(X, y, accum="f64"), counts, ref_counts,
                             TOL, 10)


def test_plan_path_runs_the_decision_check():
    """ShardedMultiSURF.step() (bench.py's step, TuRF's resident scorer, the
    multi-process path) checks the 16-bit decisions as the one-shot call does:
    uniform noise trips it, the plan moves to 32-bit operands, and the step's
    scores equal the one-shot fit's bit for bit."""
    import fastselect_amd as F
    from fastselect_amd import _lib
    X, y = mk.make("uniform_16k")
    job, s, *_ = _job(X, y)
    try:
        risk, switched = job.last_guard
        assert risk > 5e-6 and switched
        assert not job.plan.calibration()["q16"]
        # later steps stay on 32-bit operands, nothing left to check
        s2 = job.step().cpu().numpy()
        assert job.last_guard == (-1.0, False)
    finally:
        job.close()
    np.testing.assert_array_equal(s, s2)
    one = F.MultiSURF(backend="gpu", n_features_to_select=10).fit(X, y).feature_importances_
    r1, rerun1 = _lib.multisurf_last_guard()
    assert rerun1 and r1 == pytest.approx(risk, rel=1e-12)
    np.testing.assert_array_equal(s, one)


def test_large_n_route_matches_cpu_at_small_n():
    """The colsort_global test hook sends every column through the large-n
    route (device segmented sort + k_colsort_scan); its corrections equal
    the CPU backend's exactly (a child process, as before the hook)."""
    import subprocess
    import sys
    code = (
        "import numpy as np, sys; sys.path[:0] = [%r, %r]\n"
        "from test_meancorr import lognormal, gaussian\n"
        "from fastselect_amd import parallel, _lib\n"
        "_lib.set_test_hook('colsort_global', 1)\n"
        "for X, y in (lognormal(3000, 64, seed=7), gaussian(2000, 100)):\n"
        "    out = []\n"
        "    for be in ('cpu', 'gpu'):\n"
        "        x, yv, recip, isd = parallel.prepare_inputs(X, y, backend=be)\n"
        "        job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend=be, shard=False)\n"
        "        job.step(); out.append(job.rowstats.cpu().numpy()[2::3].copy()); job.close()\n"
        "    d = np.max(np.abs(out[0] - out[1]) / np.maximum(np.abs(out[0]), 1.0))\n"
        "    assert d < 1e-12, d\n"
        "print('ok')\n" % (os.path.dirname(HERE), HERE))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
