"""The numba-quicksort replay used for ReliefF ties
(``numba_argsort_focus``, fastselect_amd/csrc/fs_internal.h) against the
oracle's port of numba's argsort: with every element in focus it must give
numba's exact permutation; with a focus subset, the same relative order of
the focus elements."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("argsort") / "argsort_focus_check")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", "argsort_focus_check.cpp"),
                    "-o", exe], check=True)
    return exe


def run(driver, tmp_path, keys, interest):
    kf, inf, of = (str(tmp_path / n) for n in ("k.bin", "i.bin", "o.bin"))
    keys.astype(np.float32).tofile(kf)
    interest.astype(np.uint8).tofile(inf)
    subprocess.run([driver, kf, inf, of], check=True)
    return np.fromfile(of, dtype=np.int32)


@pytest.mark.parametrize("n,levels,seed", [(10, 3, 0), (400, 5, 1), (5000, 40, 2), (20000, 3, 3),
                                           (3000, 100000, 4)])
def test_full_and_focused_replay_match_numba(driver, tmp_path, oracle, n, levels, seed):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, levels, n).astype(np.float32)
    keys[rng.integers(0, n)] = np.inf
    ref = oracle.numba_argsort(keys)
    full = run(driver, tmp_path, keys, np.ones(n, bool))
    np.testing.assert_array_equal(full, ref)
    for v in np.unique(keys)[:3]:
        focus = keys == v
        out = run(driver, tmp_path, keys, focus)
        np.testing.assert_array_equal(out[focus[out]], ref[focus[ref]])
