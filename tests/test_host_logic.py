"""Host-side helpers (CPU): Rodrigues, ransac.py helpers."""
import json
import os
import random

import numpy as np

from tsbb15_amd import cv, ransac


def test_rodrigues_roundtrip():
    rng = np.random.RandomState(0)
    for _ in range(50):
        r = rng.randn(3)
        r = r / np.linalg.norm(r) * rng.uniform(0, 3.1)
        R, _ = cv.Rodrigues(r)
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
        r2, _ = cv.Rodrigues(R)
        np.testing.assert_allclose(r2.ravel(), r, atol=1e-9)


def test_ransac_helpers():
    assert abs(ransac.calc_r(0.5, 8, 0.99) - 1176.6) < 0.1
    y1, y2 = np.array([2.0, 4.0, 2.0]), np.array([1.0, 1.0, 1.0])
    assert ransac.norm_p(y1) == [1.0, 2.0, 1.0]
    assert ransac.cart(y1) == [1.0, 2.0]
    assert ransac.dpp_squared(y1, y2) == 1.0 and ransac.dpp(y1, y2) == 1.0
    R = np.eye(3)
    assert np.array_equal(ransac.calc_y_prim(np.ones(3), R, np.ones(3)), 2 * np.ones(3))


def _misc():
    with open(os.path.join(os.path.dirname(__file__), "golden", "ransac_misc.json")) as f:
        return json.load(f)


def test_calc_p_calc_r_drop_in_equal_reference():
    """The drop-in ransac.calc_p / calc_r (ransac.py:6-10) against the values the reference
    itself returned (tests/golden/ransac_misc.json, written by tests/golden/make_golden.py)."""
    misc = _misc()
    for w, n, p, val in misc["calc_r"]:
        assert ransac.calc_r(w, n, p) == val
    for w, n, r, val in misc["calc_p"]:
        assert ransac.calc_p(w, n, r) == val


def test_gen_rnd_indices_drop_in_equal_reference():
    """ransac.gen_rnd_indices (ransac.py:12-19) on the global CPython stream: the reference's
    own output after random.seed(s), call by call."""
    misc = _misc()
    for key, (seed, L, n) in (("gen_rnd_indices_seed0_500_6", (0, 500, 6)),
                              ("gen_rnd_indices_seed12345_37_6", (12345, 37, 6))):
        random.seed(seed)
        got = [list(ransac.gen_rnd_indices(L, n)) for _ in range(len(misc[key]))]
        assert got == [list(x) for x in misc[key]]


def test_normalise_each_is_batch_independent():
    """twoview.normalise_each (the C-normalised first correspondences of the C4 paths): a
    point's bits do not depend on which other points are normalised with it, so the fused
    device call and the separate calls agree field for field; the values are fun.MakeHomogenous's
    K^-1 [u, v, 1] (fun.py:48-55) to rounding."""
    from conftest import golden
    from tsbb15_amd import twoview
    K = golden("dino_pnp_kat.npz")["K_last"]
    rng = np.random.default_rng(3)
    P = rng.uniform(0.0, 720.0, (257, 2))
    full = twoview.normalise_each(K, P)
    for sub in (np.arange(1), np.arange(5, 9), rng.choice(257, 100, replace=False), np.arange(257)):
        assert np.array_equal(twoview.normalise_each(K, P[sub]), full[sub])
    ref = (np.linalg.inv(K) @ np.vstack([P.T, np.ones((1, len(P)))])).T
    np.testing.assert_allclose(full, ref, rtol=1e-14, atol=1e-15)
