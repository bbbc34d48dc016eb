"""Host-side helpers (CPU): Rodrigues, ransac.py helpers."""
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
