"""Host-side stages and helpers (CPU): gold-standard refinement (fun.py:343-369),
Rodrigues, ransac.py helpers."""
import numpy as np

from conftest import golden
from oracle import ransac_ref
from tsbb15_amd import cv, ransac, twoview


def test_gold_standard_clean_pair_matches_reference():
    z = golden("dino_c1.npz")
    S = z["clean_full_S_ransac"]
    Fg = twoview.gold_standard(z["clean_full_F_ransac"], z["clean_p1"][:, S], z["clean_p2"][:, S])
    np.testing.assert_allclose(ransac_ref.normalize_F(Fg),
                               ransac_ref.normalize_F(z["clean_full_F_gold"]), atol=1e-9)


def test_twoview_primitives_consistent():
    z = golden("dino_c1.npz")
    F = z["F_file"]
    C1, C2 = twoview.fmatrix_cameras(F)
    F2 = twoview.fmatrix_from_cameras(C1, C2)
    np.testing.assert_allclose(ransac_ref.normalize_F(F2), ransac_ref.normalize_F(F), atol=1e-9)
    x1, x2 = z["clean_p1"][:, 0], z["clean_p2"][:, 0]
    X = twoview.triangulate_optimal(C1, C2, x1, x2)
    np.testing.assert_allclose(twoview.project(X, C1), x1, atol=1e-6)
    np.testing.assert_allclose(twoview.project(X, C2), x2, atol=1e-6)


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
