"""Pin oracle/tables_ref.py against the reference's own outputs (tests/golden/tables.npz,
written by tests/golden/make_golden_tables.py).  CPU only."""
import numpy as np
import pytest

from conftest import golden
from oracle import tables_ref as tr


@pytest.mark.parametrize("tag", ["clean", "noisy"])
def test_matching_loop_matches_reference(tag):
    z = golden("tables.npz")
    g = lambda k: z[f"{tag}_{k}"]
    m = tr.match_observations(g("match_obs_coords"), g("match_obs_point"), g("match_queries"))
    found = m >= 0
    nC = int(g("ba_n_views"))
    pts = g("ba_x_final")[12 * nC:].reshape(-1, 3)     # the table's points after BA
    np.testing.assert_array_equal(pts[m[found]], g("match_D3"))
    np.testing.assert_array_equal(g("match_y2")[found], g("match_Dimg"))
    np.testing.assert_array_equal(g("match_y1")[~found], g("match_A_y1"))
    np.testing.assert_array_equal(g("match_y2")[~found], g("match_A_y2"))


@pytest.mark.parametrize("tag", ["clean", "noisy"])
def test_add_new_points_matches_reference(tag):
    z = golden("tables.npz")
    g = lambda k: z[f"{tag}_{k}"]
    C1, C2 = g("new_C1"), g("new_C2")
    E = tr.getEFromCameras(C1[:, :3], C1[:, 3], C2[:, :3], C2[:, 3])
    np.testing.assert_allclose(E, g("new_E"), rtol=0, atol=1e-15)
    mask, X = tr.add_new_points(g("new_y1_hom"), g("new_y2_hom"), C1, C2)
    np.testing.assert_array_equal(mask, g("new_gate"))
    assert int(mask.sum()) == int(g("new_added")) and (~mask).sum() > 0
    np.testing.assert_allclose(X, g("new_X"), rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("tag", ["clean", "noisy"])
def test_ba_residuals_and_mask_match_reference(tag):
    z = golden("tables.npz")
    g = lambda k: z[f"{tag}_{k}"]
    nC, nP = int(g("ba_n_views")), int(g("ba_n_points"))
    view, point, y = g("ba_obs_view"), g("ba_obs_point"), g("ba_obs_coords")
    for x, r in ((g("ba_x0"), g("ba_r0")), (g("ba_x1"), g("ba_r1"))):
        cams, pts = x[:12 * nC].reshape(nC, 3, 4), x[12 * nC:].reshape(nP, 3)
        np.testing.assert_allclose(tr.ba_residuals(cams, pts, view, point, y[:, 0], y[:, 1]), r,
                                   rtol=1e-12, atol=1e-15)
    m = tr.ba_sparsity(nC, nP, view, point)
    rows, cols = np.nonzero(m)
    assert np.array_equal(rows, g("ba_mask_rows")) and np.array_equal(cols, g("ba_mask_cols"))
    assert m.shape == tuple(g("ba_mask_shape"))


def test_ba_jacobian_finite_differences():
    z = golden("tables.npz")
    g = lambda k: z[f"noisy_{k}"]
    nC, nP = int(g("ba_n_views")), int(g("ba_n_points"))
    view, point, y = g("ba_obs_view"), g("ba_obs_point"), g("ba_obs_coords")
    x = g("ba_x1")
    cams, pts = x[:12 * nC].reshape(nC, 3, 4), x[12 * nC:].reshape(nP, 3)
    Jc, Jp = tr.ba_jacobian(cams, pts, view, point)
    f = lambda c, p: tr.ba_residuals(c, p, view, point, y[:, 0], y[:, 1]).reshape(-1, 2)
    h = 1e-7
    for k in (0, 5, 11):
        d = np.zeros((nC, 12))
        d[:, k] = h
        num = (f(cams + d.reshape(nC, 3, 4), pts) - f(cams - d.reshape(nC, 3, 4), pts)) / (2 * h)
        np.testing.assert_allclose(num, Jc[:, :, k], rtol=1e-5, atol=1e-7)
    for k in range(3):
        d = np.zeros((nP, 3))
        d[:, k] = h
        num = (f(cams, pts + d) - f(cams, pts - d)) / (2 * h)
        np.testing.assert_allclose(num, Jp[:, :, k], rtol=1e-5, atol=1e-7)


def test_bundle_adjust_lm_not_worse_than_reference():
    z = golden("tables.npz")
    g = lambda k: z[f"noisy_{k}"]
    nC, nP = int(g("ba_n_views")), int(g("ba_n_points"))
    view, point, y = g("ba_obs_view"), g("ba_obs_point"), g("ba_obs_coords")
    x0 = g("ba_x0")
    cams, pts = x0[:12 * nC].reshape(nC, 3, 4), x0[12 * nC:].reshape(nP, 3)
    c2, p2, info = tr.bundle_adjust_lm(cams, pts, view, point, y[:, 0], y[:, 1])
    assert info["cost"] <= float(g("ba_cost_final"))
    np.testing.assert_array_equal(c2[0], cams[0])           # camera 0 fixed, as the mask
    r = tr.ba_residuals(c2, p2, view, point, y[:, 0], y[:, 1])
    assert 0.5 * r @ r == pytest.approx(info["cost"], rel=1e-12)
