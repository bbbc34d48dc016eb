"""The table-level drop-ins (tsbb15_amd.tables.add_new_view / add_new_points_table, replacing
Tables.addNewView / addNewPoints at tables.py:104-175) on a Tables-compatible fixture rebuilt
from tests/golden/tables.npz (tests/tables_fixture.py), against what the reference's own
methods produced in make_golden_tables.py.

With the golden's stand-in PnP (the reference run had no OpenCV; make_golden_tables.py:120-128)
the bookkeeping must be the reference's exactly: the D / A partition, the new view's pose, one
observation per consensus point (image coordinates y2_hom, the matched 3D point index), then
addNewPoints' count, points and observation pairs.  With the GPU solvePnPRansac the new pose
must reproject its consensus set within the 8 px threshold, and too few matches must raise a
ValueError naming the count."""
import numpy as np
import pytest

from conftest import golden
from oracle import tables_ref as tr
from tables_fixture import Pose, tables_after_ba
from tsbb15_amd import cv
from tsbb15_amd import tables as gt

pytestmark = pytest.mark.gpu


def _found(g):
    """Which putative correspondences match a known 3D point (oracle restatement)."""
    return tr.match_observations(g("match_obs_coords"), g("match_obs_point"),
                                 g("match_queries")) >= 0


def _stand_in(z, tag, captured):
    def fake_pnp(D3, Dimg, K, dist, useExtrinsicGuess=True):
        captured["D3"], captured["Dimg"] = np.array(D3), np.array(Dimg)
        return (True, np.zeros((3, 1)), z[f"{tag}_pnp_t"].reshape(3, 1),
                np.arange(len(D3)).reshape(-1, 1))

    def fake_rodrigues(r, dst=None):
        return z[f"{tag}_pnp_R"].copy(), None
    return fake_pnp, fake_rodrigues


@pytest.mark.parametrize("tag", ["clean", "noisy"])
def test_add_new_view_then_new_points_match_reference(ctx, tag):
    z = golden("tables.npz")
    g = lambda k: z[f"{tag}_{k}"]
    T = tables_after_ba(z, tag)
    n_obs0, n_pts0 = T.T_obs.size, T.T_points.size
    cap = {}
    pnp, rod = _stand_in(z, tag, cap)
    A_y1, A_y2 = gt.add_new_view(T, g("K"), 2, g("match_queries"), g("match_y2_hom"),
                                 g("match_y1"), g("match_y2"), solvePnPRansac=pnp, Rodrigues=rod)
    np.testing.assert_array_equal(A_y1, g("match_A_y1"))
    np.testing.assert_array_equal(A_y2, g("match_A_y2"))
    np.testing.assert_array_equal(cap["D3"], g("match_D3"))
    np.testing.assert_array_equal(cap["Dimg"], g("match_Dimg"))
    # the new view, with the table's own pose class, and one observation per consensus point
    assert T.T_views.size == 3 and isinstance(T.T_views[2].camera_pose, Pose)
    np.testing.assert_array_equal(T.T_views[2].camera_pose.R, g("pnp_R"))
    np.testing.assert_array_equal(T.T_views[2].camera_pose.t, g("pnp_t"))
    nD = len(g("match_D3"))
    assert T.T_obs.size == n_obs0 + nD
    np.testing.assert_array_equal(T.T_views[2].observations_index,
                                  np.r_[0, np.arange(n_obs0, n_obs0 + nD)])
    found = _found(g)
    new_obs = T.T_obs[n_obs0:]
    np.testing.assert_array_equal(np.array([o.image_coordinates for o in new_obs]),
                                  g("match_y2_hom")[found])
    pts = np.array([T.T_points[o.point_3D_index].point for o in new_obs])
    np.testing.assert_array_equal(pts, g("match_D3"))
    assert all(o.view_index == 2 for o in new_obs)
    np.testing.assert_array_equal(T.T_views[2].camera_pose.GetCameraMatrix(), g("new_C2"))

    # Tables.addNewPoints(A_y1_hom, A_y2_hom, 1, 2) on the same table
    n_obs1 = T.T_obs.size
    added = gt.add_new_points_table(T, g("new_y1_hom"), g("new_y2_hom"), 1, 2)
    assert added == int(g("new_added"))
    X = np.array([p.point for p in T.T_points[n_pts0:]])
    ref = g("new_X")
    err = np.abs(X - ref).max(axis=1) / np.abs(ref).max(axis=1)
    assert err.max() < 1e-6, err.max()
    acc = np.flatnonzero(g("new_gate"))
    obs = T.T_obs[n_obs1:]
    assert len(obs) == 2 * added
    for k, i in enumerate(acc):
        o1, o2 = obs[2 * k], obs[2 * k + 1]
        assert (o1.view_index, o2.view_index) == (1, 2)
        assert o1.point_3D_index == o2.point_3D_index == n_pts0 + k
        np.testing.assert_array_equal(o1.image_coordinates, g("new_y1_hom")[i])
        np.testing.assert_array_equal(o2.image_coordinates, g("new_y2_hom")[i])
        np.testing.assert_array_equal(T.T_points[n_pts0 + k].observations_index,
                                      [0, n_obs1 + 2 * k, n_obs1 + 2 * k + 1])


@pytest.mark.parametrize("tag", ["clean", "noisy"])
def test_add_new_view_with_gpu_solvepnpransac(ctx, tag):
    z = golden("tables.npz")
    g = lambda k: z[f"{tag}_{k}"]
    T = tables_after_ba(z, tag)
    n_obs0 = T.T_obs.size
    A_y1, _ = gt.add_new_view(T, g("K"), 2, g("match_queries"), g("match_y2_hom"),
                              g("match_y1"), g("match_y2"))
    np.testing.assert_array_equal(A_y1, g("match_A_y1"))
    C = T.T_views[2].camera_pose
    new_obs = T.T_obs[n_obs0:]
    assert len(new_obs) >= 6
    X = np.array([T.T_points[o.point_3D_index].point for o in new_obs])
    uv = (g("K") @ np.array([o.image_coordinates for o in new_obs]).T).T[:, :2]
    rv, _ = cv.Rodrigues(C.R)
    e = np.linalg.norm(cv.project_points(X, rv, C.t, g("K")) - uv, axis=1)
    # the RANSAC consensus (<= 8 px under the RANSAC pose); LM moves the pose only slightly
    assert np.median(e) < 8.0 and e.max() < 16.0, (np.median(e), e.max())
    # the golden's stand-in pose is the true BAdino2 pose of view 2 in this frame
    assert np.abs(C.R - g("pnp_R")).max() < 0.05


def test_add_new_view_too_few_matches_raises(ctx):
    z = golden("tables.npz")
    g = lambda k: z["clean_" + k]
    T = tables_after_ba(z, "clean")
    n_views = T.T_views.size
    found = _found(g)
    keep = np.sort(np.r_[np.flatnonzero(found)[:3], np.flatnonzero(~found)])
    with pytest.raises(ValueError, match=r"\b3 putative correspondences matched"):
        gt.add_new_view(T, g("K"), 2, g("match_queries")[keep], g("match_y2_hom")[keep],
                        g("match_y1")[keep], g("match_y2")[keep])
    assert T.T_views.size == n_views


@pytest.mark.parametrize("n", [4, 5])
def test_add_new_view_registers_with_4_or_5_matches(ctx, n):
    """Views with only 4 or 5 matched 2D<->3D correspondences register, as OpenCV's kernels
    (P3P / EPnP) allow: the pose from exactly those points, every one an inlier."""
    z = golden("tables.npz")
    g = lambda k: z["clean_" + k]
    T = tables_after_ba(z, "clean")
    n_views, n_obs0 = T.T_views.size, T.T_obs.size
    found = _found(g)
    keep = np.sort(np.r_[np.flatnonzero(found)[:n], np.flatnonzero(~found)])
    gt.add_new_view(T, g("K"), 2, g("match_queries")[keep], g("match_y2_hom")[keep],
                    g("match_y1")[keep], g("match_y2")[keep])
    assert T.T_views.size == n_views + 1 and T.T_obs.size == n_obs0 + n
    assert np.abs(T.T_views[2].camera_pose.R - g("pnp_R")).max() < 0.05
