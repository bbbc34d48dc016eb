"""Pin oracle/twoview_ref.py against vectors produced by the reference itself
(tests/golden/make_golden_twoview.py -> twoview.npz, make_golden.py -> dino_*.npz).  CPU only.

The gold-standard oracle runs scipy's least_squares exactly as fun.py:358 does; it is checked
on the clean pair (2 evaluations) and on the 180-inlier synthetic pair through its objective:
the reference's own F_gold and the restatement's F_gold agree in gs_cost."""
import numpy as np
import pytest

from conftest import golden
from oracle import ransac_ref
from oracle import twoview_ref as tv


def test_fmatrix_cameras_and_triangulate_optimal_match_reference():
    z = golden("twoview.npz")
    c1 = golden("dino_c1.npz")
    C1, C2 = tv.fmatrix_cameras(c1["F_file"])
    np.testing.assert_allclose(C1, z["cam_F_file_C1"], rtol=0, atol=1e-15)
    for tag in ("clean", "noisy"):
        p1, p2 = c1[f"{tag}_p1"], c1[f"{tag}_p2"]
        X = np.array([tv.triangulate_optimal(C1, C2, p1[:, i], p2[:, i])
                      for i in range(p1.shape[1])])
        np.testing.assert_allclose(X, z[f"tri_{tag}_X"], rtol=1e-9, atol=1e-9)
    s = golden("synth_c2.npz")
    Cs1, Cs2 = tv.fmatrix_cameras(s["F_ransac"])
    X = np.array([tv.triangulate_optimal(Cs1, Cs2, s["p1"][:, i], s["p2"][:, i])
                  for i in z["tri_c2_idx"]])
    np.testing.assert_allclose(X, z["tri_c2_X"], rtol=1e-9, atol=1e-9)


def test_camera_resectioning_matches_reference():
    z = golden("twoview.npz")
    k = golden("dino_pnp_kat.npz")
    for P, K, R, t in [(z["resect_P"], z["resect_K"], z["resect_R"], z["resect_t"]),
                       (k["Ps"], k["K"], k["R"], k["t"])]:
        for v in range(P.shape[0]):
            Kv, Rv, tv_ = tv.camera_resectioning(P[v])
            np.testing.assert_allclose(Kv, K[v], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(Rv, R[v], rtol=0, atol=1e-12)
            np.testing.assert_allclose(tv_, t[v], rtol=1e-12, atol=1e-12)


def test_relative_camera_pose_matches_reference():
    z = golden("twoview.npz")
    k = golden("dino_pnp_kat.npz")
    C = k["Ps"][None]
    E, K = tv.getEAndK(C, golden("dino_c1.npz")["F_file"])
    np.testing.assert_allclose(E, k["E"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(K, k["K_last"], rtol=1e-14, atol=0)
    for i in range(len(z["pose_pairs"])):
        E = z["pose_K"].T @ z["pose_F"][i] @ z["pose_K"]
        np.testing.assert_allclose(E, z["pose_E"][i], rtol=1e-12, atol=1e-20)
        R, t = tv.relative_camera_pose(z["pose_E"][i], z["pose_y1"][i], z["pose_y2"][i])
        np.testing.assert_allclose(R, z["pose_R"][i], rtol=0, atol=1e-10)
        np.testing.assert_allclose(t, z["pose_t"][i], rtol=0, atol=1e-10)
    R, t = tv.relative_camera_pose(k["E"], *_first_normalised(k["K_last"]))
    np.testing.assert_allclose(R, k["R01"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(R, k["clean_data_eval"][1], rtol=0, atol=1e-12)


def _first_normalised(K):
    c1 = golden("dino_c1.npz")
    y1 = tv.MakeHomogenous(K, c1["clean_p1"].T)
    y2 = tv.MakeHomogenous(K, c1["clean_p2"].T)
    return y1[0, :2], y2[0, :2]


def test_gold_standard_clean_pair_matches_reference():
    z = golden("twoview.npz")
    c1 = golden("dino_c1.npz")
    S = c1["clean_full_S_ransac"]
    Fg, sol = tv.gold_standard(c1["clean_full_F_ransac"], c1["clean_p1"][:, S],
                               c1["clean_p2"][:, S])
    np.testing.assert_allclose(ransac_ref.normalize_F(Fg), ransac_ref.normalize_F(z["gs_clean_F_gold"]),
                               atol=1e-9)
    np.testing.assert_allclose(z["gs_clean_X_init"],
                               [tv.triangulate_optimal(z["gs_clean_C1_init"], tv.I34, a, b)
                                for a, b in zip(c1["clean_p1"][:, S].T, c1["clean_p2"][:, S].T)],
                               rtol=1e-9, atol=1e-9)


def _dense_jac(p, a, b):
    C = p[:12].reshape(3, 4)
    X = p[12:].reshape(-1, 3).T
    N = X.shape[1]
    _, A, B = tv._residuals_jac(C, X, a, b)
    J = np.zeros((4 * N, 12 + 3 * N))
    for k in range(2):
        J[k * N:(k + 1) * N, :12] = A[:, k, :]
    for k in range(4):
        for i in range(3):
            J[k * N + np.arange(N), 12 + 3 * np.arange(N) + i] = B[:, k, i]
    return J


def test_objective_and_converged_gold_standard():
    """The reference objective, profiled: gs_objective(F_RANSAC) <= the reference's initial
    cost (its start, optimal triangulation, is not always optimal), and the reference's final
    F_gold is not a minimum (scipy stopped on ftol).  The converged restatement
    (gold_standard_lm, Schur LM) equals MINPACK LM with the analytic Jacobian from the same
    start, and beats the reference's objective."""
    from scipy.optimize import least_squares
    z = golden("twoview.npz")
    p1, p2, S = z["gs_s300_p1"], z["gs_s300_p2"], z["gs_s300_S_ransac"]
    a, b = p1[:, S], p2[:, S]
    C1, _ = tv.fmatrix_cameras(z["gs_s300_F_ransac"])
    X0 = np.array([tv.triangulate_optimal(C1, tv.I34, u, v) for u, v in zip(a.T, b.T)]).T
    assert tv.gs_cost_at(C1, X0, a, b) == pytest.approx(float(z["gs_s300_cost_init"]), rel=1e-9)
    obj_ref = tv.gs_objective(z["gs_s300_F_gold"], a, b)
    assert obj_ref <= float(z["gs_s300_cost_final"])
    F, info = tv.gold_standard_lm(z["gs_s300_F_ransac"], a, b)
    sol = least_squares(tv.fmatrix_residuals_gs, np.hstack([C1.ravel(), X0.T.ravel()]),
                        jac=_dense_jac, args=(a, b), method="lm", ftol=1e-15, xtol=1e-15,
                        gtol=1e-15)
    assert info["cost"] == pytest.approx(sol.cost, rel=1e-12)
    Fs = tv.fmatrix_from_cameras(sol.x[:12].reshape(3, 4), tv.I34)
    np.testing.assert_allclose(ransac_ref.normalize_F(F), ransac_ref.normalize_F(Fs), atol=1e-9)
    assert tv.gs_objective(F, a, b) <= obj_ref
    assert info["cost"] <= float(z["gs_s300_cost_final"])


def test_vectorised_2point_jacobian_equals_scipy():
    """oracle.twoview_ref.fmatrix_residuals_gs_jac_2point = scipy's approx_derivative(
    '2-point') of the residual (the Jacobian fun.py:358's least_squares forms), bit for bit
    and in scipy's column-major layout, at the reference's noisy / s300 starts."""
    from scipy.optimize._numdiff import approx_derivative
    from conftest import golden
    tr = golden("gs_trace.npz")
    c1, tvz = golden("dino_c1.npz"), golden("twoview.npz")
    cases = {"noisy": (c1["noisy_p1"][:, c1["noisy_full_S_ransac"]],
                       c1["noisy_p2"][:, c1["noisy_full_S_ransac"]]),
             "s300": (tvz["gs_s300_p1"][:, tvz["gs_s300_S_ransac"]],
                      tvz["gs_s300_p2"][:, tvz["gs_s300_S_ransac"]])}
    for tag, (a, b) in cases.items():
        x0 = tr[f"{tag}_x0"]
        assert np.array_equal(tv.fmatrix_residuals_gs(x0, a, b), tr[f"{tag}_f0"])
        J = tv.fmatrix_residuals_gs_jac_2point(x0, a, b)
        Jr = approx_derivative(tv.fmatrix_residuals_gs, x0, method="2-point", args=(a, b))
        assert J.flags["F_CONTIGUOUS"] and J.shape == Jr.shape
        assert np.array_equal(J, Jr)
        assert np.array_equal(np.signbit(J), np.signbit(Jr))
