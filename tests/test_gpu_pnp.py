"""GPU parity of the PnP path (DLT pnp.py:132-160, consensus ransac.py:37-113) against the
oracle restatement and the reference's noise-free BAdino2 scene (R, t from the reference's
fun.camera_resectioning).  Parity with OpenCV solvePnPRansac is unpinned (absent)."""
import random

import numpy as np
import pytest

from conftest import golden
from oracle import pnp_ref
from tsbb15_amd import cv, pnp, ransac, synth

pytestmark = pytest.mark.gpu


def _view(z, v):
    vis = np.flatnonzero(z["points2d"][v, 0] != -1)
    X = z["points3d"][vis]
    uv = z["points2d"][v][:, vis]
    y = (np.linalg.inv(z["K"][v]) @ np.vstack([uv, np.ones((1, len(vis)))])).T
    return X, uv.T, y


def test_dlt_known_answers_badino2(ctx):
    z = golden("dino_pnp_kat.npz")
    for v in (1, 5, 20, 35):
        X, _, y = _view(z, v)
        R, t = pnp.pnp_minimize(X, y, len(X))
        np.testing.assert_allclose(R, z["R"][v], atol=1e-9)
        np.testing.assert_allclose(t, z["t"][v], atol=1e-9)
        R6, t6 = pnp.pnp_minimize(X[:6], y[:6], 6)
        np.testing.assert_allclose(R6, z["R"][v], atol=1e-7)
        Xh = np.hstack([X, np.ones((len(X), 1))])  # homogeneous input form
        R4, _ = pnp.pnp_minimize(Xh, y, len(X))
        np.testing.assert_allclose(R4, R, atol=1e-12)


def test_dlt_noisy_minimal_samples_match_oracle(ctx):
    X, _, y, _, _, inl = synth.pnp_scene(500, 0.0, seed=9)
    rs = np.random.RandomState(1)
    for _ in range(20):
        s = rs.choice(500, 6, replace=False)
        R, t = pnp.pnp_minimize(X[s], y[s], 6)
        Ro, to = pnp_ref.pnp_dlt(X[s], y[s])
        np.testing.assert_allclose(R, Ro, atol=1e-6)
        np.testing.assert_allclose(t, to, rtol=1e-6, atol=1e-6)
    with pytest.raises(ValueError):
        pnp.pnp_minimize(X[:5], y[:5], 5)


def test_ransac_pnp_exact_stream_parity(ctx):
    X, _, y, Rt, tt, truth = synth.pnp_scene(500, 0.30, seed=3)
    thr = (1.5 / 800.0) ** 2
    r = 400
    R, t, im, ih, best, cnt = ransac.ransac_pnp(X, y, X, y, r, thr, 6, rng=random.Random(0))
    Ro, to, imo, iho, besto, counts = pnp_ref.ransac_pnp(y, X, y, X, r, thr, 6,
                                                         rng=random.Random(0), trace=True)
    assert best == besto
    assert cnt == counts.max()
    assert np.array_equal(im, imo) and np.array_equal(ih, iho)
    np.testing.assert_allclose(R, Ro, atol=1e-6)
    np.testing.assert_allclose(t, to, rtol=1e-6, atol=1e-6)
    assert truth[im].mean() > 0.95


def test_gen_rnd_indices_advances_global_stream(ctx):
    random.seed(7)
    a = [ransac.gen_rnd_indices(100, 6) for _ in range(5)]
    after = random.random()
    random.seed(7)
    b = [pnp_ref.gen_rnd_indices(100, 6) for _ in range(5)]
    assert a == b and random.random() == after


def test_ransac_robust_surface(ctx):
    # The reference's unnormalised 6-point DLT is poorly conditioned on noisy data
    # (s11/s12 ~ 4 here), so minimal-sample poses are rough and consensus sets small; the
    # drop-in must reproduce the oracle exactly, not an idealised estimator.
    X, _, y, _, _, truth = synth.pnp_scene(120, 0.2, seed=5)
    D = np.stack([y, X], axis=1)            # (N, 2, 3): D[:,0] = y, D[:,1] = x
    thr = (8.0 / 800) ** 2
    random.seed(0)
    R_est, t_est, C_est = ransac.ransac_robust(D, D, 200, thr, 6)
    Ro, to, imo, iho, besto, _ = pnp_ref.ransac_pnp(y, X, y, X, 200, thr, 6,
                                                    rng=random.Random(0))
    assert len(R_est) == 1 and R_est[0].shape == (3, 3)
    assert np.allclose(R_est[0] @ R_est[0].T, np.eye(3), atol=1e-9)
    np.testing.assert_allclose(R_est[0], Ro, atol=1e-6)
    np.testing.assert_allclose(t_est[0], to, rtol=1e-6, atol=1e-6)
    assert np.array_equal(C_est[0][0], D[imo]) and np.array_equal(C_est[0][1], D[iho])
    with pytest.raises(ValueError, match="Not implemented yet"):
        ransac.ransac_robust(D, D, 10, 1e-5, 4)
    with pytest.raises(ValueError, match="No PnP algorithm"):
        ransac.ransac_robust(D, D, 10, 1e-5, 5)


def test_ransac_robust_p3p_branch_equals_oracle(ctx):
    """The n = 3 branch (ransac.py:81-82, 91-111): P3P poses per trial, each scored on D_med,
    strict ">" over (trial, pose).  Parity unpinned (the reference raises at ransac.py:77 and
    its p3p is OpenCV): against the oracle restatement at r = 400 on the CPython stream --
    winner trial and pose, every per-pose count, both consensus sets, R, t -- and the stream
    advanced as gen_rnd_indices would."""
    X, _, y, Rt, tt, truth = synth.pnp_scene(300, 0.30, seed=8)
    thr = (2.0 / 800.0) ** 2
    r = 400
    rng_g, rng_o = random.Random(0), random.Random(0)
    R, t, im, ih, best, cnt = ransac.ransac_pnp(X, y, X, y, r, thr, 3, rng=rng_g)
    Ro, to, imo, iho, besto, poseo, counts = pnp_ref.ransac_pnp_p3p(y, X, y, X, r, thr,
                                                                    rng=rng_o, trace=True)
    assert best == besto and cnt == counts[besto, poseo]
    assert np.array_equal(im, imo) and np.array_equal(ih, iho)
    np.testing.assert_allclose(R, Ro, atol=1e-9)
    np.testing.assert_allclose(t, to, rtol=1e-9, atol=1e-9)
    assert rng_g.getstate() == rng_o.getstate()
    assert truth[im].mean() > 0.95
    np.testing.assert_allclose(R, Rt, atol=2e-2)
    # the drop-in surface: lists as ransac.py:109-113 builds them
    D = np.stack([y, X], axis=1)
    random.seed(0)
    R_est, t_est, C_est = ransac.ransac_robust(D, D, r, thr, 3)
    np.testing.assert_allclose(R_est[0], Ro, atol=1e-9)
    assert np.array_equal(C_est[0][0], D[imo]) and np.array_equal(C_est[0][1], D[iho])


def test_ransac_robust_p3p_noisy_near_planar_keeps_depths_positive(ctx):
    """on a noisy near-planar scene the mirrored-depth twin of the true pose (a turn
    about the plane's normal, the scene behind the camera) reprojects almost like it and can
    out-count it by a few points; the winner must still put every inlier in front of the
    camera (OpenCV's p3p, the reference's, never returns a mirrored pose).  GPU = oracle."""
    from tsbb15_amd import synth as sy
    for seed in range(6):
        rs = np.random.RandomState(100 + seed)
        m = 200
        X = np.column_stack([rs.uniform(-1.0, 1.0, m), rs.uniform(-1.0, 1.0, m),
                             6.0 + rs.normal(0.0, 0.01, m)])   # a plane 6 units ahead
        R0, t0 = sy.rot_y(0.15), np.array([0.1, -0.05, 0.3])
        P = (R0 @ X.T).T + t0
        y = np.column_stack([P[:, 0] / P[:, 2], P[:, 1] / P[:, 2], np.ones(m)])
        y[:, :2] += rs.normal(0.0, 1.5 / 800.0, (m, 2))          # ~1.5 px of noise
        out = rs.permutation(m)[:40]
        y[out, :2] = rs.uniform(-0.4, 0.4, (40, 2))
        thr = (3.0 / 800.0) ** 2
        rg, ro = random.Random(seed), random.Random(seed)
        R, t, im, ih, best, cnt = ransac.ransac_pnp(X, y, X, y, 300, thr, 3, rng=rg)
        Ro, to, imo, iho, besto, poseo, _ = pnp_ref.ransac_pnp_p3p(y, X, y, X, 300, thr, rng=ro)
        assert best == besto and np.array_equal(im, imo)
        z = (np.asarray(R) @ X[im].T).T[:, 2] + np.asarray(t)[2]
        assert len(im) > 100 and (z > 0).all(), (seed, len(im), z.min())


def test_ransac_robust_p3p_known_answers_badino2(ctx):
    """Noise-free BAdino2 views (negative-scale cameras: the mirrored-depth P3P twin carries
    the pose): the winner is the reference's camera_resectioning pose and every point agrees."""
    z = golden("dino_pnp_kat.npz")
    for v in (3, 17, 30):
        X, _, y = _view(z, v)
        D = np.stack([y, X], axis=1)
        random.seed(v)
        R_est, t_est, C_est = ransac.ransac_robust(D, D, 50, 1e-10, 3)
        np.testing.assert_allclose(R_est[0], z["R"][v], atol=1e-6)
        np.testing.assert_allclose(t_est[0], z["t"][v], rtol=1e-6, atol=1e-6)
        assert len(C_est[0][0]) == len(X)


def test_p3p_philox_sampler(ctx):
    X, _, y, Rt, tt, truth = synth.pnp_scene(500, 0.30, seed=3)
    thr = (1.5 / 800.0) ** 2
    R, t, im, ih, best, cnt = ransac.ransac_pnp(X, y, X, y, 20_000, thr, 3, sampler="philox",
                                                seed=4)
    assert np.array_equal(im, np.flatnonzero(thr >= pnp_ref.pose_errors(R, t, X, y)))
    assert cnt == len(im) and truth[im].mean() > 0.99
    np.testing.assert_allclose(R, Rt, atol=5e-3)


def test_full_size_c3_properties(ctx):
    """C3: M = 500 points, 30 % outliers, 50 000 hypotheses, Philox sampler."""
    X, _, y, Rt, tt, truth = synth.pnp_scene(500, 0.30, seed=3)
    thr = (1.5 / 800.0) ** 2
    R, t, im, ih, best, cnt = ransac.ransac_pnp(X, y, X, y, 50_000, thr, 6, sampler="philox",
                                                seed=11)
    e = pnp_ref.pose_errors(R, t, X, y)
    assert np.array_equal(im, np.flatnonzero(thr >= e))
    assert cnt == len(im)
    assert truth[im].mean() > 0.99
    np.testing.assert_allclose(R, Rt, atol=5e-3)


def test_solvepnpransac_surface_badino2(ctx):
    z = golden("dino_pnp_kat.npz")
    v = 7
    X, uv, _ = _view(z, v)
    ok, rvec, tvec, inliers = cv.solvePnPRansac(X, uv, z["K"][v], np.zeros((4, 1)),
                                                useExtrinsicGuess=True)
    assert ok and rvec.shape == (3, 1) and tvec.shape == (3, 1)
    assert inliers.dtype == np.int32 and inliers.shape == (len(X), 1)
    R, _ = cv.Rodrigues(rvec)
    np.testing.assert_allclose(R, z["R"][v], atol=1e-8)
    np.testing.assert_allclose(tvec[:, 0], z["t"][v], atol=1e-8)


def _aniso_scene(seed=4):
    """Anisotropic, skewed camera (fx 800, fy 1200, skew 0.5): 100 exact correspondences, 10
    moved 7 px along u, 10 moved 9 px along v, 20 gross outliers (>= 60 px)."""
    rs = np.random.RandomState(seed)
    K = np.array([[800.0, 0.5, 640.0], [0.0, 1200.0, 480.0], [0.0, 0.0, 1.0]])
    R, _ = cv.Rodrigues(np.array([0.1, -0.2, 0.05]))
    t = np.array([0.2, -0.1, 6.0])
    X = rs.uniform(-2, 2, (140, 3))
    uv = cv.project_points(X, cv.Rodrigues(R)[0], t, K)
    uv[100:110, 0] += 7.0
    uv[110:120, 1] += 9.0
    uv[120:] += rs.choice([-1, 1], (20, 2)) * rs.uniform(60, 200, (20, 2))
    return X, uv, K, R, t


def test_solvepnpransac_pixel_threshold_through_K(ctx):
    """The consensus test is |K pi(R x + t) - uv| <= reprojectionError in PIXELS: with
    fx != fy a 7 px offset along u is an inlier and a 9 px offset along v is not (the old
    normalised test with f = sqrt(fx fy) decided both the other way)."""
    X, uv, K, Rt, tt = _aniso_scene()
    ok, rvec, tvec, inl = cv.solvePnPRansac(X, uv, K, np.zeros((4, 1)), iterationsCount=500,
                                            confidence=0.999999)
    assert ok
    inl = inl[:, 0]
    # exactly the pixel test under the RANSAC pose (before refinement)
    rr = cv.last_ransac
    e = np.linalg.norm(cv.project_points(X, cv.Rodrigues(rr["R"])[0], rr["t"], K) - uv, axis=1)
    np.testing.assert_array_equal(inl, np.flatnonzero(e <= 8.0))
    # the winner holds at least the true pose's 110 (a 5-point EPnP pose fitted through some
    # of the 7 px points may trade a few of those for 9 px ones and count more), every exact
    # point and no gross outlier
    assert len(inl) >= 110 and set(range(100)) <= set(inl) and inl.max() < 120, inl
    # LM refinement on the consensus set: no worse than the RANSAC pose, near the truth
    R, _ = cv.Rodrigues(rvec)
    e2 = np.linalg.norm(cv.project_points(X[inl], rvec, tvec[:, 0], K) - uv[inl], axis=1)
    assert (e2 ** 2).sum() <= (e[inl] ** 2).sum() * (1 + 1e-12)
    np.testing.assert_allclose(R, Rt, atol=5e-3)


def test_solvepnpransac_adaptive_iterations_and_determinism(ctx):
    X, uv, K, _, _ = _aniso_scene()
    # noise-free, no outliers: the first model has outlier ratio 0 -> RANSACUpdateNumIters = 0
    ok, *_ = cv.solvePnPRansac(X[:100], uv[:100], K, None, iterationsCount=1000)
    assert ok and cv.last_ransac["iterations"] == 1
    # confidence 1: the budget never shrinks below iterationsCount while outliers remain
    ok, *_ = cv.solvePnPRansac(X, uv, K, None, iterationsCount=300, confidence=1.0)
    assert ok and cv.last_ransac["iterations"] == 300
    used, best = [], []
    for conf in (0.5, 0.99, 0.9999):
        ok, _, _, inl = cv.solvePnPRansac(X, uv, K, None, iterationsCount=1000, confidence=conf)
        used.append(cv.last_ransac["iterations"])
        best.append((cv.last_ransac["best_index"], len(inl)))
    assert used == sorted(used) and used[-1] < 1000, used
    # OpenCV's budget at the winner's outlier ratio (EPnP kernel, m = 5):
    # log(1 - p) / log(1 - (1 - ep)^5); the loop stops at that budget, or right after the
    # winner when it came later
    ep = 1 - best[1][1] / 140
    bound = int(np.ceil(np.log(0.01) / np.log(1 - (1 - ep) ** 5))) + 1
    assert used[1] <= max(bound, best[1][0] + 1), (used, best, bound)
    # equal inputs, equal outputs, whatever ran in between
    a = cv.solvePnPRansac(X, uv, K, None)
    cv.solvePnPRansac(X[::-1].copy(), uv[::-1].copy(), K, None, iterationsCount=37)
    b = cv.solvePnPRansac(X, uv, K, None)
    for u, v in zip(a[1:], b[1:]):
        np.testing.assert_array_equal(u, v)


def test_solvepnpransac_rejects_bad_input(ctx):
    X, uv, K, _, _ = _aniso_scene()
    with pytest.raises(ValueError, match="at least 4"):
        cv.solvePnPRansac(X[:3], uv[:3], K, None)
    with pytest.raises(ValueError, match="flags"):
        cv.solvePnPRansac(X, uv, K, None, flags=7)     # e.g. SOLVEPNP_SQPNP: not provided
    with pytest.raises(ValueError):
        cv.solvePnPRansac(X, uv, K, np.array([0.1, 0, 0, 0]))
    Kb = K.copy()
    Kb[1, 0] = 1.0
    with pytest.raises(ValueError, match="upper triangular"):
        cv.solvePnPRansac(X, uv, Kb, None)
    # nothing agrees: False, like OpenCV
    rs = np.random.RandomState(0)
    ok, r, t, inl = cv.solvePnPRansac(X[:12], rs.uniform(0, 2000, (12, 2)), K, None,
                                      reprojectionError=1e-6)
    assert not ok and inl is None


def test_p3p_solvepnp_iterative(ctx):
    """pnp.p3p = cv.solvePnP(SOLVEPNP_ITERATIVE) over all points (pnp.py:7-10): known answers
    on noise-free BAdino2 views, and on a noisy view the LM refinement never raises the pixel
    reprojection error of its DLT start and lands near the true pose.  OpenCV parity unpinned."""
    z = golden("dino_pnp_kat.npz")
    for v in (1, 20):
        X, uv, _ = _view(z, v)
        R, t = pnp.p3p(X, uv, z["K"][v])
        np.testing.assert_allclose(R, z["R"][v], atol=1e-7)
        np.testing.assert_allclose(t, z["t"][v], rtol=1e-6, atol=1e-7)
        ok, rv, tv = cv.solvePnP(X, uv, z["K"][v], np.zeros((4, 1)))
        assert ok and rv.shape == (3, 1) and tv.shape == (3, 1)
    # noisy pixels: refinement against the DLT start
    X, uv, _ = _view(z, 5)
    K = z["K"][5]
    rs = np.random.RandomState(3)
    uvn = uv + rs.normal(0.0, 0.7, uv.shape)
    ok, rv, tv = cv.solvePnP(X, uvn, K, None)
    assert ok
    err = np.sum((cv.project_points(X, rv, tv, K) - uvn) ** 2)
    c = X.mean(axis=0)
    s = np.sqrt(np.mean(np.sum((X - c) ** 2, axis=1)))
    y = (np.linalg.inv(K) @ np.vstack([uvn.T, np.ones((1, len(uvn)))])).T
    Rd, td = pnp.pnp_minimize((X - c) / s, y, len(X))
    rd, _ = cv.Rodrigues(Rd)
    err_dlt = np.sum((cv.project_points(X, rd, s * td - Rd @ c, K) - uvn) ** 2)
    err_true = np.sum((cv.project_points(X, cv.Rodrigues(z["R"][5])[0], z["t"][5], K) - uvn) ** 2)
    assert err <= err_dlt * (1 + 1e-12)
    assert err <= err_true * (1 + 1e-9)  # the least-squares pose fits the noisy pixels best
    R, _ = cv.Rodrigues(rv)
    assert np.linalg.norm(R - z["R"][5]) < 1e-2
    # the guess path starts from the given pose; too few points without a guess raises
    ok, rv2, tv2 = cv.solvePnP(X, uvn, K, None, rv, tv, useExtrinsicGuess=True)
    assert ok and np.allclose(rv2, rv, atol=1e-6) and np.allclose(tv2, tv, atol=1e-6)
    with pytest.raises(ValueError):
        cv.solvePnP(X[:3], uvn[:3], K, None)


def test_minimal_pnp_known_answers_badino2(ctx):
    """The OpenCV kernels on noise-free BAdino2 views (poses from the reference's
    camera_resectioning): EPnP on 5 points and on all of a view's points, P3P on 4 (three
    solve, the fourth chooses), through cv.solvePnP(flags) and through cv.solvePnPRansac's
    direct path (as many correspondences as the kernel's sample: every point an inlier)."""
    z = golden("dino_pnp_kat.npz")
    K0 = None
    for v in (1, 7, 20, 33):
        X, uv, _ = _view(z, v)
        K = z["K"][v]
        rs = np.random.RandomState(v)
        for trial in range(3):
            s = rs.choice(len(X), 5, replace=False)
            ok, rv, tv = cv.solvePnP(X[s], uv[s], K, None, flags=cv.SOLVEPNP_EPNP)
            assert ok
            np.testing.assert_allclose(cv.Rodrigues(rv)[0], z["R"][v], atol=1e-6)
            np.testing.assert_allclose(tv[:, 0], z["t"][v], rtol=1e-6, atol=1e-6)
            ok, rv, tv, inl = cv.solvePnPRansac(X[s], uv[s], K, None)
            assert ok and np.array_equal(inl[:, 0], np.arange(5))
            np.testing.assert_allclose(cv.Rodrigues(rv)[0], z["R"][v], atol=1e-6)
            s4 = s[:4]
            for call in (lambda: cv.solvePnP(X[s4], uv[s4], K, None, flags=cv.SOLVEPNP_P3P),
                         lambda: cv.solvePnPRansac(X[s4], uv[s4], K, None)[:3]):
                ok, rv, tv = call()
                assert ok
                np.testing.assert_allclose(cv.Rodrigues(rv)[0], z["R"][v], atol=1e-6)
                np.testing.assert_allclose(tv[:, 0], z["t"][v], rtol=1e-6, atol=1e-6)
        ok, rv, tv = cv.solvePnP(X, uv, K, None, flags=cv.SOLVEPNP_EPNP)
        np.testing.assert_allclose(cv.Rodrigues(rv)[0], z["R"][v], atol=1e-8)
        K0 = K
    with pytest.raises(ValueError):
        cv.solvePnP(X[:5], uv[:5], K0, None, flags=cv.SOLVEPNP_P3P)   # P3P takes exactly 4


def test_minimal_poses_are_front_facing_on_positive_depth_data(ctx):
    """OpenCV's EPnP / P3P return front-facing poses only.  The kernels also score the mirrored
    solution (every depth negated: BAdino2's negative-scale cameras need it), which the pixel
    error x / z alone cannot tell apart on near-degenerate samples; a mirrored pose must be
    clearly better to win (pnp_minimal.h kMirrorWins).  On ordinary positive-depth scenes with
    noisy pixels every returned pose puts all its inliers at z > 0."""
    rs = np.random.RandomState(11)
    K = np.array([[700.0, 0.0, 640.0], [0.0, 700.0, 480.0], [0.0, 0.0, 1.0]])
    for trial in range(40):
        R, _ = cv.Rodrigues(rs.normal(0, 0.3, 3))
        t = np.array([rs.uniform(-0.5, 0.5), rs.uniform(-0.5, 0.5), rs.uniform(4, 8)])
        X = rs.uniform(-1.5, 1.5, (60, 3))
        uv = cv.project_points(X, cv.Rodrigues(R)[0], t, K) + rs.normal(0, 0.8, (60, 2))
        s = rs.choice(60, 5, replace=False)
        for flags, sel in ((cv.SOLVEPNP_EPNP, s), (cv.SOLVEPNP_P3P, s[:4]),
                           (cv.SOLVEPNP_EPNP, np.arange(60))):
            ok, rv, tv = cv.solvePnP(X[sel], uv[sel], K, None, flags=flags)
            if not ok:
                continue
            Rm, _ = cv.Rodrigues(rv)
            z = (X[sel] @ Rm.T + tv[:, 0])[:, 2]
            assert np.all(z > 0), (trial, flags, z)
        ok, rv, tv, inl = cv.solvePnPRansac(X, uv, K, None, iterationsCount=200,
                                            flags=cv.SOLVEPNP_EPNP)
        assert ok
        Rm, _ = cv.Rodrigues(rv)
        assert np.all((X[inl[:, 0]] @ Rm.T + tv[:, 0])[:, 2] > 0), trial


def test_solvepnpransac_kernels_and_guess(ctx):
    """RANSAC with the EPnP (5-point) and P3P (4-point, flags=SOLVEPNP_P3P) kernels on the
    anisotropic scene: each keeps every exact point and no gross outlier; the extrinsic guess (useExtrinsicGuess) is
    scored first, so a correct guess wins at hypothesis 0."""
    X, uv, K, Rt, tt = _aniso_scene()
    for flags in (cv.SOLVEPNP_ITERATIVE, cv.SOLVEPNP_EPNP, cv.SOLVEPNP_P3P):
        ok, rv, tv, inl = cv.solvePnPRansac(X, uv, K, None, iterationsCount=2000,
                                            confidence=0.999999, flags=flags)
        inl = inl[:, 0]
        assert ok and len(inl) >= 110 and set(range(100)) <= set(inl) and inl.max() < 120, flags
        np.testing.assert_allclose(cv.Rodrigues(rv)[0], Rt, atol=5e-3)
    # exact points and gross outliers only: the true pose's 100 is the maximum consensus, and a
    # later hypothesis needs strictly more to replace hypothesis 0
    sel = np.r_[0:100, 120:140]
    rg, _ = cv.Rodrigues(Rt)
    ok, rv, tv, inl = cv.solvePnPRansac(X[sel], uv[sel], K, None, rg, tt.reshape(3, 1),
                                        useExtrinsicGuess=True, iterationsCount=50)
    assert ok and cv.last_ransac["best_index"] == 0
    assert np.array_equal(inl[:, 0], np.arange(100))
    # a wrong guess is just one more hypothesis
    ok, rv, tv, inl = cv.solvePnPRansac(X[sel], uv[sel], K, None, -rg, tt.reshape(3, 1) + 1.0,
                                        useExtrinsicGuess=True, iterationsCount=200)
    assert ok and cv.last_ransac["best_index"] > 0 and np.array_equal(inl[:, 0], np.arange(100))


def test_c3_full_size_exact_stream_equals_oracle_fixture(ctx):
    """C3 at full size (500 points, 50 000 trials) on random.seed(0)'s CPython stream: the
    winner, its consensus count, both consensus sets, R, t and the advanced stream state equal
    tests/golden/full_c3.npz (the oracle restatement of the intended ransac.py:37-113,
    make_golden_c3.py; the reference's own loop raises at ransac.py:77, so this is the pinned
    oracle, not a run of the reference)."""
    z = golden("full_c3.npz")
    rng = random.Random(0)
    R, t, im, ih, best, cnt = ransac.ransac_pnp(z["X"], z["y"], z["X"], z["y"], int(z["r"]),
                                                float(z["thresh"]), 6, rng=rng)
    assert best == int(z["best"])
    assert cnt == int(z["counts"].max()) == len(z["inl_med"])
    assert np.array_equal(im, z["inl_med"]) and np.array_equal(ih, z["inl_high"])
    np.testing.assert_allclose(R, z["R"], atol=1e-6)
    np.testing.assert_allclose(t, z["t"], rtol=1e-6, atol=1e-6)
    st = rng.getstate()
    assert int(st[1][624]) == int(z["py_pos_out"])
    assert np.array_equal(np.array(st[1][:624], np.uint32), z["py_key_out"])


def test_refine_lm_gpu_reaches_the_least_squares_pose(ctx):
    """rs_pnp_refine_lm (the SOLVEPNP_ITERATIVE refinement, one GPU workgroup) against scipy's
    MINPACK LM on the same pixel residual from the same perturbed start, on noisy BAdino2 views:
    equal final cost (1e-9 relative), equal pose (1e-6), never above the start's cost."""
    from scipy.optimize import least_squares
    z = golden("dino_pnp_kat.npz")
    rs = np.random.RandomState(11)
    for v in (2, 7, 13):
        X, uv, _ = _view(z, v)
        K = z["K"][v]
        uvn = uv + rs.normal(0.0, 1.0, uv.shape)
        r_true, _ = cv.Rodrigues(z["R"][v])
        r0 = r_true + rs.normal(0.0, 0.02, (3, 1))
        t0 = z["t"][v].reshape(3, 1) * (1.0 + rs.normal(0.0, 0.02, (3, 1)))

        def res(x):
            return (cv.project_points(X, x[:3], x[3:], K) - uvn).ravel()

        x0 = np.concatenate((r0.ravel(), t0.ravel()))
        ref = least_squares(res, x0, method="lm", xtol=1e-15, ftol=1e-15, gtol=1e-15)
        rv, tv = cv._refine_lm(X, uvn, K, r0, t0)
        c_gpu = 0.5 * float(np.sum(res(np.concatenate((rv.ravel(), tv.ravel()))) ** 2))
        assert c_gpu <= 0.5 * float(res(x0) @ res(x0))
        assert cv.last_lm["cost"] == pytest.approx(c_gpu, rel=1e-9)
        assert c_gpu == pytest.approx(ref.cost, rel=1e-9), (v, c_gpu, ref.cost)
        np.testing.assert_allclose(rv.ravel(), ref.x[:3], atol=1e-6)
        np.testing.assert_allclose(tv.ravel(), ref.x[3:], rtol=1e-6, atol=1e-6)
    with pytest.raises(ValueError):  # fewer than 3 correspondences
        _ffi_refine_short(X, uvn, K)


def _ffi_refine_short(X, uv, K):
    from tsbb15_amd import _ffi
    R, t, c = np.eye(3), np.zeros(3), np.zeros(4)
    _ffi.check(_ffi.lib().rs_pnp_refine_lm(_ffi.default_context().handle,
                                           _ffi.ptr(np.ascontiguousarray(X[:2]), _ffi.C.c_double),
                                           _ffi.ptr(np.ascontiguousarray(uv[:2]), _ffi.C.c_double),
                                           2, _ffi.ptr(np.ascontiguousarray(K), _ffi.C.c_double),
                                           _ffi.ptr(R, _ffi.C.c_double), _ffi.ptr(t, _ffi.C.c_double),
                                           20, _ffi.ptr(c, _ffi.C.c_double)))


def test_consensus_counts_exact_at_the_threshold(ctx):
    """ransac.py:104-105 keeps a point when thresh >= e.  Points whose e lies within a few
    hundred ulps of thresh (copies of one point nudged by 1..12 ulps of its world coordinates)
    are decided by the last bits of the reference's arithmetic; the counting kernel must agree
    with it exactly (division-free test + exact guard band + reference-order re-test), for the
    pose that placed the threshold and for nearby poses."""
    import pnp_exact
    X, _, y, R, t, _ = synth.pnp_scene(64, 0.0, seed=21)
    P0 = np.concatenate([R.ravel(), t])
    picks = [3, 17, 40]
    Xb, yb = pnp_exact.boundary_cloud(X, y, P0, picks, spread=12, seed=1)
    Xa, ya = np.vstack([X, Xb]), np.vstack([y, yb])
    rs = np.random.RandomState(2)
    poses = np.array([P0] + [P0 * (1.0 + rs.normal(0, s, 12)) for s in [1e-15] * 7 + [1e-13] * 8])
    e_all = [pnp_exact.errors_exact(P, Xa, ya) for P in poses]
    straddled = 0
    for q, j in enumerate(picks):
        centre = len(X) + q * 25 + 12
        thresh = e_all[0][centre]
        ref = np.array([np.count_nonzero(thresh >= e) for e in e_all], np.int32)
        got = ransac.consensus_counts(Xa, ya, poses, thresh, ctx=ctx)
        np.testing.assert_array_equal(got, ref)
        block = e_all[0][len(X) + q * 25: len(X) + (q + 1) * 25]
        straddled += int(0 < np.count_nonzero(thresh >= block) < 25)
    assert straddled == len(picks)   # the threshold really cuts each cloud


def test_consensus_counts_threshold_sweep_equals_reference_order(ctx):
    """Every point's own e as the threshold (inclusive test), C3-like noisy scene, 16 poses."""
    import pnp_exact
    X, _, y, R, t, _ = synth.pnp_scene(48, 0.3, seed=8)
    rs = np.random.RandomState(4)
    P0 = np.concatenate([R.ravel(), t])
    poses = np.array([P0 * (1.0 + rs.normal(0, 1e-6, 12)) for _ in range(16)])
    e_all = [pnp_exact.errors_exact(P, X, y) for P in poses]
    for j in range(0, 48, 3):
        thresh = e_all[j % 16][j]
        ref = np.array([np.count_nonzero(thresh >= e) for e in e_all], np.int32)
        np.testing.assert_array_equal(ransac.consensus_counts(X, y, poses, thresh, ctx=ctx), ref)


def test_ransac_pnp_best_count_is_the_consensus_size(ctx):
    """The winner's count equals its D_med consensus set (the library fails otherwise)."""
    X, _, y, _, _, _ = synth.pnp_scene(300, 0.3, seed=12)
    thr = (1.5 / 800.0) ** 2
    for n, sampler in ((6, "philox"), (3, "philox"), (6, "exact")):
        R, t, im, ih, best, cnt = ransac.ransac_pnp(X, y, X, y, 2000, thr, n, sampler=sampler,
                                                    seed=5, rng=random.Random(3), ctx=ctx)
        assert best >= 0 and cnt == len(im)
        assert cnt == int(ransac.consensus_counts(X, y, np.concatenate([R.ravel(), t])[None],
                                                  thr, ctx=ctx)[0])


def test_dlt_minimal_samples_accuracy_against_numpy_svd(ctx):
    """400 noisy 6-point samples of the C3 scene (30 % outliers): the GPU DLT (block factor,
    three-vector inverse iteration) against the oracle's numpy SVD.  The bar is the sample's own
    conditioning floor (the reference's SVD and ours agree to ~1e-12 on R), far inside 1e-6."""
    X, _, y, _, _, _ = synth.pnp_scene(500, 0.30, seed=3)
    rs = np.random.RandomState(7)
    dr, dt = [], []
    for _ in range(400):
        s = rs.choice(500, 6, replace=False)
        R, t = pnp.pnp_minimize(X[s], y[s], 6)
        Ro, to = pnp_ref.pnp_dlt(X[s], y[s])
        if not (np.isfinite(R).all() and np.isfinite(Ro).all()):
            continue
        dr.append(np.abs(R - Ro).max())
        dt.append(np.abs(t - to).max() / np.abs(to).max())
    dr, dt = np.array(dr), np.array(dt)
    print(f"\nDLT vs numpy SVD over {len(dr)} samples: R max {dr.max():.3g} p99 "
          f"{np.percentile(dr, 99):.3g}; t rel max {dt.max():.3g} p99 {np.percentile(dt, 99):.3g}")
    assert len(dr) >= 390
    assert dr.max() < 1e-8 and dt.max() < 1e-8
