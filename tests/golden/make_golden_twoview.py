"""Generate tests/golden/twoview.npz -- two-view geometry after RANSAC -- from the reference.

Runs ONLY in the build container (the reference lives at /root/reference and never travels
to the GPU box); imports the reference exactly as make_golden.py does (import-only cv2 stub,
SURVEY.md 8(c) / A.2).  Every expected value is produced by reference code:

  * lab3.triangulate_optimal            lab3.py:382-475  (uses fmatrix_from_cameras 331-351,
                                                          fmatrix_epipoles 505-527,
                                                          triangulate_linear 477-503)
  * lab3.fmatrix_cameras                lab3.py:353-380
  * fun.camera_resectioning + specRQ    fun.py:181-188, 260-280
  * fun.getEAndK / fun.MakeHomogenous   fun.py:48-55, 91-102
  * fun.relative_camera_pose + specSVD  fun.py:190-258
  * the gold-standard tail of fun.getFFromLabCode (fun.py:336-369), driven by ``_ref_gold``
    below for given (F_RANSAC, S_RANSAC); it is cross-checked bit-exactly against the
    unmodified getFFromLabCode outputs already held in dino_c1.npz.

Usage:  python tests/golden/make_golden_twoview.py   (about 9 minutes, single-threaded BLAS)
"""
from __future__ import annotations

import os
import sys
import time

# single-threaded BLAS: dino_c1.npz was written that way, and the cross-check against it is
# bit-exact only with the same reduction order
os.environ["OPENBLAS_NUM_THREADS"] = "1"
os.environ["OMP_NUM_THREADS"] = "1"

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference, noisy_pair, _ref_loop, _save  # noqa: E402


def _ref_gold(lab3, least_squares, F_RANSAC, S_RANSAC, p1, p2):
    """fun.py:336-369 verbatim in behaviour: cameras, optimal triangulation of the inliers,
    scipy least_squares(xtol=2.22e-14, tr_solver='lsmr'), F from the refined cameras."""
    C1, C2 = lab3.fmatrix_cameras(F_RANSAC)
    a = p1[:, S_RANSAC]
    b = p2[:, S_RANSAC]
    X = np.vstack([lab3.triangulate_optimal(C1, C2, x1, x2) for x1, x2 in zip(a.T, b.T)]).T
    params = np.hstack((C1.ravel(), X.T.ravel()))
    res = least_squares(lab3.fmatrix_residuals_gs, params, xtol=2.22e-14, tr_solver='lsmr',
                        args=(a, b))
    sol = res.x
    C1g = sol[:12].reshape(3, 4)
    C2g = np.zeros((3, 4)); C2g[:3, :3] = np.eye(3)
    F_gold = lab3.fmatrix_from_cameras(C1g, C2g)
    return dict(F_gold=F_gold, C1_init=C1, X_init=X.T.copy(), C1_final=C1g,
                cost_init=0.5 * float(np.sum(lab3.fmatrix_residuals_gs(params, a, b) ** 2)),
                cost_final=float(res.cost), nfev=int(res.nfev), status=int(res.status))


def main():
    lab3, fun, ransac, correspondences = import_reference()
    from scipy.optimize import least_squares
    import scipy.io as sio
    from tsbb15_amd import synth

    out = {}
    c1 = np.load(os.path.join(HERE, "dino_c1.npz"))
    F_file = c1["F_file"]

    # ---- lab3.triangulate_optimal / fmatrix_cameras --------------------------------------
    C1, C2 = lab3.fmatrix_cameras(F_file)
    out["cam_F_file_C1"] = C1
    for tag in ("clean", "noisy"):
        p1, p2 = c1[f"{tag}_p1"], c1[f"{tag}_p2"]
        out[f"tri_{tag}_X"] = np.array([lab3.triangulate_optimal(C1, C2, p1[:, i], p2[:, i])
                                        for i in range(p1.shape[1])])
    z2 = np.load(os.path.join(HERE, "synth_c2.npz"))
    S2 = z2["S_ransac"][:300]
    Cs1, Cs2 = lab3.fmatrix_cameras(z2["F_ransac"])
    out["tri_c2_C1"] = Cs1
    out["tri_c2_idx"] = S2
    out["tri_c2_X"] = np.array([lab3.triangulate_optimal(Cs1, Cs2, z2["p1"][:, i], z2["p2"][:, i])
                                for i in S2])

    # ---- camera_resectioning on the noisy dino cameras (imgdata/dino_Ps.mat) ------------
    Pn = np.asarray(sio.loadmat("imgdata/dino_Ps.mat")["P"].tolist())[0]   # (36,3,4)
    Kn, Rn, tn = zip(*[fun.camera_resectioning(P) for P in Pn])
    out.update(resect_P=Pn, resect_K=np.array(Kn), resect_R=np.array(Rn), resect_t=np.array(tn))

    # ---- getEAndK + relative_camera_pose over BAdino2 pairs -----------------------------
    m = sio.loadmat("BAdino2.mat")
    C = np.asarray(m["newPs"].tolist())                       # (1,36,3,4) as fun.py:85-87
    corr = correspondences.Correspondences()
    pairs, Fs, Es, y1s, y2s, Rs, ts, found = [], [], [], [], [], [], [], []
    for i in range(36):
        for j in range(i + 1, 36):
            a, b = corr.getCorrByIndices(i, j)
            if a.shape[0] < 8:
                continue
            F = lab3.fmatrix_stls(a.T, b.T)                   # least-squares F of the pair
            E, K = fun.getEAndK(C, F)
            yh1, yh2 = fun.MakeHomogenous(K, a), fun.MakeHomogenous(K, b)
            r = fun.relative_camera_pose(E, yh1[0, :2].T, yh2[0, :2].T)
            pairs.append((i, j)); Fs.append(F); Es.append(E)
            y1s.append(yh1[0, :2]); y2s.append(yh2[0, :2])
            if r is None:
                found.append(0); Rs.append(np.full((3, 3), np.nan)); ts.append(np.full(3, np.nan))
            else:
                found.append(1); Rs.append(r[0]); ts.append(r[1])
            if len(pairs) == 64:
                break
        if len(pairs) == 64:
            break
    out.update(pose_pairs=np.array(pairs), pose_F=np.array(Fs), pose_E=np.array(Es),
               pose_K=K, pose_y1=np.array(y1s), pose_y2=np.array(y2s), pose_R=np.array(Rs),
               pose_t=np.array(ts), pose_found=np.array(found))
    print(f"pose: {len(pairs)} pairs, {sum(found)} with a pose")

    # ---- gold standard (fun.py:336-369) --------------------------------------------------
    for tag in ("clean", "noisy"):
        p1, p2 = c1[f"{tag}_p1"], c1[f"{tag}_p2"]
        t0 = time.time()
        g = _ref_gold(lab3, least_squares, c1[f"{tag}_full_F_ransac"],
                      c1[f"{tag}_full_S_ransac"], p1, p2)
        dt = time.time() - t0
        assert np.array_equal(g["F_gold"], c1[f"{tag}_full_F_gold"]), \
            "gold-standard harness != unmodified getFFromLabCode"
        for k, v in g.items():
            out[f"gs_{tag}_{k}"] = v
        out[f"gs_{tag}_seconds"] = dt
        print(f"gold {tag}: cost {g['cost_init']:.6g} -> {g['cost_final']:.6g} "
              f"nfev {g['nfev']} ({dt:.1f}s)")
    # a synthetic pair (the smoke() scene): reference loop, then the gold standard
    p1, p2, _ = synth.two_view(300, 0.3, seed=11)
    np.random.seed(0)
    lp = _ref_loop(lab3, p1, p2, 500)
    t0 = time.time()
    g = _ref_gold(lab3, least_squares, lp["F_ransac"], lp["S_ransac"], p1, p2)
    print(f"gold synth300: cost {g['cost_init']:.6g} -> {g['cost_final']:.6g} nfev {g['nfev']} "
          f"({time.time() - t0:.1f}s)")
    out.update(gs_s300_p1=p1, gs_s300_p2=p2, gs_s300_F_ransac=lp["F_ransac"],
               gs_s300_S_ransac=lp["S_ransac"])
    for k, v in g.items():
        out[f"gs_s300_{k}"] = v
    _save("twoview.npz", **out)


if __name__ == "__main__":
    main()
