"""Generate tests/golden/tables.npz -- the per-view SfM steps around PnP -- from the reference.

Runs ONLY in the build container (imports the reference as make_golden.py does, with the
import-only cv2 stub).  It replays main.py's INIT1-3 on the BAdino2 data with the reference's
own functions (fun.getEAndK, fun.relative_camera_pose, Tables.addView,
Tables.triangulateAndAddPoints), then the first iteration of main.py's loop (i = 1):

  * Tables.BundleAdjustment2 (tables.py:254-333): scipy's least_squares is wrapped so the
    reference's own objective EpsilonBA (tables.py:264-293) is evaluated at x0 and at a
    perturbed x, and its jac_sparsity (Tables.sparsity_mask, tables.py:339-372) recorded;
    then the real least_squares call runs (trf, x_scale='jac', ftol=1e-4) and its result
    is kept.
  * Tables.addNewView (tables.py:104-158): the O(N M) 2D<->3D matching loop (tables.py:
    116-135).  OpenCV is absent, so cv.solvePnPRansac / cv.Rodrigues are replaced by a
    recorder that returns a fixed stand-in pose (the true BAdino2 pose of the view, mapped into
    the reconstruction frame) and accepts every correspondence; the matching result (the D
    and A sets) is the reference's.
  * Tables.addNewPoints (tables.py:161-175): fun.getEFromCameras (fun.py:12-21), the epipolar
    gate |y1^T E y2| < 0.1, lab3.triangulate_optimal of the accepted pairs.

Usage:  python tests/golden/make_golden_tables.py
"""
from __future__ import annotations

import os
import sys

os.environ["OPENBLAS_NUM_THREADS"] = "1"
os.environ["OMP_NUM_THREADS"] = "1"

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference, _save  # noqa: E402


def main():
    lab3, fun, ransac, correspondences = import_reference()
    from make_golden import noisy_pair
    corr = correspondences.Correspondences()
    out = {}
    for tag, get in (("clean", corr.getCorrByIndices), ("noisy", noisy_pair)):
        for k, v in run(lab3, fun, get).items():
            out[f"{tag}_{k}"] = v
    _save("tables.npz", **out)


def run(lab3, fun, get_pair):
    import scipy.io as sio
    import tables
    from help_classes import CameraPose

    out = {}
    m = sio.loadmat("BAdino2.mat")
    C = np.asarray(m["newPs"].tolist())
    F = np.load("Fmatrix.npy")

    T = tables.Tables.__new__(tables.Tables)           # skip __init__ (fun.getImages, cv2)
    T.T_obs = np.array([], dtype="object")
    T.T_views = np.array([], dtype="object")
    T.T_points = np.array([], dtype="object")
    T.images = np.zeros((36, 1200, 1200, 3), dtype=np.int64)   # colours are not compared
    # ---- INIT1-3 (main.py:25-78) ---------------------------------------------------------
    y1, y2 = get_pair(0, 1)
    E, K = fun.getEAndK(C, F)
    T.K = K
    y1_hom, y2_hom = fun.MakeHomogenous(K, y1), fun.MakeHomogenous(K, y2)
    R, t = fun.relative_camera_pose(E, y1_hom[0, :2].T, y2_hom[0, :2].T)
    C1, C2 = CameraPose(), CameraPose(R, t)
    v1, v2 = T.addView(0, C1), T.addView(1, C2)
    T.triangulateAndAddPoints(v1, v2, C1, C2, y1_hom, y2_hom)
    out["init_points"] = np.array([p.point for p in T.T_points])
    out["init_R"], out["init_t"], out["K"] = R, t, K

    # ---- BundleAdjustment2 (tables.py:254-333) through a recording least_squares -------
    rec = {}
    real_ls = tables.least_squares

    def recording_ls(fn, x0, args=(), **kw):
        rec["x0"] = x0.copy()
        rec["r0"] = fn(x0, *args)
        rng = np.random.RandomState(7)
        x1 = x0 + 1e-3 * rng.randn(x0.size)
        rec["x1"], rec["r1"] = x1, fn(x1, *args)
        A = kw["jac_sparsity"]
        rec["mask_rows"], rec["mask_cols"] = A.nonzero()
        rec["mask_shape"] = np.array(A.shape)
        kw = dict(kw, verbose=0)
        res = real_ls(fn, x0, args=args, **kw)
        rec["x_final"], rec["cost_final"], rec["nfev"] = res.x, res.cost, res.nfev
        return res

    tables.least_squares = recording_ls
    obs_view = np.array([o.view_index for o in T.T_obs])
    obs_point = np.array([o.point_3D_index for o in T.T_obs])
    obs_coords = np.array([o.image_coordinates for o in T.T_obs])
    try:
        T.BundleAdjustment2()
    finally:
        tables.least_squares = real_ls
    for k, v in rec.items():
        out[f"ba_{k}"] = np.asarray(v)
    out.update(ba_obs_view=obs_view, ba_obs_point=obs_point, ba_obs_coords=obs_coords,
               ba_n_views=len(T.T_views), ba_n_points=len(T.T_points))
    print(f"BA: {len(T.T_obs)} observations, cost -> {rec['cost_final']:.6g}, "
          f"nfev {rec['nfev']}")

    # ---- addNewView for view 2 (tables.py:104-158) --------------------------------------
    z = np.load(os.path.join(HERE, "dino_pnp_kat.npz"))
    Rw, tw = z["R"], z["t"]
    # stand-in PnP pose: the true view-2 pose in the reconstruction frame of views 0/1
    # (rotation R2 R0^T; translation mirrored and scaled like the relative pose's unit t)
    R02 = Rw[2] @ Rw[0].T
    t01 = tw[1] - (Rw[1] @ Rw[0].T) @ tw[0]
    s = np.linalg.norm(t01)
    t02 = -(tw[2] - R02 @ tw[0]) / s
    captured = {}

    def fake_pnp(D3, Dimg, Kc, dist, useExtrinsicGuess=True):
        captured["D3"], captured["Dimg"] = np.array(D3), np.array(Dimg)
        return True, np.zeros((3, 1)), t02.reshape(3, 1), np.arange(len(D3)).reshape(-1, 1)

    def fake_rodrigues(r, dst=None):
        return R02.copy(), None

    tables.cv.solvePnPRansac = fake_pnp
    tables.cv.Rodrigues = fake_rodrigues
    yp2, yp3 = get_pair(1, 2)
    yp2_hom, yp3_hom = fun.MakeHomogenous(K, yp2), fun.MakeHomogenous(K, yp3)
    last = T.T_views[len(T.T_views) - 1]
    out["match_obs_coords"] = np.array([T.T_obs[v].image_coordinates for v in last.observations_index])
    out["match_obs_point"] = np.array([T.T_obs[v].point_3D_index for v in last.observations_index])
    out["match_queries"] = yp2_hom
    out["match_y1"], out["match_y2"], out["match_y2_hom"] = yp2, yp3, yp3_hom
    A_y1, A_y2 = T.addNewView(K, 2, yp2_hom, yp3_hom, yp2, yp3)
    out.update(match_D3=captured["D3"], match_Dimg=captured["Dimg"], match_A_y1=A_y1,
               match_A_y2=A_y2, pnp_R=R02, pnp_t=t02)
    print(f"addNewView: {len(yp2)} putative, {len(captured['D3'])} matched, {len(A_y1)} new")

    # ---- addNewPoints (tables.py:161-175) ------------------------------------------------
    n0 = len(T.T_points)
    # plus 8 mismatched putative pairs (y2 rolled) and 4 far-off ones, so the epipolar gate
    # (loose in C-normalised units) has something to reject
    A_y1 = np.vstack([A_y1, yp2[:8], yp2[:4]])
    A_y2 = np.vstack([A_y2, np.roll(yp3[:8], 3, axis=0), yp3[:4] + [[4000.0, -3000.0]]])
    A_y1_hom, A_y2_hom = fun.MakeHomogenous(K, A_y1), fun.MakeHomogenous(K, A_y2)
    Cv1, Cv2 = T.T_views[1].camera_pose, T.T_views[2].camera_pose
    E12 = fun.getEFromCameras(Cv1, Cv2)
    added = T.addNewPoints(A_y1_hom, A_y2_hom, 1, 2)
    gate = np.array([abs(A_y1_hom[i].T @ E12 @ A_y2_hom[i]) < 0.1 for i in range(len(A_y1_hom))])
    out.update(new_y1_hom=A_y1_hom, new_y2_hom=A_y2_hom, new_E=E12, new_gate=gate,
               new_X=np.array([p.point for p in T.T_points[n0:]]).reshape(-1, 3),
               new_C1=Cv1.GetCameraMatrix(), new_C2=Cv2.GetCameraMatrix(), new_added=added)
    print(f"addNewPoints: {added} of {len(A_y1_hom)} pass the gate")
    return out


if __name__ == "__main__":
    main()
