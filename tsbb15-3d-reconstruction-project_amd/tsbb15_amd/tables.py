"""GPU drop-ins for the per-view SfM steps around PnP (tables.py).

Array-level functions (HIP kernels of tables.hip):

  * ``match_observations``  the 2D<->3D matching loop of Tables.addNewView (tables.py:116-135)
  * ``getEFromCameras``     fun.getEFromCameras (fun.py:12-21)
  * ``add_new_points``      the arithmetic of Tables.addNewPoints (tables.py:161-175): epipolar
                            gate |y1^T E y2| < 0.1 and optimal triangulation of the accepted
  * ``ba_residuals``        EpsilonBA of Tables.BundleAdjustment2 (tables.py:264-293)
  * ``ba_jacobian``         its Jacobian blocks (the nonzeros of tables.py:339-372)

Table-level replacements for the reference's methods (they take a reference ``Tables``
object -- anything with T_obs / T_views / T_points, addView / addPoint / addObs -- run the
arithmetic above on the GPU and do the same bookkeeping in the same order):

  * ``add_new_view(T, K, img_index, y1_hom, y2_hom, y1, y2)``      Tables.addNewView
  * ``add_new_points_table(T, A_y1_hom, A_y2_hom, v1, v2)``       Tables.addNewPoints
"""
from __future__ import annotations

import numpy as np

from . import _ffi

_d = _ffi.C.c_double
MATCH_TOL = 1e-4     # tables.py:125
EPIPOLAR_GATE = 0.1  # tables.py:168


def _ctx(ctx):
    return (ctx or _ffi.default_context()).handle


def _pose(C):
    """A CameraPose (R, t) or a (3, 4) matrix -> contiguous (3, 4) [R | t]."""
    if hasattr(C, "R"):
        M = np.zeros((3, 4))
        M[:, :3] = C.R
        M[:, 3] = np.asarray(C.t).ravel()
        return M
    M = _ffi.f64c(C)
    if M.shape != (3, 4):
        raise ValueError('camera must be (3, 4) or a CameraPose')
    return M


def match_observations(obs_coords, obs_point, queries, tol=MATCH_TOL, ctx=None):
    obs = _ffi.f64c(obs_coords).reshape(-1, 3)
    op = np.ascontiguousarray(obs_point, dtype=np.int64).ravel()
    if len(op) != len(obs):
        raise ValueError('one point index per observation')
    q = _ffi.f64c(queries).reshape(-1, 3)
    out = np.empty(len(q), dtype=np.int64)
    _ffi.check(_ffi.lib().rs_match_observations(
        _ctx(ctx), _ffi.ptr(obs, _d) if len(obs) else None,
        _ffi.ptr(op, _ffi.C.c_int64) if len(op) else None, len(obs),
        _ffi.ptr(q, _d) if len(q) else None, len(q), float(tol), _ffi.ptr(out, _ffi.C.c_int64)))
    return out


def getEFromCameras(C1, C2, ctx=None):
    a, b = _pose(C1), _pose(C2)
    E = np.empty((3, 3))
    _ffi.check(_ffi.lib().rs_e_from_cameras(_ctx(ctx), _ffi.ptr(a, _d), _ffi.ptr(b, _d), 1,
                                            _ffi.ptr(E, _d)))
    return E


def add_new_points(y1_hom, y2_hom, C1, C2, gate=EPIPOLAR_GATE, ctx=None):
    """Returns (accepted mask (n,) bool, X (n, 3) with NaN rows where rejected)."""
    a, b = _pose(C1), _pose(C2)
    y1 = _ffi.f64c(y1_hom).reshape(-1, 3)
    y2 = _ffi.f64c(y2_hom).reshape(-1, 3)
    if y1.shape != y2.shape:
        raise ValueError('y1_hom and y2_hom must have the same shape')
    n = len(y1)
    mask = np.empty(n, dtype=np.int32)
    X = np.empty((n, 3))
    if n:
        _ffi.check(_ffi.lib().rs_add_new_points(_ctx(ctx), _ffi.ptr(a, _d), _ffi.ptr(b, _d),
                                                _ffi.ptr(y1, _d), _ffi.ptr(y2, _d), n,
                                                float(gate), _ffi.ptr(mask, _ffi.C.c_int32),
                                                _ffi.ptr(X, _d)))
    return mask.astype(bool), X


def _ba_args(cams, pts, obs_view, obs_point):
    cams = _ffi.f64c(cams).reshape(-1, 3, 4)
    pts = _ffi.f64c(pts).reshape(-1, 3)
    ov = np.ascontiguousarray(obs_view, dtype=np.int32).ravel()
    op = np.ascontiguousarray(obs_point, dtype=np.int32).ravel()
    if len(ov) != len(op):
        raise ValueError('obs_view and obs_point differ in length')
    return cams, pts, ov, op


def ba_residuals(cams, pts, obs_view, obs_point, uv, ctx=None):
    """EpsilonBA: (2 nObs,) interleaved [u - c1.x/c3.x, v - c2.x/c3.x]."""
    cams, pts, ov, op = _ba_args(cams, pts, obs_view, obs_point)
    uv = _ffi.f64c(uv).reshape(-1, 2)
    if len(uv) != len(ov):
        raise ValueError('one (u, v) per observation')
    r = np.empty(2 * len(ov))
    if len(ov):
        _ffi.check(_ffi.lib().rs_ba_residuals(
            _ctx(ctx), _ffi.ptr(cams, _d), len(cams), _ffi.ptr(pts, _d), len(pts),
            _ffi.ptr(ov, _ffi.C.c_int32), _ffi.ptr(op, _ffi.C.c_int32), _ffi.ptr(uv, _d), len(ov),
            _ffi.ptr(r, _d)))
    return r


def ba_jacobian(cams, pts, obs_view, obs_point, ctx=None):
    """Per observation: Jc (n, 2, 12), Jp (n, 2, 3)."""
    cams, pts, ov, op = _ba_args(cams, pts, obs_view, obs_point)
    n = len(ov)
    Jc, Jp = np.empty((n, 2, 12)), np.empty((n, 2, 3))
    if n:
        _ffi.check(_ffi.lib().rs_ba_jacobian(
            _ctx(ctx), _ffi.ptr(cams, _d), len(cams), _ffi.ptr(pts, _d), len(pts),
            _ffi.ptr(ov, _ffi.C.c_int32), _ffi.ptr(op, _ffi.C.c_int32), n, _ffi.ptr(Jc, _d),
            _ffi.ptr(Jp, _d)))
    return Jc, Jp


# ------------------------------------------------------------------------------------------
# table-level replacements
# ------------------------------------------------------------------------------------------
def add_new_view(T, K, img_index, y1_hom, y2_hom, y1, y2, solvePnPRansac=None, Rodrigues=None):
    """Tables.addNewView (tables.py:104-158) with the matching loop on the GPU and, by default,
    the GPU solvePnPRansac of tsbb15_amd.cv.  Returns (A_y1, A_y2) as the reference.

    The new view's pose is built with the class of the table's existing poses (the reference's
    help_classes.CameraPose in the pipeline), so no reference module is imported here.  When
    PnP-RANSAC fails -- fewer than 4 matched 2D<->3D correspondences (OpenCV asserts 4 too) or
    no consensus -- a ValueError names the number of matched points instead of the reference's
    crash inside Rodrigues / inliers[:, 0]."""
    from . import cv as gcv
    solvePnPRansac = solvePnPRansac or gcv.solvePnPRansac
    Rodrigues = Rodrigues or gcv.Rodrigues
    last = T.T_views[len(T.T_views) - 1]
    pose_cls = type(last.camera_pose)
    idx = np.asarray(last.observations_index, dtype=np.int64)
    obs = np.array([T.T_obs[v].image_coordinates for v in idx]).reshape(-1, 3)
    opt = np.array([T.T_obs[v].point_3D_index for v in idx], dtype=np.int64)
    m = match_observations(obs, opt, np.asarray(y1_hom)[:, :3])
    found = m >= 0
    x_i = m[found]
    D_3D = np.array([T.T_points[j].point for j in x_i]).reshape(-1, 3)
    D_img = np.asarray(y2)[found].reshape(-1, 2)
    D_img_hom = np.asarray(y2_hom)[found].reshape(-1, 3)
    A_y1 = np.asarray(y1)[~found].reshape(-1, 2).astype(np.float64)
    A_y2 = np.asarray(y2)[~found].reshape(-1, 2).astype(np.float64)
    if len(x_i) < 4:
        raise ValueError(f"solvePnPRansac found no pose for view {img_index}: {len(x_i)} "
                         f"putative correspondences matched known 3D points (PnP needs >= 4)")
    retval, R, t, inliers = solvePnPRansac(D_3D[:, :3], D_img[:, :2], K, np.zeros((4, 1)),
                                           useExtrinsicGuess=True)
    if not retval or R is None or inliers is None:
        raise ValueError(f"solvePnPRansac found no pose for view {img_index}: {len(x_i)} "
                         f"putative correspondences matched known 3D points, no consensus")
    R, _ = Rodrigues(R)
    view_index = T.addView(img_index, pose_cls(R, np.asarray(t)[:, 0]))
    for yy, x in zip(D_img_hom[inliers[:, 0]], x_i[inliers[:, 0]]):
        T.addObs(yy, view_index, x)
    return A_y1, A_y2


def add_new_points_table(T, A_y1_hom, A_y2_hom, view_index_1, view_index_2):
    """Tables.addNewPoints (tables.py:161-175): the gate and the triangulations in one GPU
    launch, then the reference's bookkeeping in the reference's order.  Returns the count."""
    C1 = T.T_views[view_index_1].camera_pose
    C2 = T.T_views[view_index_2].camera_pose
    mask, X = add_new_points(A_y1_hom, A_y2_hom, C1, C2)
    counter = 0
    for i in np.flatnonzero(mask):
        point_index = T.addPoint(X[i])
        T.addObs(A_y1_hom[i], view_index_1, point_index)
        T.addObs(A_y2_hom[i], view_index_2, point_index)
        counter += 1
    return counter
