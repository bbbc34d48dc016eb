"""A Tables-compatible fixture for the table-level drop-ins (tsbb15_amd.tables.add_new_view /
add_new_points_table), rebuilt from tests/golden/tables.npz.

The classes hold the same fields and do the same bookkeeping as the reference's data
structures (help_classes.py CameraPose / View / Observation / Point_3D, and Tables.addView /
addPoint / addObs at tables.py:22-39): every View and Point_3D starts its observations_index
with a spurious 0, and addObs appends the new observation's index to both.  Colours
(tables.py:34-35, an image lookup) are not kept.  Test infrastructure only.
"""
from __future__ import annotations

import numpy as np


class Pose:
    def __init__(self, R=np.eye(3), t=np.zeros(3)):
        self.R, self.t = R, t

    def GetCameraMatrix(self):
        M = np.zeros((3, 4))
        M[:, :3], M[:, 3] = self.R, self.t
        return M


class ViewRec:
    def __init__(self, image, camera_pose):
        self.image, self.camera_pose = image, camera_pose
        self.observations_index = np.array([0], dtype=int)


class PointRec:
    def __init__(self, point):
        self.point = point
        self.observations_index = np.array([0], dtype=int)


class ObsRec:
    def __init__(self, image_coordinates, view_index, point_3D_index):
        self.image_coordinates = image_coordinates
        self.view_index, self.point_3D_index = view_index, point_3D_index


class MiniTables:
    def __init__(self, K):
        self.T_obs = np.array([], dtype=object)
        self.T_views = np.array([], dtype=object)
        self.T_points = np.array([], dtype=object)
        self.K = K

    def addView(self, image, pose):
        self.T_views = np.append(self.T_views, np.array([ViewRec(image, pose)]))
        return self.T_views.size - 1

    def addPoint(self, coord):
        self.T_points = np.append(self.T_points, np.array([PointRec(coord)]))
        return self.T_points.size - 1

    def addObs(self, coord, view_index, point_index):
        self.T_obs = np.append(self.T_obs, np.array([ObsRec(coord, view_index, point_index)]))
        k = self.T_obs.size - 1
        v, p = self.T_views[view_index], self.T_points[point_index]
        v.observations_index = np.concatenate((v.observations_index, [k]))
        p.observations_index = np.concatenate((p.observations_index, [k]))


def tables_after_ba(z, tag):
    """The table as Tables.addNewView (tables.py:104) sees it in make_golden_tables.py: views
    0 and 1 and the points with their bundle-adjusted values (ba_x_final), and the
    observations in T_obs order (ba_obs_*)."""
    g = lambda k: z[f"{tag}_{k}"]
    nC, nP = int(g("ba_n_views")), int(g("ba_n_points"))
    x = g("ba_x_final")
    cams, pts = x[:12 * nC].reshape(nC, 3, 4), x[12 * nC:].reshape(nP, 3)
    T = MiniTables(g("K"))
    for v in range(nC):
        T.addView(v, Pose(cams[v, :, :3].copy(), cams[v, :, 3].copy()))
    for p in pts:
        T.addPoint(p.copy())
    for c, v, p in zip(g("ba_obs_coords"), g("ba_obs_view"), g("ba_obs_point")):
        T.addObs(c.copy(), int(v), int(p))
    return T
