"""The five-point oracle (oracle/essential_ref.py) pinned by the reference's known answers.
There is no five-point solver in the reference (parity unpinned); its noise-free BAdino2
scene gives exact answers: the E of two views by fun.getEFromCameras (restated as
e_from_cameras) must be among the solutions of any five of their correspondences, and the
Dino pair's E of fun.getEAndK (dino_pnp_kat.npz "E") among those of five Dino matches."""
import numpy as np

from conftest import golden
from oracle import essential_ref as er


def _view_pair(k, i, j, rs, m=5):
    vis = np.flatnonzero((k["points2d"][i, 0] != -1) & (k["points2d"][j, 0] != -1))
    s = rs.choice(vis, m, replace=False)

    def norm(v):
        uv = k["points2d"][v][:, s]
        return (np.linalg.inv(k["K"][v]) @ np.vstack([uv, np.ones(m)])).T
    return norm(i), norm(j)


def test_five_point_contains_badino2_essential():
    k = golden("dino_pnp_kat.npz")
    rs = np.random.RandomState(3)
    for i, j in [(0, 1), (2, 3), (5, 6), (10, 11), (20, 22), (34, 35)]:
        y1, y2 = _view_pair(k, i, j, rs)
        Et = er.e_from_cameras(k["R"][i], k["t"][i], k["R"][j], k["t"][j])
        sols = er.five_point(y1, y2)
        assert 1 <= len(sols) <= 10
        assert any(er.same_e(E, Et, 1e-8) for E in sols), (i, j)
        for E in sols:  # every solution satisfies the five constraints and is essential
            assert np.abs(np.einsum("ia,ab,ib->i", y1, E, y2)).max() < 1e-9
            s = np.linalg.svd(E, compute_uv=False)
            assert abs(s[0] - s[1]) < 1e-8 and s[2] < 1e-8


def test_five_point_contains_dino_pair_essential():
    k = golden("dino_pnp_kat.npz")
    c1 = golden("dino_c1.npz")
    K = k["K_last"]
    y1 = (np.linalg.inv(K) @ np.vstack([c1["clean_p1"], np.ones(37)])).T
    y2 = (np.linalg.inv(K) @ np.vstack([c1["clean_p2"], np.ones(37)])).T
    rs = np.random.RandomState(1)
    for _ in range(5):
        s = rs.choice(37, 5, replace=False)
        assert any(er.same_e(E, k["E"], 1e-8) for E in er.five_point(y1[s], y2[s]))
