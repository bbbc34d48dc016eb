"""Full-size parity against the reference at the sizes BASELINE.json names.

C2: N = 2 000, 1e5 hypotheses.  C5: N = 10 000, 60 % outliers, 1e6 hypotheses.  The goldens
(tests/golden/full_c2.npz, full_c5.npz) come from tests/golden/make_golden_full.py, which
draws the np.random.seed(0) tuples serially exactly as fun.py:305-306 does and evaluates
every hypothesis with the reference's own lab3.fmatrix_stls / fmatrix_residuals, then
replays fun.py:320-328.  Here the GPU drop-in runs the same loop (fun.ransac_f: tuples parsed
from the numpy stream on the GPU, solve / count / select on the GPU) and must give:

  * every per-hypothesis inlier count (1e5 / 1e6 int), bit-exact;
  * the winner index, S_RANSAC (bit-exact index set), F_RANSAC (1e-6 after normalisation);
  * the advanced np.random state (624 words + position), bit-exact.
"""
import numpy as np
import pytest

from conftest import golden
from oracle import ransac_ref
from tsbb15_amd import _ffi, fun

pytestmark = pytest.mark.gpu

F_TOL = 1e-6  # relative, after normalize_F (north_star)


def _run(ctx, z, base):
    H = int(z["H"])
    p1, p2 = base["p1"], base["p2"]
    n = p1.shape[1]
    key, pos = _ffi.np_seed(0)
    plan = _ffi.F8Plan(ctx, n, H)
    try:
        plan.set_points(p1, p2)
        key2, pos2 = plan.run_np(H, key, pos)
        r, inl = plan.result()
        counts = plan.counts(H)
    finally:
        plan.close()
    return r, inl, counts, key2, pos2


@pytest.mark.parametrize("full,base", [("full_c2.npz", "synth_c2.npz"),
                                       ("full_c5.npz", "synth_c5.npz")])
def test_full_size_parity_vs_reference(ctx, full, base):
    z, b = golden(full), golden(base)
    r, inl, counts, key2, pos2 = _run(ctx, z, b)
    bad = np.flatnonzero(counts != z["counts"].astype(np.int32))
    assert bad.size == 0, f"{bad.size} per-hypothesis counts differ, first {bad[:5]}"
    assert r.best_index == int(z["best"])
    assert r.best_count == len(z["S_ransac"])
    assert np.array_equal(inl, z["S_ransac"].astype(np.int64))
    dF = np.abs(ransac_ref.normalize_F(np.array(r.F[:]).reshape(3, 3))
                - ransac_ref.normalize_F(z["F_ransac"])).max()
    assert dF <= F_TOL, dF
    assert r.guard_mismatch == 0
    assert pos2 == int(z["mt_pos_out"]) and np.array_equal(key2, z["mt_key_out"])


def test_c2_drop_in_full_size(ctx):
    """The drop-in surface (fun.ransac_f on the global np.random, as getFFromLabCode consumes
    it) at C2's 1e5 hypotheses: same winner, S_RANSAC, F and advanced global state."""
    z, b = golden("full_c2.npz"), golden("synth_c2.npz")
    np.random.seed(0)
    res = fun.ransac_f(b["p1"], b["p2"], r=int(z["H"]))
    assert res.best_index == int(z["best"])
    assert np.array_equal(res.inliers, z["S_ransac"].astype(np.int64))
    st = np.random.get_state()
    assert st[2] == int(z["mt_pos_out"]) and np.array_equal(np.asarray(st[1], np.uint32),
                                                           z["mt_key_out"])
