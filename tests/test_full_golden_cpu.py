"""CPU checks of the full-size goldens (tests/golden/full_c2.npz, full_c5.npz; written from the
reference by tests/golden/make_golden_full.py) against the host stream replay and the oracle.

The GPU parity tests (tests/test_gpu_full_parity.py) compare the HIP path with these goldens;
here the goldens themselves are cross-checked without a GPU: the host C++ replay of numpy's
legacy choice stream (pinned to numpy in tests/test_samplers.py) reproduces the last tuples
and the advanced MT state of the C2 run, and the oracle restatement of lab3.py / fun.py
reproduces the winner's count, S_RANSAC and F and the replay of fun.py:320-328."""
import numpy as np

from conftest import golden
from oracle import ransac_ref
from tsbb15_amd import _ffi


def test_full_c2_golden_stream_tail_and_state():
    z = golden("full_c2.npz")
    H = int(z["H"])
    key, pos = _ffi.np_seed(0)
    tup, key2, pos2 = _ffi.np_choice_tuples(key, pos, 2000, 8, H)
    assert np.array_equal(tup[-64:], z["tuples_tail"].astype(np.int32))
    assert pos2 == int(z["mt_pos_out"]) and np.array_equal(key2, z["mt_key_out"])
    # the first 2000 hypotheses are the round-1 C2 golden
    b = golden("synth_c2.npz")
    assert np.array_equal(z["counts"][:2000], b["counts"])
    # the oracle re-evaluates the winner and every hypothesis tied at the maximum
    p1, p2 = b["p1"], b["p2"]
    best = int(z["best"])
    F = ransac_ref.fmatrix_stls(p1[:, tup[best]], p2[:, tup[best]])
    d = np.max(np.abs(ransac_ref.fmatrix_residuals(F, p1, p2)), axis=0)
    S = np.flatnonzero(d < ransac_ref.INLIER_THRESHOLD)
    assert np.array_equal(S, z["S_ransac"].astype(np.int64))
    assert np.abs(ransac_ref.normalize_F(F) - ransac_ref.normalize_F(z["F_ransac"])).max() < 1e-9
    assert int(z["counts"].max()) == len(S)
    for i in z["tie_index"]:
        Fi = ransac_ref.fmatrix_stls(p1[:, tup[i]], p2[:, tup[i]])
        di = np.max(np.abs(ransac_ref.fmatrix_residuals(Fi, p1, p2)), axis=0)
        assert np.count_nonzero(di < 1.5) == len(S)


def test_full_goldens_replay_rule():
    """fun.py:320-328 over the stored records picks the stored winner: the first hypothesis
    at the maximum count, then later ties only when |std(best)| > norm(d)."""
    for name in ("full_c2.npz", "full_c5.npz"):
        z = golden(name)
        counts = z["counts"].astype(np.int64)
        cmax = counts.max()
        ties = z["tie_index"]
        assert np.array_equal(ties, np.flatnonzero(counts == cmax))
        best, d_best = int(ties[0]), float(z["tie_std"][0])
        for i, s, nrm in zip(ties[1:], z["tie_std"][1:], z["tie_norm"][1:]):
            if abs(d_best) > nrm:
                best, d_best = int(i), float(s)
        assert best == int(z["best"])
        assert len(z["S_ransac"]) == cmax
