"""Pin the oracle (oracle/*.py) against vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, golden
from oracle import pnp_ref, ransac_ref


@pytest.mark.parametrize("tag", ["clean", "noisy"])
def test_oracle_loop_matches_reference_dino(tag):
    z = golden("dino_c1.npz")
    p1, p2 = z[f"{tag}_p1"], z[f"{tag}_p2"]
    rs = np.random.RandomState(0)
    F, S, d, best, tr = ransac_ref.ransac_f(p1, p2, r=1000, rng=rs, trace=True)
    assert np.array_equal(tr.tuples, z[f"{tag}_tuples"])
    assert np.array_equal(tr.counts, z[f"{tag}_counts"])
    assert best == int(z[f"{tag}_best"])
    assert np.array_equal(S, z[f"{tag}_S_ransac"])
    np.testing.assert_allclose(F, z[f"{tag}_F_ransac"], rtol=1e-10, atol=1e-18)
    st = rs.get_state()
    assert np.array_equal(np.asarray(st[1], np.uint32), z[f"{tag}_mt_key_out"])
    assert st[2] == int(z[f"{tag}_mt_pos_out"])


def test_oracle_loop_matches_reference_synth_c2():
    z = golden("synth_c2.npz")
    rs = np.random.RandomState(0)
    r = len(z["counts"])
    F, S, d, best, tr = ransac_ref.ransac_f(z["p1"], z["p2"], r=r, rng=rs, trace=True)
    assert np.array_equal(tr.tuples, z["tuples"])
    assert np.array_equal(tr.counts, z["counts"])
    assert best == int(z["best"])
    assert np.array_equal(S, z["S_ransac"])
    np.testing.assert_allclose(F, z["F_ransac"], rtol=1e-9, atol=1e-18)
    assert np.array_equal(np.asarray(rs.get_state()[1], np.uint32), z["mt_key_out"])
    # selection replay from per-hypothesis statistics == the loop's own decision
    assert ransac_ref.select_replay(tr.counts, tr.stds, tr.norms) == best


def test_oracle_fmatrix_and_residuals_match_reference():
    z = golden("synth_c2.npz")
    p1, p2 = z["p1"], z["p2"]
    for t, Fg in zip(z["tuples"][:64], z["F_tuples64"]):
        F = ransac_ref.fmatrix_stls(p1[:, t], p2[:, t])
        np.testing.assert_allclose(F, Fg, rtol=1e-9, atol=1e-15)
    for Fg, rg in zip(z["F_tuples64"][:2], z["residuals2"]):
        np.testing.assert_allclose(ransac_ref.fmatrix_residuals(Fg, p1, p2), rg, rtol=1e-12,
                                   atol=1e-12)
    c1 = golden("dino_c1.npz")
    for tag in ("clean", "noisy"):
        np.testing.assert_allclose(
            ransac_ref.fmatrix_residuals(c1["F_file"], c1[f"{tag}_p1"], c1[f"{tag}_p2"]),
            c1[f"{tag}_res_Ffile"], rtol=1e-12, atol=1e-12)


def test_oracle_synth_c5_prefix():
    z = golden("synth_c5.npz")
    rs = np.random.RandomState(0)
    r = 60
    _, _, _, _, tr = ransac_ref.ransac_f(z["p1"], z["p2"], r=r, rng=rs, trace=True)
    assert np.array_equal(tr.tuples, z["tuples"][:r])
    assert np.array_equal(tr.counts, z["counts"][:r])


def test_cached_fmatrix_consistent_with_clean_pair():
    # Fmatrix.npy (main.py:42) is the F of the clean Dino pair: the 8-point
    # estimate on all 37 clean points agrees with it up to scale and sign.
    z = golden("dino_c1.npz")
    F = ransac_ref.fmatrix_stls(z["clean_p1"], z["clean_p2"])
    np.testing.assert_allclose(ransac_ref.normalize_F(F), ransac_ref.normalize_F(z["F_file"]),
                               atol=1e-10)


def test_pnp_oracle_known_answers_on_badino2():
    z = golden("dino_pnp_kat.npz")
    for v in (1, 5, 20, 35):
        vis = np.flatnonzero(z["points2d"][v, 0] != -1)
        X = z["points3d"][vis]
        uv = z["points2d"][v][:, vis]
        K = z["K"][v]
        y = (np.linalg.inv(K) @ np.vstack([uv, np.ones((1, len(vis)))])).T
        R, t = pnp_ref.pnp_dlt(X, y)
        np.testing.assert_allclose(R, z["R"][v], atol=1e-9)
        np.testing.assert_allclose(t, z["t"][v], atol=1e-9)
        # minimal 6-point DLT on the noise-free scene recovers the same pose
        R6, t6 = pnp_ref.pnp_dlt(X[:6], y[:6])
        np.testing.assert_allclose(R6, z["R"][v], atol=1e-7)


def test_ransac_helpers_match_reference():
    with open(os.path.join(GOLDEN, "ransac_misc.json")) as f:
        misc = json.load(f)
    for w, n, p, val in misc["calc_r"]:
        assert pnp_ref.calc_r(w, n, p) == pytest.approx(val, rel=1e-14)
    for w, n, r, val in misc["calc_p"]:
        assert pnp_ref.calc_p(w, n, r) == pytest.approx(val, rel=1e-14)
    rng = random.Random(0)
    got = [pnp_ref.gen_rnd_indices(500, 6, rng) for _ in range(50)]
    assert got == misc["gen_rnd_indices_seed0_500_6"]
    rng = random.Random(12345)
    got = [pnp_ref.gen_rnd_indices(37, 6, rng) for _ in range(50)]
    assert got == misc["gen_rnd_indices_seed12345_37_6"]
    with pytest.raises(ValueError):
        pnp_ref.gen_rnd_indices(5, 6)


def test_essential_golden_consistent():
    z = golden("dino_pnp_kat.npz")
    np.testing.assert_allclose(z["R01"], z["clean_data_eval"][1], atol=1e-12)


def test_full_c3_fixture_prefix_replays():
    """full_c3.npz (make_golden_c3.py) replays: the first 1 500 trials of the oracle loop on
    random.seed(0) give the fixture's per-trial consensus sizes."""
    import random
    z = golden("full_c3.npz")
    *_, counts = pnp_ref.ransac_pnp(z["y"], z["X"], z["y"], z["X"], 1500, float(z["thresh"]), 6,
                                    rng=random.Random(0), trace=True)
    assert np.array_equal(counts, z["counts"][:1500].astype(np.int64))
