"""Host C++ stream replays vs numpy / CPython themselves and vs the reference goldens.

These run on the CPU: the samplers are host code inside librsamd.so (no device needed)."""
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, golden
from tsbb15_amd import _ffi


def _np_state(seed):
    st = np.random.RandomState(seed).get_state()
    return np.asarray(st[1], np.uint32), int(st[2])


def test_np_seed_matches_randomstate():
    for seed in (0, 1, 12345, 2**32 - 1):
        key, pos = _ffi.np_seed(seed)
        k2, p2 = _np_state(seed)
        assert np.array_equal(key, k2) and pos == p2


@pytest.mark.parametrize("n,count", [(8, 50), (9, 50), (37, 200), (257, 100), (1000, 20),
                                     (2000, 10), (4096, 5), (10000, 3)])
@pytest.mark.parametrize("seed", [0, 7])
def test_np_choice_tuples_match_numpy(n, count, seed):
    key, pos = _np_state(seed)
    tup, key2, pos2 = _ffi.np_choice_tuples(key, pos, n, 8, count)
    rs = np.random.RandomState(seed)
    ref = np.array([rs.choice(np.arange(n), 8, replace=False) for _ in range(count)])
    assert np.array_equal(tup, ref)
    st = rs.get_state()
    assert np.array_equal(key2, np.asarray(st[1], np.uint32)) and pos2 == st[2]


def test_np_choice_other_k_and_midstream_state():
    rs = np.random.RandomState(3)
    rs.random_sample(1001)  # arbitrary position inside the 624-word block
    st = rs.get_state()
    tup, key2, pos2 = _ffi.np_choice_tuples(st[1], st[2], 300, 5, 40)
    ref = np.array([rs.choice(np.arange(300), 5, replace=False) for _ in range(40)])
    assert np.array_equal(tup, ref)
    assert pos2 == rs.get_state()[2]


def test_np_choice_errors():
    key, pos = _np_state(0)
    with pytest.raises(ValueError, match="larger sample"):
        _ffi.np_choice_tuples(key, pos, 7, 8, 1)


def test_np_choice_matches_reference_goldens():
    z = golden("synth_c2.npz")
    tup, key, pos = _ffi.np_choice_tuples(z["mt_key_in"], z["mt_pos_in"], 2000, 8,
                                          len(z["tuples"]))
    assert np.array_equal(tup, z["tuples"].astype(np.int32))
    assert np.array_equal(key, z["mt_key_out"]) and pos == int(z["mt_pos_out"])
    c1 = golden("dino_c1.npz")
    for tag in ("clean", "noisy"):
        n = c1[f"{tag}_p1"].shape[1]
        tup, key, pos = _ffi.np_choice_tuples(c1[f"{tag}_mt_key_in"], c1[f"{tag}_mt_pos_in"], n,
                                              8, 1000)
        assert np.array_equal(tup, c1[f"{tag}_tuples"])
        assert np.array_equal(key, c1[f"{tag}_mt_key_out"])
        assert pos == int(c1[f"{tag}_mt_pos_out"])


def _py_state(seed):
    r = random.Random(seed)
    st = r.getstate()[1]
    return np.array(st[:624], np.uint32), int(st[624]), r


@pytest.mark.parametrize("seed", [0, 1, 5, 12345, 2**40 + 17])
def test_py_seed_matches_cpython(seed):
    key, pos = _ffi.py_seed(seed)
    k2, p2, _ = _py_state(seed)
    assert np.array_equal(key, k2) and pos == p2


@pytest.mark.parametrize("n,k,count", [(6, 6, 30), (37, 6, 100), (500, 6, 50), (1000, 8, 20)])
def test_py_shuffle_matches_cpython(n, k, count):
    key, pos, r = _py_state(42)
    tup, key2, pos2 = _ffi.py_shuffle_tuples(key, pos, n, k, count)
    ref = []
    for _ in range(count):
        x = list(range(n))
        r.shuffle(x)
        ref.append(x[:k])
    assert np.array_equal(tup, np.array(ref))
    st = r.getstate()[1]
    assert np.array_equal(key2, np.array(st[:624], np.uint32)) and pos2 == st[624]


def test_py_shuffle_matches_reference_gen_rnd_indices():
    with open(os.path.join(GOLDEN, "ransac_misc.json")) as f:
        misc = json.load(f)
    key, pos = _ffi.py_seed(0)
    tup, _, _ = _ffi.py_shuffle_tuples(key, pos, 500, 6, 50)
    assert tup.tolist() == misc["gen_rnd_indices_seed0_500_6"]
    key, pos = _ffi.py_seed(12345)
    tup, _, _ = _ffi.py_shuffle_tuples(key, pos, 37, 6, 50)
    assert tup.tolist() == misc["gen_rnd_indices_seed12345_37_6"]
    with pytest.raises(ValueError, match="Cannot generate more indices"):
        _ffi.py_shuffle_tuples(key, pos, 5, 6, 1)


@pytest.mark.parametrize("seed,pre", [(0, 0), (7, 300), (12345, 624)])
def test_mt_jump_matches_sequential_draws(seed, pre):
    """rs_mt_jump (x^J mod the characteristic polynomial) lands on the exact state CPython's
    generator reaches after J getrandbits(32) draws, from fresh and mid-block states."""
    r = random.Random(seed)
    for _ in range(pre):
        r.getrandbits(32)
    st = r.getstate()[1]
    key0, pos0 = np.array(st[:624], np.uint32), st[624]
    done = 0
    for steps in (0, 1, 623 - pos0 % 624 + 1, 624, 625, 1000, 20_000, 123_457):
        while done < steps:
            r.getrandbits(32)
            done += 1
        key, pos = _ffi.mt_jump(key0, pos0, steps)
        ref = r.getstate()[1]
        assert pos == ref[624], steps
        assert np.array_equal(key, np.array(ref[:624], np.uint32)), steps


@pytest.mark.parametrize("j1,j2", [(0, 1), (624, 565_248), (3 * 565_248, 4 * 565_248),
                                   (7 * 64 * 565_248, 64 * 565_248)])
def test_mt_poly_product_is_the_jump_sum(j1, j2):
    """The radix-8 jump tree's level polynomials x^(m 8^k J) are products mod phi
    (mt_poly_mulmod): x^j1 * x^j2 = x^(j1 + j2) mod phi, at C2's chunk length J."""
    assert _ffi.lib().rs_mt_poly_selftest(j1, j2) == 1


def test_np_choice_tuples_multi_equals_single_streams():
    """Threaded replay of many independent numpy streams (config C4's per-pair seeds) = one
    rs_np_choice_tuples call per stream, state included; streams with n < k stay zero."""
    ns = [8, 37, 3, 176, 9, 445, 100, 8]
    keys = np.empty((len(ns), 624), np.uint32)
    poss = np.empty(len(ns), np.int32)
    for b in range(len(ns)):
        keys[b], poss[b] = _ffi.np_seed(1000 + b)
    out, k2, p2 = _ffi.np_choice_tuples_multi(keys, poss, ns, 8, 300, threads=3)
    for b, n in enumerate(ns):
        if n < 8:
            assert not out[b].any() and p2[b] == poss[b] and np.array_equal(k2[b], keys[b])
            continue
        ref, rk, rp = _ffi.np_choice_tuples(keys[b], poss[b], n, 8, 300)
        assert np.array_equal(out[b], ref) and rp == p2[b] and np.array_equal(rk, k2[b])
    o2, k3, p3 = _ffi.np_choice_tuples_multi(None, None, ns, 8, 300, seeds=1000 + np.arange(8))
    assert np.array_equal(o2, out) and np.array_equal(k3, k2) and np.array_equal(p3, p2)
    rs = np.random.RandomState(1003)  # and numpy itself, for one stream
    ref = np.array([rs.choice(np.arange(176), 8, replace=False) for _ in range(300)])
    assert np.array_equal(out[3], ref)


@pytest.mark.parametrize("bad", [-1, 2 ** 32, 2 ** 40, 1.5])
def test_np_seeds_outside_numpy_range_raise(bad):
    """np.random.seed raises ValueError outside [0, 2**32); so do the seeded samplers
    (instead of silently wrapping into another stream)."""
    with pytest.raises((ValueError, TypeError)):
        np.random.RandomState(bad)
    with pytest.raises(ValueError):
        _ffi.np_seed(bad)
    with pytest.raises(ValueError):
        _ffi.np_choice_tuples_multi(None, None, [50, 60], 8, 3, seeds=[0, bad])
    t, _, _ = _ffi.np_choice_tuples_multi(None, None, [50], 8, 3, seeds=[2 ** 32 - 1])
    rs = np.random.RandomState(2 ** 32 - 1)
    np.testing.assert_array_equal(t[0], [rs.choice(np.arange(50), 8, replace=False)
                                         for _ in range(3)])


def test_gen_rnd_tuples_host_route_without_device():
    """With no device (this container) or with the GPU route switched off, gen_rnd_tuples
    draws a long stream on the native host replay: CPython's own tuples and final state."""
    from tsbb15_amd import ransac
    assert 1.4 * 600 * 5000 >= ransac._GPU_MIN_DRAWS  # long enough for the GPU route
    for gpu in (None, False):
        rng, ref = random.Random(5), random.Random(5)
        tup = ransac.gen_rnd_tuples(600, 6, 5000, rng, gpu=gpu)
        want = []
        for _ in range(5000):  # ransac.py:12-19 (random.shuffle of the index list)
            x = list(range(600))
            ref.shuffle(x)
            want.append(x[:6])
        np.testing.assert_array_equal(tup, np.array(want))
        assert rng.getstate() == ref.getstate()
