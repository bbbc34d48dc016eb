"""GPU parity stream (rs_np_choice_tuples_gpu) against the host replay of numpy's legacy
MT19937 choice (rs_np_choice_tuples, itself pinned to numpy and to the reference goldens in
tests/test_samplers.py).  The bar is bit-exact: every tuple and the advanced (key, pos)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG_DIR, REPO, golden
from tsbb15_amd import _ffi

pytestmark = pytest.mark.gpu


def _state(seed, skip=0):
    rs = np.random.RandomState(seed)
    if skip:
        rs.random_sample(skip)
    st = rs.get_state()
    return np.asarray(st[1], np.uint32), int(st[2])


def _same(n, k, count, seed, skip=0):
    key, pos = _state(seed, skip)
    ref, rkey, rpos = _ffi.np_choice_tuples(key, pos, n, k, count)
    got, gkey, gpos = _ffi.np_choice_tuples_gpu(key, pos, n, k, count)
    bad = np.flatnonzero((got != ref).any(axis=1))
    assert bad.size == 0, f"first mismatching hypothesis {bad[:5]}"
    assert gpos == rpos and np.array_equal(gkey, rkey)


@pytest.mark.parametrize("n,count", [(8, 20000), (9, 5000), (37, 3000), (65, 2000), (66, 2000),
                                     (257, 1000), (2000, 3000), (4097, 300), (10000, 200)])
def test_gpu_stream_matches_host_replay(ctx, n, count):
    _same(n, 8, count, seed=n)


def test_gpu_stream_midstream_state_and_other_k(ctx):
    _same(300, 5, 400, seed=3, skip=1001)
    _same(2000, 8, 50, seed=4, skip=623)
    _same(50, 1, 1000, seed=5, skip=624)


def test_gpu_stream_c2_size(ctx):
    """Config C2's 1e5 hypotheses at N = 2000 (~2.8e8 words, one segment)."""
    _same(2000, 8, 100000, seed=11)


@pytest.mark.parametrize("n,count", [(2000, 30000), (1000, 20000), (300, 40000)])
def test_gpu_stream_two_pass_and_pauses(ctx, monkeypatch, n, count):
    """Chunk-aligned generators with the stream in two passes (the entry kernel beside the
    second), chunks that pause at the first pass's end and resume (RSAMD_NP_XDRAWS: a short
    first pass), and the single-pass layout (RSAMD_NP_SPLIT=0) all give the host replay."""
    _same(n, 8, count, seed=n + 5)
    monkeypatch.setenv("RSAMD_NP_XDRAWS", "700")
    _same(n, 8, count, seed=n + 6)
    monkeypatch.setenv("RSAMD_NP_SPLIT", "0")
    _same(n, 8, count, seed=n + 7)


def test_gpu_stream_reference_goldens(ctx):
    z = golden("synth_c2.npz")
    tup, key, pos = _ffi.np_choice_tuples_gpu(z["mt_key_in"], z["mt_pos_in"], 2000, 8,
                                              len(z["tuples"]))
    assert np.array_equal(tup, z["tuples"].astype(np.int32))
    assert np.array_equal(key, z["mt_key_out"]) and pos == int(z["mt_pos_out"])
    c1 = golden("dino_c1.npz")
    for tag in ("clean", "noisy"):
        n = c1[f"{tag}_p1"].shape[1]
        tup, key, pos = _ffi.np_choice_tuples_gpu(c1[f"{tag}_mt_key_in"],
                                                  c1[f"{tag}_mt_pos_in"], n, 8, 1000)
        assert np.array_equal(tup, c1[f"{tag}_tuples"])
        assert np.array_equal(key, c1[f"{tag}_mt_key_out"])
        assert pos == int(c1[f"{tag}_mt_pos_out"])


def test_gpu_stream_errors(ctx):
    key, pos = _state(0)
    with pytest.raises(ValueError, match="larger sample"):
        _ffi.np_choice_tuples_gpu(key, pos, 7, 8, 1)
    with pytest.raises(ValueError, match="too large"):
        _ffi.np_choice_tuples_gpu(key, pos, 20000, 8, 1)


_SEG_CHILD = """
import numpy as np
from tsbb15_amd import _ffi
for n, count in ((2000, 2000), (37, 40000), (257, 3000), (10000, 100)):
    st = np.random.RandomState(21).get_state()
    key, pos = np.asarray(st[1], np.uint32), int(st[2])
    ref = _ffi.np_choice_tuples(key, pos, n, 8, count)
    got = _ffi.np_choice_tuples_gpu(key, pos, n, 8, count)
    assert np.array_equal(got[0], ref[0]) and got[2] == ref[2] and np.array_equal(got[1], ref[1])
print("ok")
"""


@pytest.mark.parametrize("knobs", [{"RSAMD_NP_SEGWORDS": str(1 << 20)},
                                   {"RSAMD_NP_KW": "8192"},
                                   {"RSAMD_NP_KW": "262144"}])
def test_gpu_stream_many_segments(knobs):
    """Segments of 2^20 words and the shortest / longest parse chunks (these knobs are read
    once per process, so in a child)."""
    env = dict(os.environ, **knobs,
               PYTHONPATH=os.pathsep.join([PKG_DIR, REPO, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c", _SEG_CHILD], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


@pytest.mark.parametrize("knob", [None, "RSAMD_NP_SYNC", "RSAMD_NP_RERUN_TEST"])
@pytest.mark.parametrize("n,H,seed,out", [(2000, 100000, 0, 0.3), (257, 10000, 3, 0.3),
                                          (10240, 2000, 7, 0.3), (10000, 100000, 5, 0.6)])
def test_plan_run_np_equals_host_tuple_run(ctx, monkeypatch, n, H, seed, out, knob):
    """rs_f8_plan_run_np (tuples parsed on the GPU into the run's buffer) = the same plan fed the
    host replay's tuples: winner, S_RANSAC, F bits and the advanced stream state.  C2 at full
    size, and C5's pair (N = 10 000, 60 % outliers) with 1e5 of its 1e6 hypotheses.  Default:
    the run queued behind the parse before its outcome is read; RSAMD_NP_SYNC: the parse waited
    for first; RSAMD_NP_RERUN_TEST: the queued run superseded as after a wrap-log overflow."""
    if knob:
        monkeypatch.setenv(knob, "1")
    from tsbb15_amd import synth
    p1, p2, _ = synth.two_view(n, out, seed=seed + 1)
    key, pos = _state(seed)
    plan = _ffi.F8Plan(ctx, n, H)
    try:
        plan.set_points(p1, p2)
        gkey, gpos = plan.run_np(H, key, pos)
        g = plan.result()
        tup, rkey, rpos = _ffi.np_choice_tuples(key, pos, n, 8, H)
        plan.run(H, mode=_ffi.SAMPLER_TUPLES, tuples=tup)
        h = plan.result()
    finally:
        plan.close()
    assert gpos == rpos and np.array_equal(gkey, rkey)
    assert g[0].best_index == h[0].best_index and g[0].best_count == h[0].best_count
    assert np.array_equal(g[1], h[1])
    assert np.array_equal(np.array(g[0].F[:]), np.array(h[0].F[:]))


@pytest.mark.parametrize("n", [129, 257, 513, 1025, 2049])
def test_gpu_stream_pow2_populations_with_pauses(ctx, monkeypatch, n):
    """N - 1 = 2^k (the top state alone in its mask bucket, the two-bucket batches' edge) with
    the stream in two passes and many chunks pausing at the first pass's end (RSAMD_NP_XDRAWS,
    read at every call): the r04d_tree1 fault's parameters (N = 257, 1e4 hypotheses, seed 3)
    among them.  The parse fails loudly on a corrupt hand-over (err bits 4 / 8) and the host
    checks the segment layout, so an out-of-range index cannot pass silently."""
    count = max(2000, 2_600_000 // n)
    _same(n, 8, count, seed=3)
    for xd in ("700", "5000"):
        monkeypatch.setenv("RSAMD_NP_XDRAWS", xd)
        _same(n, 8, count, seed=n)
    monkeypatch.setenv("RSAMD_NP_XDRAWS", "700")
    key, pos = _state(3)
    from tsbb15_amd import synth
    p1, p2, _ = synth.two_view(n, 0.3, seed=4)
    plan = _ffi.F8Plan(ctx, n, 10000)
    try:
        plan.set_points(p1, p2)
        gkey, gpos = plan.run_np(10000, key, pos)
        g = plan.result()
        tup, rkey, rpos = _ffi.np_choice_tuples(key, pos, n, 8, 10000)
        plan.run(10000, mode=_ffi.SAMPLER_TUPLES, tuples=tup)
        h = plan.result()
    finally:
        plan.close()
    assert gpos == rpos and np.array_equal(gkey, rkey)
    assert g[0].best_index == h[0].best_index and np.array_equal(g[1], h[1])


def test_drop_in_session_across_populations():
    """fun.ransac_f on ONE context for pairs of different N, growing and shrinking (the plan and
    the parse session are retargeted, their buffers kept): every call equals the oracle loop
    (fun.py:303-328 restated) on its own RandomState -- winner, inlier set, F, MT state."""
    from oracle import ransac_ref
    from tsbb15_amd import fun, synth
    c = _ffi.Context(0)
    try:
        for j, n in enumerate((300, 2000, 257, 1500, 2000, 64, 4097)):
            p1, p2, _ = synth.two_view(n, 0.3, seed=20 + j)
            rg, rc = np.random.RandomState(j), np.random.RandomState(j)
            res = fun.ransac_f(p1, p2, r=400, rng=rg, ctx=c)
            F, S, _, best, _ = ransac_ref.ransac_f(p1, p2, r=400, rng=rc)
            assert res.best_index == best, (n, res.best_index, best)
            assert np.array_equal(res.inliers, S), n
            d = np.abs(ransac_ref.normalize_F(res.F) - ransac_ref.normalize_F(F)).max()
            assert d < 1e-6, (n, d)
            assert np.array_equal(rg.get_state()[1], rc.get_state()[1]) and \
                rg.get_state()[2] == rc.get_state()[2], n
    finally:
        c.close()


# ---- the CPython stream (ransac.gen_rnd_indices: random.shuffle, getrandbits rejection) ----
def _py_state(seed, skip=0):
    import random
    r = random.Random(seed)
    for _ in range(skip):
        r.getrandbits(32)
    st = r.getstate()[1]
    return np.asarray(st[:624], np.uint32), int(st[624])


@pytest.mark.parametrize("n,k,count,skip", [(2, 1, 5000, 0), (6, 6, 20000, 0), (9, 6, 5000, 7),
                                            (37, 6, 20000, 0), (65, 3, 3000, 623),
                                            (500, 6, 50000, 0), (2000, 8, 3000, 1),
                                            (4097, 6, 300, 0), (10241, 6, 100, 0)])
def test_gpu_py_stream_matches_host_replay(ctx, n, k, count, skip):
    key, pos = _py_state(n + skip, skip)
    ref, rkey, rpos = _ffi.py_shuffle_tuples(key, pos, n, k, count)
    got, gkey, gpos = _ffi.py_shuffle_tuples_gpu(key, pos, n, k, count)
    bad = np.flatnonzero((got != ref).any(axis=1))
    assert bad.size == 0, f"first mismatching hypothesis {bad[:5]}"
    assert gpos == rpos and np.array_equal(gkey, rkey)


def test_gpu_py_stream_reference_goldens_and_errors(ctx):
    import json
    with open(os.path.join(REPO, "tests", "golden", "ransac_misc.json")) as f:
        misc = json.load(f)
    key, pos = _ffi.py_seed(0)
    tup, _, _ = _ffi.py_shuffle_tuples_gpu(key, pos, 500, 6, 50)
    assert tup.tolist() == misc["gen_rnd_indices_seed0_500_6"]
    key, pos = _ffi.py_seed(12345)
    tup, _, _ = _ffi.py_shuffle_tuples_gpu(key, pos, 37, 6, 50)
    assert tup.tolist() == misc["gen_rnd_indices_seed12345_37_6"]
    with pytest.raises(ValueError, match="Cannot generate more indices"):
        _ffi.py_shuffle_tuples_gpu(key, pos, 5, 6, 1)
    tup, k2, p2 = _ffi.py_shuffle_tuples_gpu(key, pos, 1, 1, 10)  # draws nothing
    assert not tup.any() and p2 == pos and np.array_equal(k2, key)


def test_gen_rnd_tuples_gpu_route_equals_cpython(ctx):
    """ransac.gen_rnd_tuples at C3's size (500 points, 6-point DLT, 5e4 trials) takes the GPU
    stream; the tuples and the advanced global random state equal CPython's own shuffles
    replayed on the host."""
    import random
    from tsbb15_amd import ransac
    random.seed(3)
    st0 = random.getstate()
    tup = ransac.gen_rnd_tuples(500, 6, 50000)
    st1 = random.getstate()
    random.setstate(st0)
    key, pos = np.asarray(st0[1][:624], np.uint32), int(st0[1][624])
    ref, rkey, rpos = _ffi.py_shuffle_tuples(key, pos, 500, 6, 50000)
    assert np.array_equal(tup, ref)
    assert st1[1][624] == rpos and np.array_equal(np.asarray(st1[1][:624], np.uint32), rkey)
    x = list(range(500))  # the next CPython shuffle continues from the advanced state
    random.setstate(st1)
    random.shuffle(x)
    random.setstate(st1)
    assert ransac.gen_rnd_indices(500, 6) == x[:6]


_HOST_CHILD = """
import gc
import numpy as np
from tsbb15_amd import _ffi, synth
from oracle import ransac_ref
ctx = _ffi.default_context()
p1, p2, _ = synth.two_view(500, 0.3, seed=4)
plan = _ffi.F8Plan(ctx, 500, 3000)
plan.set_points(p1, p2)
key, pos = _ffi.np_seed(9)
# back-to-back host-replay runs: no result() in between, the host tuples freed at once
for r in range(4):
    key, pos = plan.run_np(3000, key, pos)
    gc.collect()
out = plan.result()
rs = np.random.RandomState(9)
for r in range(4):
    F, S, _, best, _ = ransac_ref.ransac_f(p1, p2, r=3000, rng=rs)
assert out[0].best_index == best, (out[0].best_index, best)
assert np.array_equal(out[1], S)
assert pos == rs.get_state()[2] and np.array_equal(key, np.asarray(rs.get_state()[1], np.uint32))
# F8Plan.run with temporaries: each tuple array is dropped right after the call
for r in range(3):
    plan.run(3000, mode=_ffi.SAMPLER_TUPLES,
             tuples=np.random.RandomState(r).randint(0, 500, size=(3000, 8)).astype(np.int32))
gc.collect()
res = plan.result()
tup = np.random.RandomState(2).randint(0, 500, size=(3000, 8)).astype(np.int32)
plan.run(3000, mode=_ffi.SAMPLER_TUPLES, tuples=tup)
ref = plan.result()
assert res[0].best_index == ref[0].best_index and np.array_equal(res[1], ref[1])
print("ok")
"""


@pytest.mark.parametrize("knobs", [{"RSAMD_NP_HOST": "1"}])
def test_host_tuple_runs_back_to_back(knobs):
    """The host-replay parity path (RSAMD_NP_HOST) issues runs whose
    tuples live in host memory the library no longer references after the call: back-to-back
    runs with the arrays dropped at once still equal the oracle."""
    env = dict(os.environ, **knobs,
               PYTHONPATH=os.pathsep.join([PKG_DIR, REPO, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c", _HOST_CHILD], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
