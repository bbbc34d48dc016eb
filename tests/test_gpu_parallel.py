"""Sharded execution on the GPU: hypothesis shards (Philox counters are global hypothesis
indices, so shards reproduce the single run), the RCCL communicator at world size 1, and the
36-view Dino ring (config C4: all C(36,2) pairs of BAdino2.mat)."""
import itertools

import numpy as np
import pytest

from conftest import golden
from oracle import ransac_ref
from tsbb15_amd import _ffi, parallel, synth

pytestmark = pytest.mark.gpu


class _Boot:
    def broadcast_bytes(self, b, src=0):
        return b


class _Solo:
    rank, world = 0, 1

    def allgather_bytes(self, b):
        return [b]

    def allreduce_max_int(self, v):
        return int(v)


def test_hypothesis_shards_reproduce_single_run(ctx):
    p1, p2, _ = synth.two_view(2000, 0.3, seed=1)
    H, seed = 20_000, 77
    plan = _ffi.F8Plan(ctx, 2000, H)
    plan.set_points(p1, p2)
    plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=seed)
    ref, ref_inl = plan.result()
    ref_counts = plan.counts(H)
    parts = []
    for w in range(4):
        lo, n = parallel.shard_range(H, 4, w)
        plan.run(n, mode=_ffi.SAMPLER_PHILOX, seed=seed, hyp_offset=lo)
        plan.result()
        assert np.array_equal(plan.counts(n), ref_counts[lo:lo + n])
        parts.append(parallel.candidates_from_plan(plan, lo))
    allc = np.concatenate(parts)
    cstar = allc["count"].max()
    win = parallel.replay_rule(allc[allc["count"] == cstar])
    assert int(win["index"]) == ref.best_index and int(win["count"]) == ref.best_count


def test_rccl_world_one_sharded_api(ctx):
    p1, p2, _ = synth.two_view(500, 0.3, seed=2)
    comm = parallel.RcclComm(ctx, 0, 1, _Boot())
    try:
        assert comm.allreduce_max_int(17) == 17
        assert comm.allgather_bytes(b"abcdefgh") == [b"abcdefgh"]
        best, inl = parallel.ransac_f_sharded(comm, ctx, p1, p2, 5000, seed=3)
    finally:
        comm.close()
    plan = _ffi.F8Plan(ctx, 500, 5000)
    plan.set_points(p1, p2)
    plan.run(5000, mode=_ffi.SAMPLER_PHILOX, seed=3)
    r, rinl = plan.result()
    assert int(best["index"]) == r.best_index
    assert np.array_equal(inl, rinl)


def test_parity_mode_slices_reproduce_run_np(ctx):
    """Parity-mode sharding in one process: four slices of a C2-sized numpy-stream run
    (rs_f8_plan_run_np_slice), merged by the fun.py:320-328 replay, equal the single run_np:
    winner, count, and the advanced stream state of every slice."""
    p1, p2, _ = synth.two_view(2000, 0.3, seed=1)
    H = 100_000
    key, pos = _ffi.np_seed(0)
    plan = _ffi.F8Plan(ctx, 2000, H)
    plan.set_points(p1, p2)
    rkey, rpos = plan.run_np(H, key, pos)
    ref, ref_inl = plan.result()
    ref_counts = plan.counts(H)
    plan.close()
    ev = parallel.GpuSliceEvaluator(ctx, p1, p2, H, max_slice=H // 4 + 1)
    parts = []
    try:
        for w in range(4):
            lo, n = parallel.shard_range(H, 4, w)
            local, k2, p2_ = ev(lo, n, key, pos)
            assert p2_ == rpos and np.array_equal(k2, rkey)
            assert np.array_equal(ev.plan.counts(n), ref_counts[lo:lo + n])
            parts.append(local)
        allc = np.concatenate(parts)
        win = parallel.replay_rule(allc[allc["count"] == allc["count"].max()])
        assert int(win["index"]) == ref.best_index and int(win["count"]) == ref.best_count
        assert np.array_equal(ev.inliers(win), ref_inl)
    finally:
        ev.close()


def test_rccl_world_one_parity_mode(ctx):
    """ransac_f_sharded_np over the RCCL communicator at world size 1 = run_np, and the C2
    reference golden (tests/golden/full_c2.npz: winner of the unmodified loop at 1e5)."""
    z, b = golden("full_c2.npz"), golden("synth_c2.npz")
    H = int(z["H"])
    comm = parallel.RcclComm(ctx, 0, 1, _Boot())
    ev = parallel.GpuSliceEvaluator(ctx, b["p1"], b["p2"], H)
    try:
        key, pos = parallel.np_state(np.random.RandomState(0))
        best, key2, pos2 = parallel.ransac_f_sharded_np(comm, b["p1"], b["p2"], H, key, pos, ev)
        inl = ev.inliers(best)
    finally:
        ev.close()
        comm.close()
    assert int(best["index"]) == int(z["best"])
    assert np.array_equal(inl, z["S_ransac"].astype(np.int64))
    assert pos2 == int(z["mt_pos_out"]) and np.array_equal(key2, z["mt_key_out"])


def _dino_pairs():
    z = golden("dino_pnp_kat.npz")
    P = z["points2d"]
    pairs = []
    for i, j in itertools.combinations(range(36), 2):
        vis = np.flatnonzero(np.any(P[i] != -1, axis=0) & np.any(P[j] != -1, axis=0))
        pairs.append((np.ascontiguousarray(P[i][:, vis]), np.ascontiguousarray(P[j][:, vis])))
    return pairs


def test_dino_ring_all_pairs(ctx):
    pairs = _dino_pairs()
    assert len(pairs) == 630
    solver = parallel.GpuPairSolver(ctx, 1000)
    try:
        tab = parallel.run_pairs(_Solo(), pairs, 1000, solver)
    finally:
        solver.close()
    n = np.array([p1.shape[1] for p1, _ in pairs])
    # correspondences.py:37-42 filter; 284 non-empty pairs, 203 with N >= 8
    assert int((n > 0).sum()) == 284 and int((n >= 8).sum()) == 203
    assert int(n[n >= 8].sum()) == 11257
    assert np.array_equal(tab["valid"] == 1, n >= 8)
    # noise-free scene: every valid pair's winner explains all of its correspondences
    for i in np.flatnonzero(n >= 8)[::10]:
        p1, p2 = pairs[i]
        F = tab["F"][i].reshape(3, 3)
        d = ransac_ref.inlier_distance(F, p1, p2)
        assert tab["count"][i] == np.count_nonzero(d < 1.5) == p1.shape[1]


def test_dino_ring_pipeline_poses(ctx):
    """C4 end to end on the GPU: RANSAC per pair, then one batched gold-standard launch and
    one batched E / relative-pose launch over all 203 valid pairs.  The BAdino2 scene is
    noise-free, so every pair's pose must be the true relative pose of its two resectioned
    cameras (fun.camera_resectioning goldens): R = R_j R_i^T, and t = -unit(t_j - R t_i) --
    the reference's chirality convention, pinned by clean_data_eval / twoview.npz pose_t."""
    z = golden("dino_pnp_kat.npz")
    pairs = _dino_pairs()
    solver = parallel.GpuPairBatchSolver(ctx, 1000)
    refiner = parallel.GpuPairRefiner(ctx, z["K_last"])
    tab = parallel.run_pairs(_Solo(), pairs, 1000, solver, refine=refiner)
    ij = list(itertools.combinations(range(36), 2))
    valid = np.flatnonzero(tab["valid"] == 1)
    assert len(valid) == 203 and np.all(tab["refined"][valid] == 1)
    assert np.all(tab["pose"][valid] > 0)
    Rs, ts = z["R"], z["t"]
    worst_R = worst_t = 0.0
    for k in valid:
        i, j = ij[k]
        Rt = Rs[j] @ Rs[i].T
        tt = ts[j] - Rt @ ts[i]
        worst_R = max(worst_R, np.abs(tab["R"][k].reshape(3, 3) - Rt).max())
        worst_t = max(worst_t, np.abs(tab["t"][k] + tt / np.linalg.norm(tt)).max())
        assert tab["gs_cost"][k] < 1e-12
    assert worst_R < 1e-6 and worst_t < 1e-6, (worst_R, worst_t)


def test_dino_ring_array_path_matches_object_path(ctx):
    """run_pairs' array path (many_arrays / arrays: concatenated points, column-wise records)
    gives the same table as the per-pair object path (many / __call__), field for field."""
    z = golden("dino_pnp_kat.npz")
    pairs = _dino_pairs()
    solver = parallel.GpuPairBatchSolver(ctx, 1000)
    refiner = parallel.GpuPairRefiner(ctx, z["K_last"])

    class ObjSolver:  # the object path only
        def __init__(self, inner):
            self.many = inner.many

    class ObjRefiner:
        def __init__(self, inner):
            self.inner = inner

        def __call__(self, items):
            return self.inner(items)

    fast = parallel.run_pairs(_Solo(), pairs, 1000, solver, refine=refiner)
    slow = parallel.run_pairs(_Solo(), pairs, 1000, ObjSolver(solver), refine=ObjRefiner(refiner))
    for f in parallel.PAIR_DTYPE.names:
        assert np.array_equal(fast[f], slow[f], equal_nan=fast[f].dtype.kind == "f"), f
    assert int(fast["refined"].sum()) > 100 and int((fast["pose"] > 0).sum()) > 100


@pytest.mark.parametrize("with_k", [True, False])
def test_dino_ring_fused_call_matches_separate_calls(ctx, with_k):
    """rs_pairs_two_view (RANSAC, gold standard, E and pose in one device call) gives the
    table of the separate calls (rs_pairs_f8_ransac, host gather, rs_gold_standard,
    rs_essential_from_f, rs_relative_camera_pose), field for field; without K no pose."""
    z = golden("dino_pnp_kat.npz")
    pairs = _dino_pairs()
    K = z["K_last"] if with_k else None
    solver = parallel.GpuPairBatchSolver(ctx, 1000)
    fused = parallel.run_pairs(_Solo(), pairs, 1000, solver,
                               refine=parallel.GpuPairRefiner(ctx, K))
    sep = parallel.run_pairs(_Solo(), pairs, 1000, solver,
                             refine=parallel.GpuPairRefiner(ctx, K, fused=False))
    for f in parallel.PAIR_DTYPE.names:
        assert np.array_equal(fused[f], sep[f], equal_nan=fused[f].dtype.kind == "f"), f
    if not with_k:
        assert int((fused["pose"] > 0).sum()) == 0


def test_fused_call_over_1024_pairs_matches_separate_calls(ctx):
    """More than 1024 pairs in one rs_pairs_two_view call (the gather's multi-round scan in
    k_twoview_prep): the Dino ring's 630 pairs twice, fused against the separate calls."""
    z = golden("dino_pnp_kat.npz")
    pairs = _dino_pairs() * 2
    assert len(pairs) > 1024
    solver = parallel.GpuPairBatchSolver(ctx, 200)
    fused = parallel.run_pairs(_Solo(), pairs, 200, solver,
                               refine=parallel.GpuPairRefiner(ctx, z["K_last"]))
    sep = parallel.run_pairs(_Solo(), pairs, 200, solver,
                             refine=parallel.GpuPairRefiner(ctx, z["K_last"], fused=False))
    for f in parallel.PAIR_DTYPE.names:
        assert np.array_equal(fused[f], sep[f], equal_nan=fused[f].dtype.kind == "f"), f
    assert int((fused["valid"] == 1).sum()) > 300


def test_two_view_pairs_raw_edges(ctx):
    """Pairs without a consensus (N < 8, empty) inside a fused call: NaN F_gold / pose, found
    0, zero gold-standard info; the other pairs as in a call without them."""
    from tsbb15_amd import pairs as pairs_mod
    z = golden("dino_pnp_kat.npz")
    allp = _dino_pairs()
    big = [p for p in allp if p[0].shape[1] >= 20]
    dp = [big[0], big[1], big[2]]
    chosen = [dp[0], (dp[1][0][:, :5], dp[1][1][:, :5]), (np.zeros((2, 0)), np.zeros((2, 0))),
              dp[2]]
    off = np.zeros(len(chosen) + 1, dtype=np.int64)
    np.cumsum([p[0].shape[1] for p in chosen], out=off[1:])
    p1 = np.hstack([p[0] for p in chosen])
    p2 = np.hstack([p[1] for p in chosen])
    res, _, Fg, info, R, t, found = pairs_mod.two_view_pairs_raw(p1, p2, off, 1000, z["K_last"],
                                                                 ctx=ctx)
    for b in (1, 2):
        assert res["best_index"][b] == -1
        assert np.isnan(Fg[b]).all() and np.isnan(R[b]).all() and np.isnan(t[b]).all()
        assert found[b] == 0 and info["n"][b] == 0 and info["iterations"][b] == 0
    keep = [0, 3]
    off2 = np.array([0, dp[0][0].shape[1], dp[0][0].shape[1] + dp[2][0].shape[1]])
    r2 = pairs_mod.two_view_pairs_raw(np.hstack([dp[0][0], dp[2][0]]),
                                      np.hstack([dp[0][1], dp[2][1]]), off2, 1000, z["K_last"],
                                      ids=np.array(keep), ctx=ctx)
    for a, b in zip((res, Fg, info, R, t, found), (r2[0], r2[2], r2[3], r2[4], r2[5], r2[6])):
        a2 = a[keep]
        if a2.dtype.names:
            for f in a2.dtype.names:
                assert np.array_equal(a2[f], b[f], equal_nan=True), f
        else:
            assert np.array_equal(a2, b, equal_nan=True)


def test_two_view_pairs_raw_rejects_bad_arguments(ctx):
    """rs_pairs_two_view's argument errors fail loudly (ValueError from RS_EINVAL) before any
    launch: max_iter outside [1, 1e5], K without the first correspondences, bad offsets."""
    from tsbb15_amd import pairs as pairs_mod
    z = golden("dino_pnp_kat.npz")
    p = [q for q in _dino_pairs() if q[0].shape[1] >= 20][0]
    off = np.array([0, p[0].shape[1]])
    with pytest.raises(ValueError, match="max_iter"):
        pairs_mod.two_view_pairs_raw(p[0], p[1], off, 100, z["K_last"], max_iter=0, ctx=ctx)
    with pytest.raises(ValueError):
        pairs_mod.two_view_pairs_raw(p[0], p[1], np.array([0, p[0].shape[1] + 1]), 100, ctx=ctx)
    d = _ffi.C.c_double
    res = (_ffi.PairResult * 1)()
    info = (_ffi.GsInfo * 1)()
    buf = np.zeros(64)
    K = np.ascontiguousarray(z["K_last"], dtype=np.float64)
    st = _ffi.lib().rs_pairs_two_view(
        ctx.handle, _ffi.ptr(np.ascontiguousarray(p[0], dtype=np.float64), d),
        _ffi.ptr(np.ascontiguousarray(p[1], dtype=np.float64), d),
        _ffi.ptr(np.ascontiguousarray(off, dtype=np.int64), _ffi.C.c_int64), 1, 100,
        _ffi.SAMPLER_PHILOX, 0, None, None, 1.5, 50, _ffi.ptr(K, d), None, None, res,
        _ffi.ptr(np.zeros(p[0].shape[1], dtype=np.int32), _ffi.C.c_int32), _ffi.ptr(buf, d), info,
        _ffi.ptr(buf, d), _ffi.ptr(buf, d), _ffi.ptr(np.zeros(1, dtype=np.int32), _ffi.C.c_int32))
    assert st == _ffi.RS_EINVAL
    # decreasing offsets straight through the C ABI (the Python wrapper rejects them first):
    # the library's own check, before the offsets size any buffer
    n = p[0].shape[1]
    bad = np.array([0, n, n // 2], dtype=np.int64)
    res2 = (_ffi.PairResult * 2)()
    info2 = (_ffi.GsInfo * 2)()
    big = np.zeros(64)
    st = _ffi.lib().rs_pairs_two_view(
        ctx.handle, _ffi.ptr(np.ascontiguousarray(p[0], dtype=np.float64), d),
        _ffi.ptr(np.ascontiguousarray(p[1], dtype=np.float64), d), _ffi.ptr(bad, _ffi.C.c_int64),
        2, 100, _ffi.SAMPLER_PHILOX, 0, None, None, 1.5, 50, None, None, None, res2,
        _ffi.ptr(np.zeros(n, dtype=np.int32), _ffi.C.c_int32), _ffi.ptr(big, d), info2,
        _ffi.ptr(big, d), _ffi.ptr(big, d), _ffi.ptr(np.zeros(2, dtype=np.int32), _ffi.C.c_int32))
    assert st == _ffi.RS_EINVAL
    assert b"non-decreasing" in _ffi.lib().rs_last_error()
