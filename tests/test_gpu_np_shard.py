"""The split parity-stream parse on the GPU (rs_np_shard_*, tsbb15_amd.parallel.
np_sharded_segments / ransac_f_split_np), with W ranks emulated as threads of one process on
one GPU (ThreadComm, each rank its own context and stream).

  * tuples: the union of the ranks' tuples in global order equals the serial host replay of
    fun.py:305-306 (rs_np_choice_tuples) or ransac.py:12-19 (rs_py_shuffle_tuples), bit for
    bit, and every rank ends with the same advanced (key, pos);
  * RANSAC: the split C2 (1e5) and C5 (1e6) runs equal the reference-generated goldens
    (winner, S_RANSAC, F_RANSAC, MT state) at W = 1, 2, 4, 8.
"""
import numpy as np
import pytest

from conftest import golden
from oracle import ransac_ref
from tsbb15_amd import _ffi, parallel

pytestmark = pytest.mark.gpu


def _assemble(parts_per_rank, H, k):
    out = np.full((H, k), -1, np.int32)
    seen = np.zeros(H, np.int64)
    for parts in parts_per_rank:
        for g, rows in parts:
            out[g:g + len(rows)] = rows
            seen[g:g + len(rows)] += 1
    assert np.all(seen == 1), "every hypothesis is produced by exactly one rank"
    return out


def _split_tuples(world, n, k, H, key, pos, py=False):
    def rank_fn(r, comm):
        ctx = _ffi.Context(0)
        sh = _ffi.NpShard(ctx, n, k, world, r, py=py)
        try:
            return parallel.np_sharded_tuples(comm, sh, key, pos, H)
        finally:
            sh.close()
            ctx.close()

    return parallel.run_ranks(world, rank_fn)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("n,k,H,py", [
    (2000, 8, 4000, False),
    (37, 8, 20000, False),
    (9, 8, 30000, False),        # n - 1 < 64: several hypothesis ends per tracking window
    (10241, 8, 150, False),      # the largest population of the GPU parse
    (500, 6, 8000, True),        # CPython stream of gen_rnd_indices (C3)
])
def test_split_tuples_equal_serial_replay(world, n, k, H, py):
    key, pos = _ffi.py_seed(0) if py else _ffi.np_seed(0)
    rep = _ffi.py_shuffle_tuples if py else _ffi.np_choice_tuples
    want, wkey, wpos = rep(key, pos, n, k, H)
    res = _split_tuples(world, n, k, H, key, pos, py)
    assert np.array_equal(_assemble([r[0] for r in res], H, k), want)
    for _, k2, p2 in res:
        assert p2 == wpos and np.array_equal(k2, wkey)


def test_split_tuples_mid_stream_state():
    rs = np.random.RandomState(9)
    rs.random_sample(333)
    key, pos = parallel.np_state(rs)
    want, wkey, wpos = _ffi.np_choice_tuples(key, pos, 700, 8, 6000)
    res = _split_tuples(4, 700, 8, 6000, key, pos)
    assert np.array_equal(_assemble([r[0] for r in res], 6000, 8), want)
    assert all(p == wpos and np.array_equal(kk, wkey) for _, kk, p in res)


def _split_ransac(world, p1, p2, H):
    key, pos = _ffi.np_seed(0)

    def rank_fn(r, comm):
        ctx = _ffi.Context(0)
        try:
            best, k2, p2_ = parallel.ransac_f_split_np(comm, ctx, p1, p2, H, key, pos)
            return best, k2, p2_
        finally:
            ctx.close()

    return parallel.run_ranks(world, rank_fn)


@pytest.mark.parametrize("full,base,worlds", [("full_c2.npz", "synth_c2.npz", (1, 2, 4, 8)),
                                              ("full_c5.npz", "synth_c5.npz", (8,))])
def test_split_ransac_equals_reference_golden(full, base, worlds):
    z, b = golden(full), golden(base)
    H = int(z["H"])
    for world in worlds:
        res = _split_ransac(world, b["p1"], b["p2"], H)
        for best, k2, p2_ in res:
            assert int(best["index"]) == int(z["best"]), world
            assert int(best["count"]) == len(z["S_ransac"])
            inl = parallel.inliers_of(best, b["p1"], b["p2"])
            assert np.array_equal(inl, z["S_ransac"].astype(np.int64))
            dF = np.abs(ransac_ref.normalize_F(best["F"].reshape(3, 3))
                        - ransac_ref.normalize_F(z["F_ransac"])).max()
            assert dF <= 1e-6, dF
            assert p2_ == int(z["mt_pos_out"]) and np.array_equal(k2, z["mt_key_out"])


@pytest.mark.parametrize("world", [2, 4])
def test_split_projection_computes_the_golden_run(ctx, world):
    # bench.py's parity_mode.split_projection: every emulated rank's steps run alone on this
    # GPU; the merged result must be the exact run it claims to time
    z, b = golden("full_c2.npz"), golden("synth_c2.npz")
    key, pos = _ffi.np_seed(0)
    rep, best, k2, p2_ = parallel.project_split_np(ctx, b["p1"], b["p2"], int(z["H"]), key,
                                                   pos, world)
    assert int(best["index"]) == int(z["best"])
    assert np.array_equal(parallel.inliers_of(best, b["p1"], b["p2"]),
                          z["S_ransac"].astype(np.int64))
    assert p2_ == int(z["mt_pos_out"]) and np.array_equal(k2, z["mt_key_out"])
    assert rep["world"] == world and len(rep["rank_total_ms"]) == world
    assert rep["projected_ms"] == max(rep["rank_total_ms"]) > 0
    assert all(len(v) == world for v in rep["per_rank_ms"].values())


def test_split_shard_argument_errors(ctx):
    with pytest.raises(ValueError):
        _ffi.NpShard(ctx, 10, 8, 2, 2)          # rank outside the world
    with pytest.raises(ValueError):
        _ffi.NpShard(ctx, 5, 8, 1, 0)           # k > n (numpy's message)
    sh = _ffi.NpShard(ctx, 100, 8, 2, 0)
    try:
        with pytest.raises(ValueError):
            sh.compose([b"", b""])              # compose before parse
        key, pos = _ffi.np_seed(0)
        sh.parse(key, pos, 100)
        with pytest.raises(ValueError):         # blobs must be the ranks' own, in rank order
            sh.compose([sh.maps(), sh.maps()])
    finally:
        sh.close()
