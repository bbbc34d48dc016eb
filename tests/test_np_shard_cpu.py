"""The exchange of the split parity-stream parse (tsbb15_amd.parallel.np_sharded_segments,
shard_schedule, ransac_f_split_np's merge) on the CPU.

The shard steps run on tests/np_shard_mock.MockNpShard (a per-draw replay of the same
stream), the ranks are threads (ThreadComm) or gloo processes (world 2 / 3).  Every run must
give exactly the single-stream replay: the union of the ranks' tuples in global order equals
rs_np_choice_tuples / rs_py_shuffle_tuples (host C++, pinned to numpy / CPython in
tests/test_samplers.py), and every rank ends with the same advanced (key, pos).  The GPU form
of the same steps is tests/test_gpu_np_shard.py."""
import os
import socket

import numpy as np
import pytest

from np_shard_mock import MockNpShard
from tsbb15_amd import _ffi, parallel


def _replay(key, pos, n, k, H, py):
    f = _ffi.py_shuffle_tuples if py else _ffi.np_choice_tuples
    return f(key, pos, n, k, H)


def _assemble(parts_per_rank, H, k):
    out = np.full((H, k), -1, np.int32)
    seen = np.zeros(H, np.int64)
    for parts in parts_per_rank:
        for g, rows in parts:
            out[g:g + len(rows)] = rows
            seen[g:g + len(rows)] += 1
    assert np.all(seen == 1), "every hypothesis is produced by exactly one rank"
    return out


def test_shard_schedule_offsets():
    # rank 0 holds the segment's first start (draw 0) plus 3 wraps; rank 1 none; rank 2 two
    stats = [(4, 0), (0, -1), (2, 900)]
    got, base, hi, nxt, fr = parallel.shard_schedule(stats, 10, 0)
    assert (got, base, hi, nxt, fr) == (5, 0, 4, 900, 2)
    got, base, hi, nxt, fr = parallel.shard_schedule(stats, 10, 1)
    assert (base, hi, nxt) == (4, 4, 900)
    got, base, hi, nxt, fr = parallel.shard_schedule(stats, 10, 2)
    assert (base, hi, nxt) == (4, 5, -1)
    # fewer hypotheses asked for than the segment holds: the final state is start `count`
    got, base, hi, nxt, fr = parallel.shard_schedule(stats, 2, 0)
    assert (got, hi, fr) == (2, 2, 0)
    with pytest.raises(RuntimeError):
        parallel.shard_schedule([(1, 0), (0, -1)], 5, 0)


@pytest.mark.parametrize("world,n,k,H,py,seg_cap,slack", [
    (1, 37, 8, 60, False, None, None),
    (2, 37, 8, 60, False, None, None),
    (3, 50, 8, 90, False, 31, None),      # several segments
    (8, 23, 8, 40, False, None, 0),       # short rank ranges: ranks with no start at all
    (4, 41, 6, 70, True, 25, 64),         # CPython stream (gen_rnd_indices), segments
    (5, 9, 8, 200, False, 64, 0),         # n - 1 = 8 states
])
def test_thread_ranks_reproduce_the_stream(world, n, k, H, py, seg_cap, slack):
    key, pos = (_ffi.py_seed(12345) if py else _ffi.np_seed(7))
    want, wkey, wpos = _replay(key, pos, n, k, H, py)

    def rank_fn(r, comm):
        sh = MockNpShard(n, k, world, r, py=py, seg_cap=seg_cap, slack=slack)
        return parallel.np_sharded_tuples(comm, sh, key, pos, H)

    res = parallel.run_ranks(world, rank_fn)
    got = _assemble([r[0] for r in res], H, k)
    assert np.array_equal(got, want)
    for _, k2, p2 in res:
        assert p2 == wpos and np.array_equal(k2, wkey)


def test_thread_ranks_mid_stream_state():
    """A stream that does not start at a fresh seed (pos < 624, a partly used block)."""
    rs = np.random.RandomState(3)
    rs.random_sample(101)
    key, pos = parallel.np_state(rs)
    want, wkey, wpos = _replay(key, pos, 30, 8, 50, False)
    res = parallel.run_ranks(3, lambda r, c: parallel.np_sharded_tuples(
        c, MockNpShard(30, 8, 3, r, seg_cap=17), key, pos, 50))
    assert np.array_equal(_assemble([x[0] for x in res], 50, 8), want)
    assert all(p == wpos and np.array_equal(kk, wkey) for _, kk, p in res)


def test_thread_rank_failure_propagates():
    def rank_fn(r, comm):
        if r == 1:
            raise ValueError("boom")
        return parallel.np_sharded_tuples(comm, MockNpShard(20, 8, 2, r), *_ffi.np_seed(0), 5)

    with pytest.raises(ValueError, match="boom"):
        parallel.run_ranks(2, rank_fn)


# ---- gloo processes --------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, case, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        comm = parallel.TorchComm()
        n, k, H, seg = case["n"], case["k"], case["H"], case["seg_cap"]
        key, pos = _ffi.np_seed(case["seed"])
        if case["kind"] == "tuples":
            sh = MockNpShard(n, k, world, rank, seg_cap=seg)
            q.put((rank, parallel.np_sharded_tuples(comm, sh, key, pos, H)))
        else:  # RANSAC over the split stream, the slice evaluated by the oracle
            from oracle import ransac_ref
            p1, p2 = case["p1"], case["p2"]
            sh = MockNpShard(n, 8, world, rank, seg_cap=seg)
            cands = []

            def consume(off, base, hi, nxt, fidx, key):
                rows, fin = sh.tuples(base, hi, nxt, fidx, key)
                rec = np.zeros(len(rows), dtype=parallel.CAND_DTYPE)
                for j, t in enumerate(rows):
                    F = ransac_ref.fmatrix_stls(p1[:, t], p2[:, t])
                    d = ransac_ref.inlier_distance(F, p1, p2)
                    with np.errstate(all="ignore"):
                        rec[j] = (off + base + j, np.count_nonzero(d < 1.5), np.std(d),
                                  np.linalg.norm(d), F.ravel())
                cands.append(rec)
                return fin

            key2, pos2 = parallel.np_sharded_segments(comm, sh, key, pos, H, consume)
            best = parallel.merge_shard_candidates(comm, np.concatenate(cands))
            q.put((rank, (int(best["index"]), key2, pos2)))
    finally:
        dist.destroy_process_group()


def _spawn(world, case):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [out[r] for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_split_stream_equals_replay(world):
    case = {"kind": "tuples", "n": 45, "k": 8, "H": 80, "seg_cap": 33, "seed": 11}
    res = _spawn(world, case)
    key, pos = _ffi.np_seed(11)
    want, wkey, wpos = _replay(key, pos, 45, 8, 80, False)
    assert np.array_equal(_assemble([r[0] for r in res], 80, 8), want)
    for _, k2, p2 in res:
        assert p2 == wpos and np.array_equal(k2, wkey)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_split_ransac_equals_single_process(world):
    from oracle import ransac_ref
    from tsbb15_amd import synth
    p1, p2, _ = synth.two_view(60, 0.3, seed=4)
    H = 120
    F, S, _, best, st = ransac_ref.ransac_f(p1, p2, r=H, rng=np.random.RandomState(0))
    case = {"kind": "ransac", "n": 60, "k": 8, "H": H, "seg_cap": 50, "seed": 0,
            "p1": p1, "p2": p2}
    res = _spawn(world, case)
    rs = np.random.RandomState(0)
    ransac_ref.ransac_f(p1, p2, r=H, rng=rs)
    wkey, wpos = parallel.np_state(rs)
    for b, k2, p2_ in res:
        assert b == best
        assert p2_ == wpos and np.array_equal(k2, wkey)
