"""Multi-rank logic of tsbb15_amd.parallel on the CPU (gloo, world_size 2 and 3): hypothesis
sharding + candidate merge must reproduce the single-process fun.py:320-328 decision, and the
pair table assembled after the all-gather must equal a single-process run."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ransac_ref
from tsbb15_amd import parallel, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_trace(p1, p2, H):
    return ransac_ref.ransac_f(p1, p2, r=H, rng=np.random.RandomState(0), trace=True)


def _records(tr, F_of, lo, hi):
    rec = np.zeros(hi - lo, dtype=parallel.CAND_DTYPE)
    rec["index"] = np.arange(lo, hi)
    rec["count"] = tr.counts[lo:hi]
    rec["std"] = tr.stds[lo:hi]
    rec["norm"] = tr.norms[lo:hi]
    for k, h in enumerate(range(lo, hi)):
        rec["F"][k] = F_of(h).ravel()
    return rec


def _oracle_refiner(K):
    """CPU stand-in for GpuPairRefiner (same item / result layout) built on the oracle."""
    from oracle import twoview_ref as tvr

    def refine(items):
        out = []
        for i, F, a, b, f1, f2 in items:
            Fg, info = tvr.gold_standard_lm(np.asarray(F).reshape(3, 3), a, b)
            E = K.T @ Fg @ K
            y1 = tvr.MakeHomogenous(K, f1[None])[0, :2]
            y2 = tvr.MakeHomogenous(K, f2[None])[0, :2]
            r = tvr.relative_camera_pose(E, y1, y2)
            if r is None:
                out.append((Fg.ravel(), info["cost"], 0, np.full(9, np.nan), np.full(3, np.nan)))
            else:
                out.append((Fg.ravel(), info["cost"], 1, r[0].ravel(), r[1]))
        return out
    return refine


def _worker(rank, world, port, case, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    comm = parallel.TorchComm()
    try:
        if case["kind"] == "shard_np":
            # parity mode: the stream's tuples from the host replay of numpy's choice (pinned to
            # numpy in tests/test_samplers.py), the slice evaluated by the oracle
            p1, p2, H = case["p1"], case["p2"], case["H"]
            key, pos = parallel.np_state(np.random.RandomState(case["seed"]))

            def evaluate(start, cnt, key, pos):
                from tsbb15_amd import _ffi
                tup, key2, pos2 = _ffi.np_choice_tuples(key, pos, p1.shape[1], 8, H)
                rec = np.zeros(cnt, dtype=parallel.CAND_DTYPE)
                for k, h in enumerate(range(start, start + cnt)):
                    F = ransac_ref.fmatrix_stls(p1[:, tup[h]], p2[:, tup[h]])
                    d = ransac_ref.inlier_distance(F, p1, p2)
                    with np.errstate(all="ignore"):
                        rec[k] = (h, np.count_nonzero(d < 1.5), np.std(d), np.linalg.norm(d),
                                  F.ravel())
                return rec, key2, pos2
            best, key2, pos2 = parallel.ransac_f_sharded_np(comm, p1, p2, H, key, pos, evaluate)
            F = best["F"].reshape(3, 3)
            S = np.flatnonzero(ransac_ref.inlier_distance(F, p1, p2) < 1.5)
            q.put((rank, (int(best["index"]), S, F, key2, pos2), None))
        elif case["kind"] == "shard":
            p1, p2, H = case["p1"], case["p2"], case["H"]
            F, S, _, best, tr = _oracle_trace(p1, p2, H)
            lo, n = parallel.shard_range(H, world, rank)
            F_of = lambda h: ransac_ref.fmatrix_stls(p1[:, tr.tuples[h]], p2[:, tr.tuples[h]])
            local = _records(tr, F_of, lo, lo + n)
            lmax = local["count"].max() if n else 0
            win = parallel.merge_shard_candidates(comm, local[local["count"] == lmax])
            q.put((rank, int(win["index"]), best))
        else:
            pairs = case["pairs"]

            def solve(i, p1, p2):
                F, S, d, best, _ = ransac_ref.ransac_f(p1, p2, r=case["H"],
                                                       rng=np.random.RandomState(i))
                return (1, best, len(S), float(d), F.ravel(), S)
            refine = _oracle_refiner(case["K"]) if case.get("K") is not None else None
            tab = parallel.run_pairs(comm, pairs, case["H"], solve, refine=refine)
            q.put((rank, tab.tobytes(), None))
    finally:
        dist.destroy_process_group()


def _spawn(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


def test_shard_range_partitions():
    for H in (1, 7, 100, 100_000):
        for w in (1, 2, 3, 8):
            spans = [parallel.shard_range(H, w, r) for r in range(w)]
            assert spans[0][0] == 0
            assert all(a[0] + a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert spans[-1][0] + spans[-1][1] == H
            assert max(s[1] for s in spans) - min(s[1] for s in spans) <= 1


def test_lpt_assign_balances():
    rng = np.random.RandomState(0)
    costs = list(rng.randint(8, 446, size=231) * 1000)
    parts = parallel.lpt_assign(costs, 8)
    assert sorted(i for p in parts for i in p) == list(range(231))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) <= sum(costs) / 8 + max(costs)
    assert parts == parallel.lpt_assign(costs, 8)


def test_replay_rule_matches_oracle_selection():
    rng = np.random.RandomState(1)
    for _ in range(200):
        n = rng.randint(1, 40)
        counts = rng.randint(0, 4, size=n)
        stds = rng.choice([0.5, 1.0, 2.0, 50.0, np.nan], size=n)
        norms = rng.choice([0.4, 1.5, 3.0, 60.0, np.nan], size=n)
        best = ransac_ref.select_replay(counts, stds, norms)
        rec = np.zeros(n, dtype=parallel.CAND_DTYPE)
        rec["index"], rec["count"], rec["std"], rec["norm"] = np.arange(n), counts, stds, norms
        cmax = counts.max()
        win = parallel.replay_rule(rec[rec["count"] == cmax])
        assert (win is None and best == -1) or int(win["index"]) == best


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_hypothesis_sharding_equals_single_process(world):
    p1, p2, _ = synth.two_view(150, 0.3, seed=21)
    out = _spawn(world, {"kind": "shard", "p1": p1, "p2": p2, "H": 240})
    for rank, idx, best in out:
        assert idx == best


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_parity_mode_sharding_equals_single_process(world):
    """Parity mode sharded over gloo ranks: winner, S_RANSAC, F_RANSAC and the advanced MT
    state equal the single-process oracle loop on the same np.random stream."""
    p1, p2, _ = synth.two_view(150, 0.3, seed=23)
    H, seed = 241, 5
    out = _spawn(world, {"kind": "shard_np", "p1": p1, "p2": p2, "H": H, "seed": seed})
    rs = np.random.RandomState(seed)
    F, S, _, best, _ = ransac_ref.ransac_f(p1, p2, r=H, rng=rs)
    st = rs.get_state()
    for rank, (idx, S_r, F_r, key2, pos2), _ in out:
        assert idx == best
        assert np.array_equal(S_r, S)
        np.testing.assert_array_equal(F_r, F)
        assert pos2 == st[2] and np.array_equal(key2, np.asarray(st[1], np.uint32))


def test_gloo_hypothesis_sharding_all_ties():
    # noise-free data: every hypothesis ties at c* = N and the std/norm rule decides
    p1, p2, _ = synth.two_view(40, 0.0, seed=22, sigma=0.0)
    out = _spawn(2, {"kind": "shard", "p1": p1, "p2": p2, "H": 60})
    for rank, idx, best in out:
        assert idx == best


def test_gloo_pair_table_equals_single_process():
    pairs = [synth.two_view(n, 0.2, seed=30 + i)[:2] for i, n in enumerate([40, 9, 7, 120, 60])]
    out = _spawn(2, {"kind": "pairs", "pairs": pairs, "H": 50})
    tabs = [np.frombuffer(b, dtype=parallel.PAIR_DTYPE) for _, b, _ in out]
    assert tabs[0].tobytes() == tabs[1].tobytes()
    for i, (p1, p2) in enumerate(pairs):
        row = tabs[0][i]
        if p1.shape[1] < 8:
            assert row["valid"] == 0 and row["best_index"] == -1
            continue
        F, S, d, best, _ = ransac_ref.ransac_f(p1, p2, r=50, rng=np.random.RandomState(i))
        assert row["valid"] == 1 and row["best_index"] == best and row["count"] == len(S)
        np.testing.assert_array_equal(row["F"], F.ravel())


def test_gloo_pair_pipeline_refined_equals_single_process():
    """RANSAC + gold standard + E / pose per pair, sharded over 2 ranks, one all-gather: the
    refined table equals the single-process refinement of every pair."""
    K = np.array([[800.0, 0, 320], [0, 800, 240], [0, 0, 1]])
    pairs = [synth.two_view(n, 0.2, seed=40 + i)[:2] for i, n in enumerate([60, 7, 90, 45])]
    out = _spawn(2, {"kind": "pairs", "pairs": pairs, "H": 60, "K": K})
    tabs = [np.frombuffer(b, dtype=parallel.PAIR_DTYPE) for _, b, _ in out]
    assert tabs[0].tobytes() == tabs[1].tobytes()
    ref = _oracle_refiner(K)
    for i, (p1, p2) in enumerate(pairs):
        row = tabs[0][i]
        if p1.shape[1] < 8:
            assert row["valid"] == 0 and row["refined"] == 0
            continue
        F, S, d, best, _ = ransac_ref.ransac_f(p1, p2, r=60, rng=np.random.RandomState(i))
        (Fg, cost, found, R, t), = ref([(i, F, p1[:, S], p2[:, S], p1[:, 0], p2[:, 0])])
        assert row["refined"] == 1 and row["pose"] == found
        np.testing.assert_array_equal(row["F_gold"], Fg)
        np.testing.assert_array_equal(row["R"], R)


def _fileboot_worker(d, rank, q):
    from tsbb15_amd import parallel
    got = parallel.FileBoot(d, rank, timeout=30).broadcast_bytes(b"id-%d" % 7 if rank == 0 else b"")
    q.put((rank, got))


def test_fileboot_broadcasts_the_id(tmp_path):
    """The torch-free RCCL bootstrap: rank 0's bytes reach every rank through the directory."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fileboot_worker, args=(str(tmp_path), r, q)) for r in (2, 1, 0)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert out == {0: b"id-7", 1: b"id-7", 2: b"id-7"}


def _hub_worker(port, rank, world, q):
    from tsbb15_amd import parallel
    hub = parallel.TcpHub(rank, world, "127.0.0.1", port, timeout=60)
    try:
        parts = hub.allgather_bytes(b"r%d" % rank * (rank + 1))
        m = hub.allreduce_max_int(10 * rank - 7)
        f = hub.max_float(0.5 * rank)
        b = hub.broadcast_bytes(b"uid" if rank == 0 else b"", 0)
        hub.barrier()
        # the sharded parity exchange over the hub (MockNpShard steps)
        import sys
        import os
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from np_shard_mock import MockNpShard
        from tsbb15_amd import _ffi
        key, pos = _ffi.np_seed(5)
        parts2, k2, p2 = parallel.np_sharded_tuples(hub, MockNpShard(30, 8, world, rank, seg_cap=20),
                                                    key, pos, 45)
        q.put((rank, (parts, m, f, b, [(g, r.tolist()) for g, r in parts2], k2.tolist(), p2)))
    finally:
        hub.close()


@pytest.mark.parametrize("world", [2, 3])
def test_tcp_hub_collectives(world):
    """The torch-free harness (bench.py): all-gather in rank order, max-reduce, broadcast,
    barrier, and the split-stream exchange carried over it."""
    import multiprocessing as mp
    from tsbb15_amd import _ffi
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hub_worker, args=(port, r, world, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want, wkey, wpos = _ffi.np_choice_tuples(*_ffi.np_seed(5), 30, 8, 45)
    got = np.full((45, 8), -1)
    for r in range(world):
        parts, m, f, b, tp, k2, p2 = out[r]
        assert parts == [b"r%d" % q_ * (q_ + 1) for q_ in range(world)]
        assert m == 10 * (world - 1) - 7 and f == 0.5 * (world - 1) and b == b"uid"
        for g, rows in tp:
            got[g:g + len(rows)] = rows
        assert p2 == wpos and k2 == wkey.tolist()
    assert np.array_equal(got, want)
