"""The F plan's optional overlap mode (RSAMD_OVERLAP=1, f8_plan.hip: solve / count / tail on
three streams chained by per-buffer-set events) against the default single-stream plan:
more runs than buffer sets (kBufs = 3) issued back to back in every sampling mode, each
run's winner, candidates, S_RANSAC and the advanced MT state equal."""
import numpy as np
import pytest

from tsbb15_amd import _ffi, parallel, synth

pytestmark = pytest.mark.gpu

N, H = 600, 4000


def _plan(ctx, monkeypatch, overlap):
    if overlap:
        monkeypatch.setenv("RSAMD_OVERLAP", "1")
    else:
        monkeypatch.delenv("RSAMD_OVERLAP", raising=False)
    p1, p2, _ = synth.two_view(N, 0.3, seed=21)
    plan = _ffi.F8Plan(ctx, N, H)
    plan.set_points(p1, p2)
    monkeypatch.delenv("RSAMD_OVERLAP", raising=False)
    return plan


def _rec(plan):
    r, inl = plan.result()
    cands = sorted((c.index, c.count, c.std_d, c.norm_d) for c in plan.candidates())
    return (int(r.best_index), int(r.best_count), list(r.F[:]), inl.tolist(), cands)


def _runs(plan):
    out = []
    # Philox: 7 runs back to back, only the last result read (the tails ride along)
    for i in range(7):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=5, hyp_offset=i * H)
    out.append(_rec(plan))
    for i in range(5):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=6 + i)
        out.append(_rec(plan))
    # host tuples: the staging buffer of a set is refilled only after its copy finished
    key, pos = _ffi.np_seed(3)
    for i in range(5):
        tup, key, pos = _ffi.np_choice_tuples(key, pos, N, 8, H)
        plan.run(H, mode=_ffi.SAMPLER_TUPLES, tuples=tup)
    out.append(_rec(plan))
    # numpy-exact stream parsed on the GPU, whole runs and slices
    key, pos = _ffi.np_seed(0)
    for i in range(4):
        key, pos = plan.run_np(H, key, pos)
        out.append(_rec(plan) + (pos, key.tolist()))
    key0, pos0 = _ffi.np_seed(1)
    for start in (0, 1000, 2500, 3999):
        k2, p2_ = plan.run_np_slice(H, start, min(1000, H - start), key0, pos0)
        out.append(_rec(plan) + (p2_, k2.tolist()))
    return out


def test_overlap_mode_equals_single_stream(ctx, monkeypatch):
    a = _plan(ctx, monkeypatch, True)
    b = _plan(ctx, monkeypatch, False)
    try:
        ra, rb = _runs(a), _runs(b)
    finally:
        a.close()
        b.close()
    assert len(ra) == len(rb)
    for k, (x, y) in enumerate(zip(ra, rb)):
        assert x == y, k


def test_overlap_mode_sharded_parity(ctx, monkeypatch):
    # the split-parse evaluation (run_np_shard) through an overlap-mode plan
    p1, p2, _ = synth.two_view(N, 0.3, seed=21)
    key, pos = _ffi.np_seed(0)
    res = []
    for overlap in (True, False):
        plan = _plan(ctx, monkeypatch, overlap)
        try:
            for _ in range(4):   # more runs than buffer sets
                best, k2, p2_ = parallel.ransac_f_split_np(parallel.ThreadComm.group(1)[0], ctx,
                                                           p1, p2, H, key, pos, plan=plan)
            res.append((int(best["index"]), int(best["count"]), p2_, k2.tolist()))
        finally:
            plan.close()
    assert res[0] == res[1]
