"""Per-rank cost of the split parity parse (rs_np_shard_*) at C2 / C5, one GPU.

The W ranks' steps are driven one rank at a time on one device (no overlap), so each rank's
time is what its own GPU would spend: parse (jump + stream + chunk parse), compose, tuples +
evaluation.  The multi-GPU run costs about max over ranks of each step plus the collectives.
Usage: python tools/probe_split.py [--n 2000] [--hyps 100000] [--worlds 1,2,4,8] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
sys.path.insert(0, REPO)

from tsbb15_amd import _ffi, parallel, synth  # noqa: E402


def one(ctx, shards, plans, key, pos, H):
    W = len(shards)
    t = {"parse": [0.0] * W, "compose": [0.0] * W, "eval": [0.0] * W}
    done = 0
    best = None
    cands = [[] for _ in range(W)]
    while done < H:
        blobs = []
        for r, sh in enumerate(shards):
            t0 = time.perf_counter()
            sh.parse(key, pos, H - done)
            blobs.append(sh.maps())
            t["parse"][r] += time.perf_counter() - t0
        width = max(len(b) for b in blobs)
        blobs = [b + bytes(width - len(b)) for b in blobs]
        stats = []
        for r, sh in enumerate(shards):
            t0 = time.perf_counter()
            stats.append(sh.compose(blobs))
            t["compose"][r] += time.perf_counter() - t0
        fin = None
        for r, sh in enumerate(shards):
            got, base, hi, nxt, fr = parallel.shard_schedule(stats, H - done, r)
            t0 = time.perf_counter()
            f = plans[r].run_np_shard(sh, base, hi, nxt, got if fr == r else -1, key)
            if hi > base:
                cands[r].append(parallel.candidates_from_plan(plans[r], done + base))
            t["eval"][r] += time.perf_counter() - t0
            if f is not None:
                fin = f
        key, pos = fin
        done += got
    allc = np.concatenate([np.concatenate(c) for c in cands if c])
    cstar = allc["count"].max()
    best = parallel.replay_rule(allc[allc["count"] == cstar])
    return t, best, key, pos


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--outliers", type=float, default=0.30)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--hyps", type=int, default=100_000)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    ctx = _ffi.Context(0)
    p1, p2, _ = synth.two_view(a.n, a.outliers, seed=a.seed)
    key0, pos0 = _ffi.np_seed(0)
    # the single-GPU product path for reference
    plan = _ffi.F8Plan(ctx, a.n, a.hyps)
    plan.set_points(p1, p2)
    ts = []
    for _ in range(a.reps + 1):
        t0 = time.perf_counter()
        plan.run_np(a.hyps, key0, pos0)
        r, _ = plan.result()
        ts.append(time.perf_counter() - t0)
    ref_best = r.best_index
    out = {"n": a.n, "hyps": a.hyps, "run_np_ms": 1e3 * min(ts[1:]), "best": ref_best}
    for W in [int(x) for x in a.worlds.split(",")]:
        shards = [_ffi.NpShard(ctx, a.n, 8, W, r) for r in range(W)]
        plans = []
        for r in range(W):
            pl = _ffi.F8Plan(ctx, a.n, a.hyps)
            pl.set_points(p1, p2)
            plans.append(pl)
        rec = None
        for rep in range(a.reps + 1):
            t, best, k2, p2_ = one(ctx, shards, plans, key0, pos0, a.hyps)
            if rep == 0:
                continue
            tot = [t["parse"][r] + t["compose"][r] + t["eval"][r] for r in range(W)]
            cur = {"max_rank_ms": 1e3 * max(tot),
                   "parse_ms": [round(1e3 * x, 3) for x in t["parse"]],
                   "compose_ms": [round(1e3 * x, 3) for x in t["compose"]],
                   "eval_ms": [round(1e3 * x, 3) for x in t["eval"]],
                   "best": int(best["index"]), "same_winner": int(best["index"]) == ref_best}
            if rec is None or cur["max_rank_ms"] < rec["max_rank_ms"]:
                rec = cur
        out[f"W{W}"] = rec
        for s in shards:
            s.close()
        for p in plans:
            p.close()
        print(json.dumps({f"W{W}": rec}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
