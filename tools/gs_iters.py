"""C4 gold standard per pair: inlier count n and LM iterations / accepted steps (GsInfo), the
pairs that bound k_gold_standard's launch."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_c4  # noqa: F401,E402
from tsbb15_amd import _ffi, parallel, twoview  # noqa: E402

import itertools  # noqa: E402
REPO = probe_c4.REPO
z = np.load(os.path.join(REPO, "tests", "golden", "dino_pnp_kat.npz"))
Q = z["points2d"]
pairs = []
for i, j in itertools.combinations(range(36), 2):
    vis = np.flatnonzero(np.any(Q[i] != -1, axis=0) & np.any(Q[j] != -1, axis=0))
    pairs.append((np.ascontiguousarray(Q[i][:, vis]), np.ascontiguousarray(Q[j][:, vis])))
ctx = _ffi.Context(0)
captured = {}
orig = twoview.gold_standard_arrays


def spy(Fs, pl, pr, off, **kw):
    out = orig(Fs, pl, pr, off, **kw)
    captured["off"], captured["info"] = off, out[3]
    return out


twoview.gold_standard_arrays = spy
parallel.run_pairs(probe_c4._Solo(), pairs, 1000, parallel.GpuPairBatchSolver(ctx, 1000),
                   refine=parallel.GpuPairRefiner(ctx, z["K_last"], fused=False))
n = np.diff(captured["off"])
it = captured["info"]["iterations"]
print("pairs", len(n), "n: max", n.max(), "mean %.1f" % n.mean(), ">64:", int((n > 64).sum()), ">256:", int((n > 256).sum()))
print("iterations: max", it.max(), "mean %.1f" % it.mean(), "hist", np.bincount(np.minimum(it, 60)).tolist())
top = np.argsort(-it)[:10]
print("slowest pairs (n, iterations, accepted, status):", [(int(n[k]), int(it[k]), int(captured["info"]["accepted"][k]), int(captured["info"]["status"][k])) for k in top])
