"""C4 gold standard alone: the refiner's batch (captured from one run_pairs) timed at several
max_iter values -- the launch's fixed part (triangulation, set-up) against its per-iteration
part."""
import itertools
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_c4  # noqa: E402
from tsbb15_amd import _ffi, parallel, twoview  # noqa: E402

z = np.load(os.path.join(probe_c4.REPO, "tests", "golden", "dino_pnp_kat.npz"))
Q = z["points2d"]
pairs = []
for i, j in itertools.combinations(range(36), 2):
    vis = np.flatnonzero(np.any(Q[i] != -1, axis=0) & np.any(Q[j] != -1, axis=0))
    pairs.append((np.ascontiguousarray(Q[i][:, vis]), np.ascontiguousarray(Q[j][:, vis])))
ctx = _ffi.Context(0)
cap = {}
orig = twoview.gold_standard_arrays


def spy(Fs, pl, pr, off, **kw):
    cap.update(Fs=np.array(Fs), pl=np.array(pl), pr=np.array(pr), off=np.array(off))
    return orig(Fs, pl, pr, off, **kw)


twoview.gold_standard_arrays = spy
parallel.run_pairs(probe_c4._Solo(), pairs, 1000, parallel.GpuPairBatchSolver(ctx, 1000),
                   refine=parallel.GpuPairRefiner(ctx, z["K_last"], fused=False))
twoview.gold_standard_arrays = orig
for mi in (1, 2, 3, 5, 10, 500):
    ts = []
    for _ in range(15):
        t = time.perf_counter()
        orig(cap["Fs"], cap["pl"], cap["pr"], cap["off"], max_iter=mi, ctx=ctx, want_points=False)
        ts.append(time.perf_counter() - t)
    print("max_iter %3d: %.3f ms" % (mi, 1e3 * min(ts)))
