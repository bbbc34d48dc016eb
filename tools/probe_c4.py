"""C4: all C(36,2) pairs of the Dino ring (BAdino2 observations), RANSAC-F + gold standard +
E / relative pose per pair on one GPU, repeated, for kernel traces."""
import itertools
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
sys.path.insert(0, REPO)
from tsbb15_amd import _ffi, parallel  # noqa: E402


class _Solo:
    rank, world = 0, 1

    def allgather_bytes(self, b):
        return [b]


def main():
    z = np.load(os.path.join(REPO, "tests", "golden", "dino_pnp_kat.npz"))
    Q = z["points2d"]
    pairs = []
    for i, j in itertools.combinations(range(36), 2):
        vis = np.flatnonzero(np.any(Q[i] != -1, axis=0) & np.any(Q[j] != -1, axis=0))
        pairs.append((np.ascontiguousarray(Q[i][:, vis]), np.ascontiguousarray(Q[j][:, vis])))
    ctx = _ffi.Context(0)
    solver = parallel.GpuPairBatchSolver(ctx, 1000)
    refiner = None if os.environ.get("PROBE_NOREFINE") else parallel.GpuPairRefiner(
        ctx, z["K_last"], fused=not os.environ.get("PROBE_UNFUSED"))
    ts = []
    for _ in range(int(os.environ.get("PROBE_RUNS", 10))):
        t = time.perf_counter()
        parallel.run_pairs(_Solo(), pairs, 1000, solver, refine=refiner)
        ts.append(time.perf_counter() - t)
    print({"best_ms": min(ts) * 1e3, "median_ms": sorted(ts)[len(ts) // 2] * 1e3})


if __name__ == "__main__":
    main()
