"""C4 pair selection records (best index / count / std / norm / candidates, F) of all 630 Dino
ring pairs, saved to gpurun_out/<name>.npy: bitwise comparison of two libraries."""
import itertools
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, pairs as pm  # noqa: E402

z = np.load(os.path.join(REPO, "tests", "golden", "dino_pnp_kat.npz"))
Q = z["points2d"]
P = []
for i, j in itertools.combinations(range(36), 2):
    vis = np.flatnonzero(np.any(Q[i] != -1, axis=0) & np.any(Q[j] != -1, axis=0))
    if len(vis) >= 8:
        P.append((Q[i][:, vis], Q[j][:, vis]))
off = np.zeros(len(P) + 1, dtype=np.int64)
off[1:] = np.cumsum([p[0].shape[1] for p in P])
res, inl = pm.ransac_pairs_raw(np.hstack([p[0] for p in P]), np.hstack([p[1] for p in P]), off,
                               1000, ctx=_ffi.Context(0))
np.save(os.path.join(REPO, "gpurun_out", sys.argv[1] + ".npy"), res)
print(sys.argv[1], "pairs", len(P), "candidates", int(res["n_candidates"].sum()))
