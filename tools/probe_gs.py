"""Gold-standard launch time against the LM iteration cap (C2 winner, 1 318 inliers; and the
C4 batch): the slope is the cost of one LM iteration, the intercept the optimal triangulation
and the set-up."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
sys.path.insert(0, REPO)
from tsbb15_amd import fun, synth, twoview  # noqa: E402


def best(f, reps=5):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        out = f()
        ts.append(time.perf_counter() - t)
    return min(ts) * 1e3, out


def main():
    p1, p2, _ = synth.two_view(2000, 0.30, seed=1)
    res = fun.ransac_f(p1, p2, r=10_000, rng=np.random.RandomState(0))
    a, b = p1[:, res.inliers], p2[:, res.inliers]
    for it in (1, 2, 3, 5, 10, 20):
        ms, g = best(lambda: twoview.gold_standard_batch(res.F[None], [a], [b], max_iter=it)[0])
        print({"max_iter": it, "ms": round(ms, 3), "iterations": g.iterations, "cost": g.cost})


if __name__ == "__main__":
    main()
