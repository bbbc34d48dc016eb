"""Generate tests/golden/full_c3.npz -- config C3 at full size in the exact CPython stream.

C3: PnP, M = 500 points (tsbb15_amd.synth.pnp_scene(500, 0.30, seed=3), y = K^-1 [u, v, 1],
0.5 px noise, 30 % outliers), 50 000 trials of the intended ransac.ransac_robust
(ransac.py:37-113: gen_rnd_indices(500, 6) on random.seed(0)'s stream, ransac.py:12-19; the
6-point DLT of pnp.py:132-160; consensus e <= thresh inclusive, ransac.py:104-105; the first
largest D_med consensus wins, ransac.py:108), thresh = (1.5 / 800)^2.

The reference's own ransac_robust cannot run (it raises at ransac.py:77),
so the expected values come from the oracle restatement oracle/pnp_ref.ransac_pnp, itself
pinned to the reference's gen_rnd_indices output (ransac_misc.json) and its
camera_resectioning poses (dino_pnp_kat.npz).  Written: every trial's D_med consensus size,
the winner, both consensus sets, R, t, and the CPython MT state after the loop.

Usage:  python tests/golden/make_golden_c3.py   (about half a minute, BLAS 1 thread)
"""
import os
import random
import sys

os.environ["OPENBLAS_NUM_THREADS"] = "1"
import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
from oracle import pnp_ref  # noqa: E402
from tsbb15_amd import synth  # noqa: E402

R_TRIALS = 50_000
THRESH = (1.5 / 800.0) ** 2


def main():
    X, _, y, Rt, tt, truth = synth.pnp_scene(500, 0.30, seed=3)
    rng = random.Random(0)
    R, t, im, ih, best, counts = pnp_ref.ransac_pnp(y, X, y, X, R_TRIALS, THRESH, 6, rng=rng,
                                                    trace=True)
    st = rng.getstate()
    key = np.array(st[1][:624], np.uint32)
    pos = int(st[1][624])
    np.savez_compressed(os.path.join(HERE, "full_c3.npz"), X=X, y=y, r=R_TRIALS, thresh=THRESH,
                        counts=counts.astype(np.int16), best=best, R=R, t=t, inl_med=im,
                        inl_high=ih, py_key_out=key, py_pos_out=pos)
    print("best", best, "count", counts.max(), "inliers", len(im), "true-inlier share",
          truth[im].mean())


if __name__ == "__main__":
    main()
