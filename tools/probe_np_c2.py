"""The parity-mode C2 run (numpy-exact stream parsed on the GPU + the F pipeline), repeated:
a clean process for rocprofv3 kernel traces / PMC passes of the parse kernels, and the HIP-event
step split of rs_np_timing.  Every parse launch in it is a C2 launch (N = 2000, 1e5 hypotheses,
np.random.seed(0)); --n / --hyps / --outliers / --seed select another pair (C5: 10000 / 1e6 /
0.6 / 5).  Prints one JSON line (per-run wall times and the last timed split).
Usage: python tools/probe_np_c2.py [--reps 5] [--n 2000] [--hyps 100000]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))

from tsbb15_amd import _ffi, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--hyps", type=int, default=100_000)
    ap.add_argument("--outliers", type=float, default=0.30)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--split", action="store_true", help="also one run with step events")
    a = ap.parse_args()
    ctx = _ffi.Context(0)
    p1, p2, _ = synth.two_view(a.n, a.outliers, seed=a.seed)
    plan = _ffi.F8Plan(ctx, a.n, a.hyps)
    plan.set_points(p1, p2)
    key0, pos0 = _ffi.np_seed(0)
    walls = []
    for _ in range(a.reps):
        t = time.perf_counter()
        plan.run_np(a.hyps, key0, pos0)
        r, _ = plan.result()
        walls.append((time.perf_counter() - t) * 1e3)
    out = {"n": a.n, "hyps": a.hyps, "wall_ms": walls, "best_index": int(r.best_index),
           "best_count": int(r.best_count)}
    if a.split:
        _ffi.np_timing(ctx, 1)
        t = time.perf_counter()
        plan.run_np(a.hyps, key0, pos0)
        plan.result()
        out["split_wall_ms"] = (time.perf_counter() - t) * 1e3
        out["split_ms"], out["bytes"], out["segments"] = _ffi.np_timing(ctx, 0)
    print(json.dumps(out), flush=True)
    plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
