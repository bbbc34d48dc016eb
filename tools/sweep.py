"""A/B sweep of counting-kernel knobs in one process (env read at plan creation).

  python tools/sweep.py [RSAMD_WAVES=4096,8192 RSAMD_COUNT=fp32,fp64 ...]
"""
import itertools
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
import numpy as np  # noqa: E402

from tsbb15_amd import _ffi, synth  # noqa: E402


def main():
    grid = {}
    for arg in sys.argv[1:]:
        k, v = arg.split("=")
        grid[k] = v.split(",")
    n, H, reps = int(os.environ.get("SWEEP_N", 2000)), int(os.environ.get("SWEEP_H", 100000)), 20
    p1, p2, _ = synth.two_view(n, 0.3, seed=1)
    ctx = _ffi.Context(0)
    keys = list(grid)
    ref_counts = None
    for combo in itertools.product(*[grid[k] for k in keys]) if keys else [()]:
        for k, v in zip(keys, combo):
            os.environ[k] = v
        plan = _ffi.F8Plan(ctx, n, H)
        plan.set_points(p1, p2)
        ms = []
        for r in range(reps + 3):
            plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=5)
            plan.result()
            if r >= 3:
                ms.append(plan.kernel_ms())
        c = plan.counts(H)
        same = ref_counts is None or np.array_equal(c, ref_counts)
        ref_counts = c if ref_counts is None else ref_counts
        out = {k: v for k, v in zip(keys, combo)}
        out.update({m: float(np.median([x[m] for x in ms])) for m in ms[0]})
        out["counts_identical"] = bool(same)
        print(json.dumps(out), flush=True)
        plan.close()


if __name__ == "__main__":
    main()
