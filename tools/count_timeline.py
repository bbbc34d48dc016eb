"""Wave timeline of the counting kernel (RSAMD_TSTAMP): when waves start and end within a
C2 launch, to split the launch into ramp, steady state and drain.

  RSAMD_TSTAMP=/tmp/ts.bin python tools/count_timeline.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, synth  # noqa: E402


def main():
    path = os.environ["RSAMD_TSTAMP"]
    if os.path.exists(path):
        os.remove(path)
    n, H = 2000, 100_000
    p1, p2, _ = synth.two_view(n, 0.3, seed=1)
    ctx = _ffi.Context(0)
    plan = _ffi.F8Plan(ctx, n, H)
    plan.set_points(p1, p2)
    runs = 8
    for r in range(runs):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=r)
        plan.result()
    raw = np.fromfile(path, dtype=np.uint64).reshape(runs, -1, 2)
    for r in (runs - 2, runs - 1):
        t = raw[r]
        t = t[t[:, 0] > 0].astype(np.float64) * 10.0 / 1000.0  # 100 MHz ticks -> us
        t0 = t[:, 0].min()
        st, en = t[:, 0] - t0, t[:, 1] - t0
        dur = en - st
        q = lambda a, p: float(np.percentile(a, p))
        print({"waves": len(t), "launch_us": round(en.max(), 1),
               "start_p0_p50_p90_max": [round(q(st, x), 1) for x in (0, 50, 90, 100)],
               "end_min_p10_p50_max": [round(q(en, x), 1) for x in (0, 10, 50, 100)],
               "dur_p10_p50_p90": [round(q(dur, x), 1) for x in (10, 50, 90)]})
        # resident waves over time
        grid = np.arange(0, en.max() + 1, 2.0)
        live = [int(((st <= g) & (en > g)).sum()) for g in grid]
        print("live waves every 2 us:", live[:8], "...", live[-12:])


if __name__ == "__main__":
    main()
