"""Wave timeline of the counting kernel (RSAMD_TSTAMP): when waves start and end within a
C2 launch, to split the launch into ramp, steady state and drain, and what makes waves of
equal work take different times (re-test branches taken, XCD, SIMD occupancy at start).

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
    raw = np.fromfile(path, dtype=np.uint64).reshape(runs, -1, 6)
    for r in (runs - 2, runs - 1):
        rec = raw[r]
        rec = rec[rec[:, 0] > 0]
        t = rec[:, :2].astype(np.float64) * 10.0 / 1000.0  # 100 MHz ticks -> us
        t0 = t[:, 0].min()
        st, en = t[:, 0] - t0, t[:, 1] - t0
        dur = en - st
        nre = rec[:, 2].astype(np.int64)
        hw = rec[:, 3].astype(np.int64)
        cyc = (rec[:, 5] - rec[:, 4]).astype(np.float64)      # shader-clock cycles of the wave
        ghz = cyc / np.maximum(1.0, (rec[:, 1] - rec[:, 0]).astype(np.float64)) * 0.1
        xcc = hw & 7
        hwid = hw >> 8
        simd = (hwid >> 4) & 3
        cu = (hwid >> 8) & 15
        se = (hwid >> 13) & 7
        q = lambda a, p: float(np.percentile(a, p))
        print({"waves": len(t), "launch_us": round(en.max(), 1),
               "start_p0_p50_p90_max": [round(q(st, x), 1) for x in (0, 50, 90, 100)],
               "end_min_p10_p50_max": [round(q(en, x), 1) for x in (0, 10, 50, 100)],
               "dur_p10_p50_p90": [round(q(dur, x), 1) for x in (10, 50, 90)],
               "retest_p10_p50_p90_max": [int(q(nre, x)) for x in (10, 50, 90, 100)]})
        # resident waves per SIMD over the launch: the drain is the SIMD-time with few waves
        sid = ((xcc * 8 + se) * 16 + cu) * 4 + simd
        grid = np.arange(0.0, en.max(), 0.25)
        occ = np.zeros((int(sid.max()) + 1, len(grid)), np.int16)
        for a, b, k in zip(st, en, sid):
            occ[k, (grid >= a) & (grid < b)] += 1
        used = occ[np.unique(sid)]
        tot = used.size
        print({"simds": int(len(used)),
               "simd_time_frac_by_resident_waves": {str(w): round(float((used == w).sum()) / tot, 3)
                                                    for w in range(0, 7)},
               "simd_time_frac_7plus": round(float((used >= 7).sum()) / tot, 3),
               "simd_last_wave_end_p10_p50_p90_us": [
                   round(float(np.percentile([en[sid == k].max() for k in np.unique(sid)], x)), 1)
                   for x in (10, 50, 90)]})
        # is the spread of equal-work waves a clock effect or a cycle effect?
        print({"wave_clock_ghz_p10_p50_p90": [round(q(ghz, x), 3) for x in (10, 50, 90)],
               "wave_cycles_p10_p50_p90": [int(q(cyc, x)) for x in (10, 50, 90)],
               "corr(duration, cycles)": round(float(np.corrcoef(dur, cyc)[0, 1]), 3),
               "corr(duration, clock)": round(float(np.corrcoef(dur, ghz)[0, 1]), 3),
               "corr(end, cycles)": round(float(np.corrcoef(en, cyc)[0, 1]), 3)})
        for x in range(8):
            m = xcc == x
            if m.any():
                print("  xcc %d: clock p50 %.3f GHz, cycles p50 %d, dur p50 %.1f us"
                      % (x, np.median(ghz[m]), int(np.median(cyc[m])), np.median(dur[m])))
        first = st < 2.0  # the first round (all resident at once)
        if first.sum() > 10:
            d, k = dur[first], nre[first]
            cy = cyc[first]
            print("first round: cycles p10/p50/p90 %d / %d / %d, corr(cycles, retests) %.2f"
                  % (q(cy, 10), q(cy, 50), q(cy, 90), np.corrcoef(cy, k)[0, 1] if k.std() > 0 else 0.0))
            c = np.corrcoef(d, k)[0, 1] if k.std() > 0 else 0.0
            print("first round: corr(duration, retests) = %.2f" % c)
            for x in range(8):
                m = first & (xcc == x)
                if m.any():
                    print("  xcc %d: waves %d dur p50 %.1f us, retests p50 %d"
                          % (x, m.sum(), np.median(dur[m]), int(np.median(nre[m]))))
            lo, hi = k <= np.percentile(k, 25), k >= np.percentile(k, 75)
            print("  dur p50 at low / high retest quartile: %.1f / %.1f us"
                  % (np.median(d[lo]), np.median(d[hi])))
            # waves sharing a SIMD at the start
            key = (xcc * 8 + se) * 16 * 4 + cu * 4 + simd
            _, inv, cnt = np.unique(key[first], return_inverse=True, return_counts=True)
            per = cnt[inv]
            for v in np.unique(per):
                print("  %d waves on the SIMD: %d waves, dur p50 %.1f us"
                      % (v, (per == v).sum(), np.median(d[per == v])))
        grid = np.arange(0, en.max() + 1, 2.0)
        live = [int(((st <= g) & (en > g)).sum()) for g in grid]
        print("live waves every 2 us:", live[:8], "...", live[-12:])


if __name__ == "__main__":
    main()
