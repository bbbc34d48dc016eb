"""Run one C2-sized parity stream with the RSAMD_DIAG library and summarise the per-chunk
tracking statistics (k_np_track): run with RSAMD_LIB=<lib_diag/librsamd.so> RSAMD_NP_STATS=<file>,
or `python tools/np_stats.py --read <file>` to summarise an existing file."""
import os
import sys

import numpy as np

if len(sys.argv) > 2 and sys.argv[1] == "--read":
    raw = np.fromfile(sys.argv[2], dtype=np.int64)
    p = 0
    while p < raw.size:
        n1, C, kW, D = raw[p:p + 4]
        st = raw[p + 4:p + 4 + 128 * C].reshape(C, 128)
        p += 4 + 128 * C
        w = st[:, :96].reshape(C, 16, 6)  # per wave: windows, cyc1, cycN, n1, nN, intervals
        kern = st[:, 120]
        print(f"n1={n1} C={C} kW={kW} D={D}")
        print(f"  kernel cycles per chunk: mean {kern.mean():.3g} max {kern.max():.3g}")
        c1, cN = w[:, :, 1], w[:, :, 2]
        i1, iN = w[:, :, 3], w[:, :, 4]
        print(f"  one-trajectory wave-intervals {i1.sum()/C:.0f} per chunk, {c1.sum()/max(i1.sum(),1):.3g} cycles each")
        print(f"  multi-trajectory wave-intervals {iN.sum()/C:.0f} per chunk, {cN.sum()/max(iN.sum(),1):.3g} cycles each")
        print(f"  busiest wave per chunk: one {c1.max(1).mean():.3g} multi {cN.max(1).mean():.3g} cycles; intervals {w[:,0,5].mean():.0f}")
        e = st[:, 100:111].astype(float)
        if e[:, 7].any():
            cyc = e[:, 0:4].mean(0)
            dr = e[:, 4:7].mean(0)
            print(f"  entry: total {e[:,7].mean():.3g} cycles; several-slot {cyc[0]:.3g} ({dr[0]:.0f} draws), "
                  f"multi-slot fast {cyc[1]:.3g} ({dr[1]:.0f}), one-slot {cyc[2]:.3g} ({dr[2]:.0f}), "
                  f"compaction {cyc[3]:.3g}; exits at t {e[:,8].mean():.0f} with m {e[:,9].mean():.1f}; "
                  f"wave 0 general one-slot batches {e[:,10].mean():.0f} of {dr[2] / 64:.0f}")
        r0, r1 = st[:, 121], st[:, 122]
        if r0.any():
            rel0, rel1 = (r0 - r0.min()) / 100.0, (r1 - r0.min()) / 100.0  # us
            dur = rel1 - rel0
            print(f"  real time (us): start median {np.median(rel0):.1f} max {rel0.max():.1f}; duration mean {dur.mean():.0f} "
                  f"max {dur.max():.0f}; last end {rel1.max():.0f}; clock {kern.mean() / dur.mean() / 1e3:.2f} GHz (memtime / real)")
    sys.exit(0)

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi  # noqa: E402
st = np.random.RandomState(1).get_state()
key, pos = np.asarray(st[1], np.uint32), int(st[2])
n = int(os.environ.get("NP_N", "2000"))
count = int(os.environ.get("NP_COUNT", "100000"))
_ffi.np_choice_tuples_gpu(key, pos, n, 8, count)
print("done")
