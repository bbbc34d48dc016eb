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
        k0 = st[:, 121]
        if k0.any():
            rel = k0 - k0.min()
            end = rel + kern
            print(f"  chunk start offsets: median {np.median(rel):.3g} max {rel.max():.3g}; last end {end.max():.3g}; "
                  f"chunks starting after {np.percentile(kern, 50):.3g}: {(rel > np.percentile(kern, 50)).sum()}")
            print(f"  distinct hw ids {len(np.unique(st[:, 122]))}")
    sys.exit(0)

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi  # noqa: E402
st = np.random.RandomState(1).get_state()
key, pos = np.asarray(st[1], np.uint32), int(st[2])
n = int(os.environ.get("NP_N", "2000"))
count = int(os.environ.get("NP_COUNT", "100000"))
_ffi.np_choice_tuples_gpu(key, pos, n, 8, count)
print("done")
