"""Parity-stream parse time at the chunk length RSAMD_NP_KW selects (unset: automatic), for
C2 (N = 2 000, 1e5 tuples) and a C5-shaped stream (N = 10 000, 2e4 tuples); the first call
of each case is checked against the host replay.  One JSON line per case."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi  # noqa: E402

kw = os.environ.get("RSAMD_NP_KW", "auto")
cases = ((2000, 100000, 6), (10000, 20000, 4))
only = os.environ.get("NP_ONLY")  # restrict to one N (kernel traces)
for n, count, reps in cases:
    if only and int(only) != n:
        continue
    st = np.random.RandomState(1).get_state()
    key, pos = np.asarray(st[1], np.uint32), int(st[2])
    g = _ffi.np_choice_tuples_gpu(key, pos, n, 8, count)
    h = _ffi.np_choice_tuples(key, pos, n, 8, count)
    same = bool(np.array_equal(g[0], h[0]) and g[2] == h[2] and np.array_equal(g[1], h[1]))
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _ffi.np_choice_tuples_gpu(key, pos, n, 8, count)
        t.append(time.perf_counter() - t0)
    print(json.dumps({"kw": kw, "n": n, "count": count, "gpu_ms": min(t) * 1e3,
                      "med_ms": sorted(t)[len(t) // 2] * 1e3, "same": same}), flush=True)
