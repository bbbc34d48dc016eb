"""Time the GPU CPython stream (rs_py_shuffle_tuples_gpu) against the host replay at C3's
size (500 points, 6-point samples, 5e4 trials) and a larger set; one JSON line per case."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi  # noqa: E402

for n, k, count in ((500, 6, 50000), (2000, 6, 50000)):
    key, pos = _ffi.py_seed(0)
    _ffi.py_shuffle_tuples_gpu(key, pos, n, k, 1000)
    tg = []
    for _ in range(5):
        t = time.perf_counter()
        g = _ffi.py_shuffle_tuples_gpu(key, pos, n, k, count)
        tg.append(time.perf_counter() - t)
    t = time.perf_counter()
    h = _ffi.py_shuffle_tuples(key, pos, n, k, count)
    th = time.perf_counter() - t
    same = bool(np.array_equal(g[0], h[0]) and g[2] == h[2] and np.array_equal(g[1], h[1]))
    print(json.dumps({"n": n, "k": k, "count": count, "gpu_ms": 1e3 * min(tg),
                      "host_ms": 1e3 * th, "same": same}), flush=True)
