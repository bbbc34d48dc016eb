"""Time the GPU parity stream (rs_np_choice_tuples_gpu) against the host replay at C2 / C5
sizes; prints one JSON line per case."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi  # noqa: E402


def best(fn, reps):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        t.append(time.perf_counter() - t0)
    return min(t), r


for n, count, reps in ((2000, 100000, 5), (10000, 20000, 3), (257, 10000, 5), (37, 100000, 3)):
    st = np.random.RandomState(1).get_state()
    key, pos = np.asarray(st[1], np.uint32), int(st[2])
    tg, g = best(lambda: _ffi.np_choice_tuples_gpu(key, pos, n, 8, count), reps)
    th, h = best(lambda: _ffi.np_choice_tuples(key, pos, n, 8, count), 1)
    same = bool(np.array_equal(g[0], h[0]) and g[2] == h[2] and np.array_equal(g[1], h[1]))
    print(json.dumps({"n": n, "count": count, "gpu_ms": tg * 1e3, "host_ms": th * 1e3,
                      "gpu_hyp_s": count / tg, "host_hyp_s": count / th, "same": same}),
          flush=True)
