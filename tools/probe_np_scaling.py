"""Parity-stream parse time against the number of hypotheses parsed at once (N = 2 000):
one parse covering several consecutive RANSAC runs' worth of the np.random stream."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi  # noqa: E402

st = np.random.RandomState(0).get_state()
key, pos = np.asarray(st[1], np.uint32), int(st[2])
for count in (100_000, 200_000, 400_000, 800_000):
    t = []
    for _ in range(4):
        t0 = time.perf_counter()
        _ffi.np_choice_tuples_gpu(key, pos, 2000, 8, count)
        t.append(time.perf_counter() - t0)
    best = min(t[1:])
    print(json.dumps({"count": count, "ms": best * 1e3, "hyp_s": count / best}), flush=True)
