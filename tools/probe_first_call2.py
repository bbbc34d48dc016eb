"""The bench's first parity call, alone under a HIP API trace: a context runs a Philox F-RANSAC
first (as the bench's headline does), then a fresh context's first fun.ransac_f at C2 is timed
between two markers (hipDeviceSynchronize calls) so the trace shows what it spends."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, fun, synth  # noqa: E402

p1, p2, _ = synth.two_view(2000, 0.3, seed=1)
H = 100_000
ctx = _ffi.Context(0)
plan = _ffi.F8Plan(ctx, 2000, H)
plan.set_points(p1, p2)
for _ in range(3):
    plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=1, thresh=1.5)
    plan.result()
hip = ctypes.CDLL("libamdhip64.so")
hip.hipDeviceSynchronize()
cnew = _ffi.Context(0)
hip.hipDeviceSynchronize()
t = time.perf_counter()
fun.ransac_f(p1, p2, r=H, rng=np.random.RandomState(0), ctx=cnew)
first = time.perf_counter() - t
hip.hipDeviceSynchronize()
t = time.perf_counter()
fun.ransac_f(p1, p2, r=H, rng=np.random.RandomState(0), ctx=cnew)
warm = time.perf_counter() - t
print({"first_ms": first * 1e3, "warm_ms": warm * 1e3})
