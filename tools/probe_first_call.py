"""First-call cost of the parity drop-in at C2 (fun.ransac_f, N = 2 000, H = 1e5): a fresh
context's first call (jump polynomials cold), its warm calls, then a second fresh context
(jump polynomials cached in the process) -- where the first call's extra time goes."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, fun, synth  # noqa: E402

p1, p2, _ = synth.two_view(2000, 0.3, seed=1)
H = 100_000


def call(ctx):
    t = time.perf_counter()
    fun.ransac_f(p1, p2, r=H, rng=np.random.RandomState(0), ctx=ctx)
    return 1e3 * (time.perf_counter() - t)


t = time.perf_counter()
_ffi.Context(0).close()  # HIP runtime up, the parse kernels' code object loaded
t0 = 1e3 * (time.perf_counter() - t)
t = time.perf_counter()
c1 = _ffi.Context(0)
tc = 1e3 * (time.perf_counter() - t)
h0 = _ffi.np_host_stats()
f1 = call(c1)
h1 = _ffi.np_host_stats()
w = [call(c1) for _ in range(3)]
c1.close()
c2 = _ffi.Context(0)
h2 = _ffi.np_host_stats()
f2 = call(c2)
h3 = _ffi.np_host_stats()
w2 = [call(c2) for _ in range(3)]
c2.close()
# a process that has run the parity path before, at another N: the new N's own first-call
# cost (jump polynomials for the new chunk length, parse buffers), as the bench measures it
q1, q2, _ = synth.two_view(1000, 0.3, seed=2)
c3 = _ffi.Context(0)
fun.ransac_f(q1, q2, r=20_000, rng=np.random.RandomState(0), ctx=c3)
c3.close()
c4 = _ffi.Context(0)
h4 = _ffi.np_host_stats()
f4 = call(c4)
h5 = _ffi.np_host_stats()
c4.close()
print({"new_n_first_ms": f4, "new_n_host_jump_ms": h5[0] - h4[0]})
print({"first_context_ms": t0, "context_ms": tc, "first_ms": f1, "first_host_jump_ms": h1[0] - h0[0], "warm_ms": min(w),
       "second_context_first_ms": f2, "second_context_host_jump_ms": h3[0] - h2[0],
       "second_context_warm_ms": min(w2)})
