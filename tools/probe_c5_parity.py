"""C5 parity-mode run (N = 10 000, 1e6 numpy-exact hypotheses) timed three times after a
1e5 warm-up, to separate first-use host work from the steady state."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, synth  # noqa: E402

ctx = _ffi.default_context()
p1, p2, _ = synth.two_view(10_000, 0.60, seed=5)
plan = _ffi.F8Plan(ctx, 10_000, 1_000_000)
plan.set_points(p1, p2)
key0, pos0 = _ffi.np_seed(0)
t = time.perf_counter()
plan.run_np(100_000, key0, pos0)
plan.result()
print({"warmup_1e5_ms": 1e3 * (time.perf_counter() - t)}, flush=True)
for k in range(3):
    t = time.perf_counter()
    plan.run_np(1_000_000, key0, pos0)
    rp, _ = plan.result()
    print({"run": k, "ms": 1e3 * (time.perf_counter() - t), "best": int(rp.best_index)}, flush=True)
