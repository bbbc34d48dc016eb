"""Five-point E-RANSAC at the bench's C2 shape (20 000 samples, N = 2 000), 10 timed calls."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import essential, synth  # noqa: E402

p1, p2, _ = synth.two_view(2000, 0.3, seed=1)
ts = []
for _ in range(10):
    t = time.perf_counter()
    r = essential.ransac_e(p1, p2, synth.K_SYNTH, samples=20000, seed=1)
    ts.append(time.perf_counter() - t)
print({"ms_min": 1e3 * min(ts)})
