"""Counting-kernel time at C5 (N = 10 000, 60 % outliers, 1e6 hypotheses) and C2, by HIP
events on the plan's stream; environment knobs select the variant."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, synth  # noqa: E402

ctx = _ffi.Context(0)
for name, n, out, H in (("C2", 2000, 0.3, 100_000), ("C5", 10_000, 0.6, 1_000_000)):
    p1, p2, _ = synth.two_view(n, out, seed=1)
    plan = _ffi.F8Plan(ctx, n, H)
    plan.set_points(p1, p2)
    for i in range(30):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=i)
    plan.result()
    for i in range(20):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=100 + i)
    plan.result()
    km = plan.kernel_ms(last_n=20)
    print(json.dumps({"case": name, "count_ms": km["count_ms"]}), flush=True)
    plan.close()
