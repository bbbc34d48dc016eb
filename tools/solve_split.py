"""Device time of the fused [tail | solve] launch split into its halves (C2 workload).

A run issued right after rs_f8_plan_result has no pending tail, so its launch is the solve
alone; back-to-back runs carry the previous run's tail.  Prints both averages (HIP events,
timing level 2) and the counting kernel for scale.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, synth  # noqa: E402


def main():
    n, H = int(os.environ.get("SWEEP_N", 2000)), int(os.environ.get("SWEEP_H", 100000))
    p1, p2, _ = synth.two_view(n, 0.3, seed=1)
    ctx = _ffi.Context(0)
    plan = _ffi.F8Plan(ctx, n, H)
    plan.set_points(p1, p2)
    plan.set_timing(2, 1)
    solo = []
    for r in range(25):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=r)
        plan.result()
        if r >= 5:
            solo.append(plan.kernel_ms()["solve_ms"])
    tail = []
    for r in range(10):  # a full run, then a 64-hypothesis run whose launch carries its tail
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=200 + r)
        plan.run(64, mode=_ffi.SAMPLER_PHILOX, seed=300 + r)
        plan.result()
        tail.append(plan.kernel_ms()["solve_ms"])
    for r in range(25):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=100 + r)
    plan.result()
    km = plan.kernel_ms(20)
    print({"solve_only_ms": sum(solo) / len(solo), "tail_only_ms": sum(tail[2:]) / len(tail[2:]),
           "tail_plus_solve_ms": km["solve_ms"],
           "count_ms": km["count_ms"], "run_total_ms": km["total_ms"]})


if __name__ == "__main__":
    main()
