"""Launch-type-pure workloads for PMC passes over k_f8_tail_solve (C2 sizes).

  PROBE=solve: every launch is a solve alone (each run waits for its result first)
  PROBE=tail:  every other launch is the tail of a full run plus a 64-hypothesis solve
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, synth  # noqa: E402


def main():
    n, H = 2000, 100_000
    p1, p2, _ = synth.two_view(n, 0.3, seed=1)
    ctx = _ffi.Context(0)
    plan = _ffi.F8Plan(ctx, n, H)
    plan.set_points(p1, p2)
    mode = os.environ.get("PROBE", "solve")
    for r in range(30):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=r)
        if mode == "tail":
            plan.run(64, mode=_ffi.SAMPLER_PHILOX, seed=1000 + r)
        plan.result()
    plan.close()


if __name__ == "__main__":
    main()
