"""Long counting launches for the effective-clock PMC pass (MI355X_MICROARCH.md "DVFS
give-back": clock = GRBM_GUI_ACTIVE / 8 / kernel time, trustworthy on dispatches >= 0.3 ms).
C5-sized runs (N = 10 000, 1e6 hypotheses: a ~5 ms counting launch), back to back."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, synth  # noqa: E402


def main():
    n, H = 10_000, 1_000_000
    p1, p2, _ = synth.two_view(n, 0.6, seed=5)
    ctx = _ffi.Context(0)
    plan = _ffi.F8Plan(ctx, n, H)
    plan.set_points(p1, p2)
    for r in range(int(os.environ.get("PROBE_RUNS", 40))):
        plan.run(H, mode=_ffi.SAMPLER_PHILOX, seed=r)
    r, _ = plan.result()
    print("best_count", r.best_count)
    plan.close()


if __name__ == "__main__":
    main()
