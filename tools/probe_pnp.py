"""C3 (PnP DLT, M = 500, 30 % outliers, 50 000 hypotheses) repeated, for kernel traces."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import ransac, synth  # noqa: E402


def main():
    X, _, y, _, _, _ = synth.pnp_scene(500, 0.30, seed=3)
    thr = (1.5 / 800.0) ** 2
    H = int(os.environ.get("PROBE_H", 50_000))
    ts = []
    for r in range(int(os.environ.get("PROBE_RUNS", 20))):
        t = time.perf_counter()
        out = ransac.ransac_pnp(X, y, X, y, H, thr, 6, sampler="philox", seed=11 + r)
        ts.append(time.perf_counter() - t)
    print({"best_ms": min(ts) * 1e3, "consensus": int(out[5])})


if __name__ == "__main__":
    main()
