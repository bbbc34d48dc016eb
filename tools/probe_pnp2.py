"""C3 PnP-RANSAC (DLT, M = 500, 30 % outliers, 5e4 hypotheses, Philox) with the HIP-event split
of rs_pnp_timing: best solve / count kernel times over 10 calls, and the results of a fixed seed
(winner, consensus) so A/B libraries (RSAMD_LIB) can be compared.  One JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tsbb15-3d-reconstruction-project_amd"))
from tsbb15_amd import _ffi, ransac, synth  # noqa: E402


def main():
    X, _, y, _, _, _ = synth.pnp_scene(500, 0.30, seed=3)
    thr = (1.5 / 800.0) ** 2
    ctx = _ffi.default_context()
    run = lambda s: ransac.ransac_pnp(X, y, X, y, 50_000, thr, 6, sampler="philox", seed=s, ctx=ctx)
    for _ in range(3):
        run(11)
    _ffi.pnp_timing(ctx, 1)
    ks, kc, wall = [], [], []
    for _ in range(10):
        t = time.perf_counter()
        out = run(11)
        wall.append((time.perf_counter() - t) * 1e3)
        a, b = _ffi.pnp_timing(ctx, 1)
        ks.append(a)
        kc.append(b)
    _ffi.pnp_timing(ctx, 0)
    print(json.dumps({"lib": os.environ.get("RSAMD_LIB", "product"), "solve_ms": min(ks),
                      "count_ms": min(kc), "wall_ms": min(wall), "best": int(out[4]),
                      "count": int(out[5]), "R": out[0].ravel().tolist()}), flush=True)


if __name__ == "__main__":
    main()
