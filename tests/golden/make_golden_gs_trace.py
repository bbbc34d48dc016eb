"""Generate tests/golden/gs_trace.npz -- the path scipy's TRF takes in the reference's gold
standard (fun.py:358) on the noisy Dino pair and the s300 synthetic pair.

Runs ONLY in the build container (imports the reference exactly as make_golden.py does,
import-only cv2 stub, BLAS threads = 1).  From the reference's own starting point (C1_init,
X_init in twoview.npz, themselves reference output) it runs

    least_squares(lab3.fmatrix_residuals_gs, params, xtol=2.22e-14, tr_solver='lsmr',
                  args=(pl, pr))                                           (fun.py:358)

with the reference's residual function wrapped to record every evaluation made OUTSIDE the
finite-difference Jacobian (scipy's approx_derivative is wrapped to tell them apart): the
parameter vector x_k and 0.5 ||f(x_k)||^2 of every such evaluation, x_k in full for the first
48 and about 64 more spread over the run, f(x_0) in full, and the final result.  A replay that feeds
scipy the same residual / Jacobian bits follows the same path; where it first leaves it is
the divergence tests/test_gpu_twoview.py reports.

Usage:  python tests/golden/make_golden_gs_trace.py   (about a minute)
"""
from __future__ import annotations

import os
import sys

os.environ["OPENBLAS_NUM_THREADS"] = "1"
os.environ["OMP_NUM_THREADS"] = "1"

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference  # noqa: E402

FULL_FIRST, FULL_EVERY = 48, 16


def trace_run(lab3, pl, pr, C1, X):
    from scipy.optimize import least_squares
    lsq_mod = sys.modules["scipy.optimize._lsq.least_squares"]
    rec = {"x": [], "cost": [], "in_jac": False}
    real_ad = lsq_mod.approx_derivative

    def ad(*a, **k):
        rec["in_jac"] = True
        try:
            return real_ad(*a, **k)
        finally:
            rec["in_jac"] = False

    def fun(x, a, b):
        f = lab3.fmatrix_residuals_gs(x, a, b)
        if not rec["in_jac"]:
            rec["x"].append(x.copy())
            rec["cost"].append(0.5 * float(f @ f))
        return f

    lsq_mod.approx_derivative = ad
    try:
        params = np.hstack((C1.ravel(), X.ravel()))
        f0 = lab3.fmatrix_residuals_gs(params, pl, pr)
        res = least_squares(fun, params, xtol=2.22e-14, tr_solver='lsmr', args=(pl, pr))
    finally:
        lsq_mod.approx_derivative = real_ad
    n = len(rec["x"])
    every = FULL_EVERY * max(1, n // (64 * FULL_EVERY))
    keep = sorted(set(range(min(FULL_FIRST, n))) | set(range(0, n, every)) | {n - 1})
    C1g = res.x[:12].reshape(3, 4)
    C2g = np.zeros((3, 4)); C2g[:3, :3] = np.eye(3)
    return {"x0": params, "f0": f0, "costs": np.array(rec["cost"]),
            "kept_idx": np.array(keep, np.int64), "kept_x": np.stack([rec["x"][i] for i in keep]),
            "x_final": res.x, "cost_final": float(res.cost), "nfev": int(res.nfev),
            "njev": int(res.njev), "status": int(res.status),
            "F_gold": lab3.fmatrix_from_cameras(C1g, C2g)}


def main():
    lab3, fun, ransac, correspondences = import_reference()
    tv = np.load(os.path.join(HERE, "twoview.npz"))
    c1 = np.load(os.path.join(HERE, "dino_c1.npz"))
    out = {}
    cases = {
        "noisy": (c1["noisy_p1"][:, c1["noisy_full_S_ransac"]],
                  c1["noisy_p2"][:, c1["noisy_full_S_ransac"]]),
        "s300": (tv["gs_s300_p1"][:, tv["gs_s300_S_ransac"]],
                 tv["gs_s300_p2"][:, tv["gs_s300_S_ransac"]]),
    }
    for tag, (pl, pr) in cases.items():
        r = trace_run(lab3, pl, pr, tv[f"gs_{tag}_C1_init"], tv[f"gs_{tag}_X_init"])
        # the traced run IS the reference's gold standard: its end must be the stored one
        assert np.array_equal(r["F_gold"], tv[f"gs_{tag}_F_gold"]), tag
        for k, v in r.items():
            out[f"{tag}_{k}"] = v
        print(tag, "nfev", r["nfev"], "njev", r["njev"], "cost", r["cost_final"], flush=True)
    np.savez_compressed(os.path.join(HERE, "gs_trace.npz"), **out)
    # the TRF path depends on the OpenBLAS kernels picked for this CPU: record them, so the
    # bit-equality tests can tell a different host from a regression
    import json
    import scipy
    import threadpoolctl
    blas = [d for d in threadpoolctl.threadpool_info() if d.get("user_api") == "blas"][0]
    with open(os.path.join(HERE, "gs_trace_blas.json"), "w") as f:
        json.dump({"note": "BLAS that tests/golden/gs_trace.npz was recorded and retraced with "
                           "(the build container); the bit-equality of a TRF path holds only "
                           "under the same OpenBLAS kernel choice",
                   "internal_api": blas["internal_api"], "version": blas["version"],
                   "architecture": blas["architecture"], "numpy": np.__version__,
                   "scipy": scipy.__version__}, f, indent=1)


if __name__ == "__main__":
    main()
