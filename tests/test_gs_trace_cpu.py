"""The gold-standard argument of DESIGN.md 2.2 / INTEGRATION.md 2, pinned on the CPU.

fun.py:358 runs scipy's TRF (xtol = 2.22e-14, tr_solver = 'lsmr') over lab3.fmatrix_residuals_gs
with a 2-point Jacobian.  Two facts carry the (f)-1 parity claim:

  * with the GPU kernel's arithmetic (the projection C @ [X; 1] in numpy's dgemm FMA order,
    the Jacobian in scipy's column-major layout) the whole reference trace recorded in the
    build container (tests/golden/gs_trace.npz: 1 067 evaluations on the noisy Dino pair) is
    retraced evaluation for evaluation, and the final x is bit-equal;
  * the reference's own end point is chaotic in its start: a 1e-15 relative change of x0
    moves F_gold by >= 1e-4 (3.07e-4 measured, after 56 evaluations instead of 1 067), so no
    implementation whose start differs in the last bits (GPU SVD / root finder vs LAPACK /
    np.roots) can reach the north_star's 1e-6 on the noisy pair.

The residual / Jacobian are tools/gs_trace_cpu.py's (numpy, dgemm mode).  The first fact holds
only under the BLAS the trace was recorded with (tests/golden/gs_trace_blas.json).
"""
import os
import sys

import numpy as np
import pytest
from threadpoolctl import threadpool_limits

from conftest import REPO, golden, trace_blas_matches

sys.path.insert(0, os.path.join(REPO, "tools"))
import gs_trace_cpu as gst  # noqa: E402


def _noisy():
    c1 = golden("dino_c1.npz")
    S = c1["noisy_full_S_ransac"]
    return c1["noisy_p1"][:, S], c1["noisy_p2"][:, S]


def _trf(x0, pl, pr):
    from scipy.optimize import least_squares
    xs, cs = [], []

    def fun(x):
        f = gst.resid(x, pl, pr, "dgemm")
        xs.append(x.copy())
        cs.append(0.5 * float(f @ f))
        return f

    # one BLAS thread, as the trace was recorded (make_golden_gs_trace.py): the threaded
    # OpenBLAS kernels sum in another order
    with threadpool_limits(limits=1, user_api="blas"):
        res = least_squares(fun, x0, jac=lambda x: gst.jac(x, pl, pr, "dgemm"), xtol=2.22e-14,
                            tr_solver="lsmr")
    return res, xs, cs


def test_dgemm_arithmetic_retraces_the_reference_trace():
    same, desc = trace_blas_matches()
    if not same:
        pytest.skip("the TRF path follows the host BLAS kernels; " + desc)
    tr = golden("gs_trace.npz")
    pl, pr = _noisy()
    x0 = tr["noisy_x0"]
    assert np.array_equal(gst.resid(x0, pl, pr, "dgemm"), tr["noisy_f0"])
    res, xs, cs = _trf(x0, pl, pr)
    assert res.nfev == int(tr["noisy_nfev"]) == 1067
    assert len(cs) == len(tr["noisy_costs"])
    assert all(a == b for a, b in zip(cs, tr["noisy_costs"]))        # every evaluation's cost
    for k, xk in zip(tr["noisy_kept_idx"], tr["noisy_kept_x"]):      # the recorded x_k
        assert np.array_equal(xs[int(k)], xk), int(k)
    assert np.array_equal(res.x, tr["noisy_x_final"])
    assert res.cost == float(tr["noisy_cost_final"])
    assert gst.dF(res.x, tr["noisy_F_gold"]) == 0.0


def test_reference_end_point_is_chaotic_in_its_start():
    tr = golden("gs_trace.npz")
    pl, pr = _noisy()
    x0 = tr["noisy_x0"].copy()
    rs = np.random.RandomState(1)
    x0[12:] *= 1.0 + 1e-15 * rs.uniform(-1, 1, x0.size - 12)   # last-bit changes of the points
    assert np.abs(x0 - tr["noisy_x0"]).max() <= 1e-12 * np.abs(tr["noisy_x0"]).max()
    res, _, _ = _trf(x0, pl, pr)
    dF = gst.dF(res.x, tr["noisy_F_gold"])
    assert dF >= 1e-4, dF        # 100x the north_star's 1e-6: unreachable by the reference itself
