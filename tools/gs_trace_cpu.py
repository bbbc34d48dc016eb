"""Where the gold-standard TRF path leaves the reference's (tests/golden/gs_trace.npz), on the CPU.

scipy's least_squares (fun.py:358's call) is driven with a residual / 2-point Jacobian of
lab3.fmatrix_residuals_gs computed in a chosen arithmetic, and the evaluated x_k / costs are
compared with the reference trace:

  dgemm   the projection C @ [X; 1] by numpy's dot (OpenBLAS dgemm: per element the FMA
          chain fma(c2, x2, fma(c1, x1, c0 x0)) + c3), i.e. the reference's own bits;
  plain   ((c0 x0 + c1 x1) + c2 x2) + c3 with separate roundings (the round-2 GPU kernel).

Usage: python tools/gs_trace_cpu.py [noisy|s300] [max_nfev]
"""
import os
import sys

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
import numpy as np  # noqa: E402
from scipy.optimize import least_squares  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EPS = float(np.finfo(np.float64).eps) ** 0.5


def proj_left(C, X, mode):
    if mode == "dgemm":
        y = np.dot(C, np.vstack((X, np.ones((1, X.shape[1])))))
        return y[0] / y[2], y[1] / y[2]
    y = [((C[i, 0] * X[0] + C[i, 1] * X[1]) + C[i, 2] * X[2]) + C[i, 3] for i in range(3)]
    return y[0] / y[2], y[1] / y[2]


def resid(x, pl, pr, mode):
    n = pl.shape[1]
    C = x[:12].reshape(3, 4)
    X = x[12:].reshape(n, 3).T
    u, v = proj_left(C, X, mode)
    return np.concatenate((pl[0] - u, pl[1] - v, pr[0] - X[0] / X[2], pr[1] - X[1] / X[2]))


def jac(x, pl, pr, mode):
    n = pl.shape[1]
    sign = (x >= 0).astype(float) * 2 - 1
    h = EPS * sign * np.maximum(1.0, np.abs(x))
    xp = x + h
    dx = xp - x
    f0 = resid(x, pl, pr, mode)
    # the entries a parameter cannot reach are (f - f) / dx = +-0 with dx's sign, as scipy's
    # approx_derivative forms them; it returns the transpose of a C-order (n, m) array, so
    # the Jacobian is Fortran-ordered (BLAS then runs J @ v and J.T @ u column-major)
    J = np.zeros((4 * n, 12 + 3 * n), order="F")
    if ZERO_SIGNS:
        J[:] = 0.0 / dx[None, :]
    C = x[:12].reshape(3, 4)
    X = x[12:].reshape(n, 3).T
    for j in range(12):
        Cp = C.copy().ravel()
        Cp[j] = xp[j]
        u, v = proj_left(Cp.reshape(3, 4), X, mode)
        J[:n, j] = ((pl[0] - u) - f0[:n]) / dx[j]
        J[n:2 * n, j] = ((pl[1] - v) - f0[n:2 * n]) / dx[j]
    idx = np.arange(n)
    for c in range(3):
        Xp = X.copy()
        Xp[c] = xp[12 + 3 * idx + c]
        u, v = proj_left(C, Xp, mode)
        r = np.concatenate((pl[0] - u, pl[1] - v, pr[0] - Xp[0] / Xp[2], pr[1] - Xp[1] / Xp[2]))
        col = 12 + 3 * idx + c
        for q in range(4):
            J[q * n + idx, col] = (r[q * n:(q + 1) * n] - f0[q * n:(q + 1) * n]) / dx[col]
    return J if FORTRAN else np.ascontiguousarray(J)


FORTRAN = os.environ.get("GS_J_ORDER", "F") == "F"
ZERO_SIGNS = os.environ.get("GS_J_ZEROS", "signed") == "signed"


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "noisy"
    tr = np.load(os.path.join(REPO, "tests", "golden", "gs_trace.npz"))
    c1 = np.load(os.path.join(REPO, "tests", "golden", "dino_c1.npz"))
    tv = np.load(os.path.join(REPO, "tests", "golden", "twoview.npz"))
    if tag == "noisy":
        S = c1["noisy_full_S_ransac"]
        pl, pr = c1["noisy_p1"][:, S], c1["noisy_p2"][:, S]
    else:
        S = tv["gs_s300_S_ransac"]
        pl, pr = tv["gs_s300_p1"][:, S], tv["gs_s300_p2"][:, S]
    x0 = tr[f"{tag}_x0"].copy()
    pert = float(os.environ.get("GS_PERTURB", "0"))   # relative perturbation of x0's points
    if pert:
        rs = np.random.RandomState(1)
        x0[12:] *= 1.0 + pert * rs.uniform(-1, 1, x0.size - 12)
    costs, kept_idx, kept_x = tr[f"{tag}_costs"], tr[f"{tag}_kept_idx"], tr[f"{tag}_kept_x"]
    for mode in os.environ.get("GS_MODES", "dgemm,plain").split(","):
        f0 = resid(x0, pl, pr, mode)
        xs, cs = [], []

        def fun(x):
            f = resid(x, pl, pr, mode)
            xs.append(x.copy())
            cs.append(0.5 * float(f @ f))
            return f

        res = least_squares(fun, x0, jac=lambda x: jac(x, pl, pr, mode), xtol=2.22e-14,
                            tr_solver='lsmr')
        first = next((k for k in range(min(len(cs), len(costs))) if cs[k] != costs[k]), None)
        kx = next((int(k) for k, xk in zip(kept_idx, kept_x)
                   if k < len(xs) and not np.array_equal(xs[k], xk)), None)
        print(f"{tag} {mode}: f0 bits equal {np.array_equal(f0, tr[f'{tag}_f0'])}, "
              f"nfev {res.nfev} (ref {int(tr[f'{tag}_nfev'])}), cost {res.cost!r} "
              f"(ref {float(tr[f'{tag}_cost_final'])!r}), first cost mismatch at eval {first}, "
              f"first kept-x mismatch at eval {kx}, x_final equal "
              f"{np.array_equal(res.x, tr[f'{tag}_x_final'])}, |dF| {dF(res.x, tr[f'{tag}_F_gold']):.3g}",
              flush=True)


def dF(x, Fref):
    C1 = x[:12].reshape(3, 4)
    e = np.array([[0, -C1[2, 3], C1[1, 3]], [C1[2, 3], 0, -C1[0, 3]], [-C1[1, 3], C1[0, 3], 0]])
    F = e @ C1[:, :3]   # [e1]x A of C1 = [A | e1] against [I | 0]: lab3.fmatrix_from_cameras up to scale
    nf = lambda M: (M / np.linalg.norm(M)) * np.sign((M / np.linalg.norm(M)).flat[np.argmax(np.abs(M))])
    return np.abs(nf(F) - nf(Fref)).max()


if __name__ == "__main__":
    main()
