"""ORACLE -- test infrastructure only, never shipped, never measured as the product.

CPU numpy restatement of the five-point essential-matrix solver (D. Nister, "An efficient
solution to the five-point relative pose problem", PAMI 2004) in the reference's E convention,
and of E-RANSAC with the reference's F-RANSAC consensus rule.

Parity status: "parity unpinned".  The reference has no five-point solver and no E-RANSAC
(`north_star` names "5-point E"; grep finds neither); E is only ever
formed as K^T F K (fun.getEAndK) or from two camera poses (fun.getEFromCameras,
fun.py:12-21).  Known answers come from the reference's own noise-free BAdino2 scene: the E
of two views by getEFromCameras must be among the solutions of any five of their
correspondences (tests/golden/dino_pnp_kat.npz), and the pose of the Dino pair's E-RANSAC
winner is checked against R01 of clean_data_eval.npy.

Convention (the reference's, fun.py:12-21 and lab3.fmatrix_residuals): y1^T E y2 = 0 for
C-normalised homogeneous points y1 (left view) and y2 (right view); E = R^T [t]_x for the
relative pose x2 = R x1 + t.

Algorithm (per minimal sample of five correspondences):
  1. Q (5 x 9), row i = vec(y1_i y2_i^T) (row-major E); its right null space {X, Y, Z, W}
     (the last four right singular vectors), E = x X + y Y + z Z + W.
  2. The ten cubic constraints det(E) = 0 and 2 E E^T E - tr(E E^T) E = 0 in the 20 monomials
     [x^3, y^3, x^2 y, x y^2, x^2 z, x^2, y^2 z, y^2, x y z, x y | x z^2, x z, x, y z^2, y z,
     y, z^3, z^2, z, 1]; Gauss-Jordan on the first ten columns gives [I | B].
  3. k = row(x^2 z) - z row(x^2), l = row(y^2 z) - z row(y^2), m = row(x y z) - z row(x y) are
     linear in (x, y, 1) with polynomial coefficients in z (degrees 3, 3, 4); det [k; l; m] is
     a degree-10 polynomial in z whose real roots give the solutions; (x, y, 1) is the null
     vector of [k; l; m](z).
"""
from __future__ import annotations

import numpy as np

# monomials x^a y^b z^c of the cubic constraints, Nister's column order
MONOS = [(3, 0, 0), (0, 3, 0), (2, 1, 0), (1, 2, 0), (2, 0, 1), (2, 0, 0), (0, 2, 1),
         (0, 2, 0), (1, 1, 1), (1, 1, 0), (1, 0, 2), (1, 0, 1), (1, 0, 0), (0, 1, 2),
         (0, 1, 1), (0, 1, 0), (0, 0, 3), (0, 0, 2), (0, 0, 1), (0, 0, 0)]
_IDX = {m: i for i, m in enumerate(MONOS)}


def _pmul(a, b):
    out = {}
    for ea, ca in a.items():
        for eb, cb in b.items():
            e = (ea[0] + eb[0], ea[1] + eb[1], ea[2] + eb[2])
            out[e] = out.get(e, 0.0) + ca * cb
    return out


def _padd(a, b, s=1.0):
    out = dict(a)
    for e, c in b.items():
        out[e] = out.get(e, 0.0) + s * c
    return out


def null_basis(y1, y2):
    """(4, 3, 3): X, Y, Z, W spanning the E with y1_i^T E y2_i = 0, i < 5."""
    Q = np.einsum("ia,ib->iab", y1, y2).reshape(len(y1), 9)
    _, _, Vt = np.linalg.svd(Q)
    return Vt[-4:].reshape(4, 3, 3)


def constraint_matrix(basis):
    """(10, 20) coefficients of det(E) = 0 and 2 E E^T E - tr(E E^T) E = 0."""
    X, Y, Z, W = basis
    E = [[{(1, 0, 0): X[i, j], (0, 1, 0): Y[i, j], (0, 0, 1): Z[i, j], (0, 0, 0): W[i, j]}
          for j in range(3)] for i in range(3)]
    EEt = [[_padd(_padd(_pmul(E[i][0], E[j][0]), _pmul(E[i][1], E[j][1])),
                  _pmul(E[i][2], E[j][2])) for j in range(3)] for i in range(3)]
    tr = _padd(_padd(EEt[0][0], EEt[1][1]), EEt[2][2])
    rows = []
    for i in range(3):
        for j in range(3):
            p = {}
            for k in range(3):
                p = _padd(p, _pmul(EEt[i][k], E[k][j]), 2.0)
            p = _padd(p, _pmul(tr, E[i][j]), -1.0)
            rows.append(p)
    det = _padd(_padd(_pmul(E[0][0], _padd(_pmul(E[1][1], E[2][2]), _pmul(E[1][2], E[2][1]), -1.0)),
                      _pmul(E[0][1], _padd(_pmul(E[1][0], E[2][2]), _pmul(E[1][2], E[2][0]), -1.0)),
                      -1.0),
                _pmul(E[0][2], _padd(_pmul(E[1][0], E[2][1]), _pmul(E[1][1], E[2][0]), -1.0)))
    rows.append(det)
    M = np.zeros((10, 20))
    for r, p in enumerate(rows):
        for e, c in p.items():
            M[r, _IDX[e]] += c
    return M


def z_polynomial(M):
    """(degree-10 coefficients of det [k; l; m](z), highest first, and (k, l, m) as
    (3, 3) lists of numpy polynomials) from the constraint matrix."""
    B = np.linalg.solve(M[:, :10], M[:, 10:])
    P = np.polynomial.polynomial

    def row(a, b):  # row(a) - z row(b): coefficients in z, lowest first
        A, Bb = B[a], B[b]
        kx = np.array([A[2], A[1] - Bb[2], A[0] - Bb[1], -Bb[0]])
        ky = np.array([A[5], A[4] - Bb[5], A[3] - Bb[4], -Bb[3]])
        k1 = np.array([A[9], A[8] - Bb[9], A[7] - Bb[8], A[6] - Bb[7], -Bb[6]])
        return [kx, ky, k1]

    k, l, m = row(4, 5), row(6, 7), row(8, 9)
    mul, sub = P.polymul, P.polysub
    det = P.polyadd(P.polyadd(
        mul(k[0], sub(mul(l[1], m[2]), mul(l[2], m[1]))),
        -mul(k[1], sub(mul(l[0], m[2]), mul(l[2], m[0])))),
        mul(k[2], sub(mul(l[0], m[1]), mul(l[1], m[0]))))
    return det[::-1], (k, l, m)


def five_point(y1, y2, imag_tol=1e-9):
    """All real essential matrices (unit Frobenius norm) of five correspondences y1_i, y2_i
    (homogeneous, C-normalised, (5, 3))."""
    y1 = np.asarray(y1, float)
    y2 = np.asarray(y2, float)
    basis = null_basis(y1, y2)
    M = constraint_matrix(basis)
    coef, klm = z_polynomial(M)
    roots = np.roots(coef)
    out = []
    P = np.polynomial.polynomial
    for z in roots:
        if abs(z.imag) > imag_tol * max(1.0, abs(z)):
            continue
        z = z.real
        A = np.array([[P.polyval(z, c) for c in r] for r in klm])
        # (x, y, 1): null vector of A, the largest of the three row cross products
        cs = [np.cross(A[0], A[1]), np.cross(A[0], A[2]), np.cross(A[1], A[2])]
        v = max(cs, key=lambda c: abs(c[2]))
        if v[2] == 0:
            continue
        x, y = v[0] / v[2], v[1] / v[2]
        E = x * basis[0] + y * basis[1] + z * basis[2] + basis[3]
        out.append(E / np.linalg.norm(E))
    return out


def e_from_cameras(R1, t1, R2, t2):
    """fun.getEFromCameras (fun.py:12-21)."""
    R = R2 @ R1.T
    t = t2 - R2 @ R1.T @ t1
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    return R.T @ tx


def same_e(E, F, tol):
    """E and F equal up to scale and sign."""
    a = E / np.linalg.norm(E)
    b = F / np.linalg.norm(F)
    return min(np.abs(a - b).max(), np.abs(a + b).max()) <= tol


def f_from_e(E, K1, K2):
    """x1^T F x2 = 0 for pixels x = K y: F = K1^-T E K2^-1."""
    return np.linalg.inv(K1).T @ E @ np.linalg.inv(K2)
