"""Orr-Sommerfeld / Squire eigen-solver (Chebyshev collocation, NumPy/SciPy) and Tollmien-
Schlichting initial conditions for linear-stability validation of the DNS (SURVEY §4.2,
'Physics: linear stability').

Plane Poiseuille flow U = 1 - y^2 (centreline velocity 1, Re = 1/nu).  For a perturbation
v = v(y) exp(i(alpha x + beta z - alpha c t)):
    (U - c)(D^2 - k^2) v - U'' v = (D^2 - k^2)^2 v / (i alpha Re),   v(+-1) = v'(+-1) = 0.
Clamped conditions are built in with v = (1 - y^2) f (Trefethen, Spectral Methods in MATLAB,
program 40).  The temporal growth rate of the mode is alpha * c_i.
"""
from __future__ import annotations

import math

import numpy as np


def cheb(N: int):
    """Chebyshev differentiation matrix and points x_j = cos(pi j / N), j = 0..N."""
    x = np.cos(np.pi * np.arange(N + 1) / N)
    c = np.ones(N + 1)
    c[0] = c[-1] = 2.0
    c *= (-1.0) ** np.arange(N + 1)
    X = np.tile(x, (N + 1, 1)).T
    dX = X - X.T
    D = np.outer(c, 1.0 / c) / (dX + np.eye(N + 1))
    D -= np.diag(D.sum(axis=1))
    return D, x


def os_eigs(Re: float, alpha: float, beta: float = 0.0, N: int = 100):
    """All eigenvalues c (phase speeds) and eigenfunctions v on the interior Chebyshev points."""
    import scipy.linalg as sla

    D, x = cheb(N)
    D2 = D @ D
    D3 = D2 @ D
    D4 = D3 @ D
    k2 = alpha * alpha + beta * beta
    S = np.diag(np.concatenate([[0.0], 1.0 / (1.0 - x[1:-1] ** 2), [0.0]]))
    D4c = (np.diag(1.0 - x ** 2) @ D4 - 8.0 * np.diag(x) @ D3 - 12.0 * D2) @ S
    I = np.eye(N - 1)
    D2i = D2[1:-1, 1:-1]
    D4i = D4c[1:-1, 1:-1]
    U = 1.0 - x[1:-1] ** 2
    Upp = -2.0
    L = D2i - k2 * I
    # i alpha Re [ (U - c) L - U'' ] v = (D^2 - k^2)^2 v  ->  A v = c B v
    A = 1j * alpha * Re * (np.diag(U) @ L - Upp * I) - (D4i - 2 * k2 * D2i + k2 * k2 * I)
    B = 1j * alpha * Re * L
    c, V = sla.eig(A, B)
    ok = np.isfinite(c)
    return c[ok], V[:, ok], x[1:-1]


def least_stable(Re: float, alpha: float, beta: float = 0.0, N: int = 100):
    """(c, v_on_interior_points, x_interior) of the mode with the largest growth rate."""
    c, V, x = os_eigs(Re, alpha, beta, N)
    i = int(np.argmax(c.imag))
    return c[i], V[:, i], x


def cheb_interp(x_nodes: np.ndarray, f_nodes: np.ndarray, y: np.ndarray) -> np.ndarray:
    """Barycentric interpolation from Chebyshev points (incl. endpoints) to y."""
    N = len(x_nodes) - 1
    w = (-1.0) ** np.arange(N + 1)
    w[0] *= 0.5
    w[-1] *= 0.5
    out = np.empty(len(y), dtype=np.result_type(f_nodes, float))
    for k, yy in enumerate(y):
        d = yy - x_nodes
        j = np.where(np.abs(d) < 1e-15)[0]
        if len(j):
            out[k] = f_nodes[j[0]]
        else:
            t = w / d
            out[k] = (t @ f_nodes) / t.sum()
    return out


def ts_mode_on_grid(y: np.ndarray, Re: float, alpha: float = 1.0, N: int = 120):
    """Least-stable OS eigenfunction v(y) interpolated to the DNS grid, normalised to max |v| = 1."""
    c, v, x = least_stable(Re, alpha, 0.0, N)
    xf = np.concatenate([[1.0], x, [-1.0]])
    vf = np.concatenate([[0.0], v, [0.0]])
    vg = cheb_interp(xf, vf, y)
    vg /= vg[np.argmax(np.abs(vg))]
    return c, vg


def ts_initial_state(plan, ops, Re: float, eps: float = 1e-6, alpha_index: int = 1):
    """Global (phi, omega, U) with U = 1 - y^2 and a small TS wave at kx = alpha_index, kz = 0."""
    y = ops.y
    alpha = plan.ax * alpha_index
    c, v = ts_mode_on_grid(y, Re, alpha)
    v = eps * v
    v[0] = v[-1] = 0.0
    phi = np.zeros((len(y), plan.nkx, plan.nkz), complex)
    om = np.zeros_like(phi)
    ph = ops.D2 @ v - alpha * alpha * v
    phi[:, alpha_index, 0] = ph
    phi[:, plan.nkx - alpha_index, 0] = np.conj(ph)
    U = 1.0 - y ** 2
    return phi, om, U, c


ORSZAG_RE10000 = 0.23752649 + 0.00373967j  # Orszag (1971), alpha = 1, Re = 10000
