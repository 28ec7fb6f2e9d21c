"""NumPy fp64 oracle of the whole solver (the "CPU reference path", BASELINE config 1).

An independent, dense-matrix implementation of the same discretisation as the HIP kernels:
  * grid / compact coefficients re-derived here (not read from the C++ tables);
  * wall-normal operators as dense N x N matrices (np.linalg.solve instead of the partitioned
    register solver);
  * transforms with numpy.fft instead of the LDS Stockham kernels;
  * optional slab decomposition through ``torch.distributed`` (gloo) all-to-alls, with the same
    data layout and block addressing as the GPU path, so the decomposition logic is testable on CPU.

Reference behaviour reproduced (file:line in /root/reference/src):
  compact D1 derivatives_nu_double.cu:60-112, 227-274; compact D2 hemholzt_nu_double.cu:58-62,
  136-185; implicit step implicitStep_nu_double.cu:133-163; influence matrix
  bilplacSolver_double.cu (discrete form); RK3 coefficients RK3_kernels.cu:24-25,113;
  KMM velocity recovery nonLinear_kernels.cu:55-82; vorticity convolution_kernels.cu:46-53;
  rotational product convolution_kernels.cu:125-131; h_v/h_g nonLinear_kernels.cu:129-181;
  mean flow meanUevol.c:439-567 (with an exact flux constraint instead of meanUevol.c:201-221).
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

GAMMA = (8.0 / 15.0, 5.0 / 12.0, 3.0 / 4.0)
ZETA = (0.0, -17.0 / 60.0, -5.0 / 12.0)
ALPHA = (29.0 / 96.0, -3.0 / 40.0, 1.0 / 6.0)
BETA = (37.0 / 160.0, 5.0 / 24.0, 1.0 / 6.0)


# --------------------------------------------------------------------------------------------
# grid and compact coefficients
# --------------------------------------------------------------------------------------------
def ygrid(N: int, stretch: float = 2.0) -> np.ndarray:
    dy = 2.0 / (N - 1)
    y = np.tanh(stretch * (np.arange(N) * dy - 1.0)) / math.tanh(stretch)
    y[0], y[-1] = -1.0, 1.0
    return y


@dataclasses.dataclass
class YOps:
    y: np.ndarray
    A1: np.ndarray   # D1 LHS
    B1: np.ndarray   # D1 RHS
    D1: np.ndarray   # dense compact first derivative
    M: np.ndarray    # compact D2 mass matrix (interior rows, zero wall rows)
    K: np.ndarray    # compact D2 stencil (interior rows, zero wall rows)
    D2: np.ndarray   # dense compact D2 with the wall closure (mean-flow / IC use)
    trap: np.ndarray

    @property
    def N(self) -> int:
        return len(self.y)


def build_ops(N: int, stretch: float = 2.0) -> YOps:
    y = ygrid(N, stretch)
    A1 = np.eye(N)
    B1 = np.zeros((N, N))
    M = np.zeros((N, N))
    K = np.zeros((N, N))
    for j in range(1, N - 1):
        a = y[j + 1] - y[j]
        b = y[j - 1] - y[j]
        amb2 = (a - b) ** 2
        A1[j, j + 1] = b * b / amb2
        A1[j, j - 1] = a * a / amb2
        Ac = 2.0 * (2.0 * a * b * b - b ** 3) / ((a * a - a * b) * amb2)
        Bc = 2.0 * (2.0 * b * a * a - a ** 3) / ((b * b - a * b) * amb2)
        B1[j, j + 1], B1[j, j - 1], B1[j, j] = Ac, Bc, -Ac - Bc
        den = a ** 3 - b ** 3 - 4.0 * a * a * b + 4.0 * b * b * a
        den2 = a ** 3 - 4.0 * a * a * b + 4.0 * a * b * b - b ** 3
        K[j, j + 1] = -12.0 * b / den
        K[j, j - 1] = 12.0 * a / den
        K[j, j] = -K[j, j + 1] - K[j, j - 1]
        M[j, j + 1] = -(-b ** 3 - a * b * b + a * a * b) / den2
        M[j, j - 1] = -(a ** 3 + b * a * a - b * b * a) / den2
        M[j, j] = 1.0
    # D1 wall closure
    for (j, s) in ((0, 1), (N - 1, -1)):
        a = y[j + s] - y[j]
        b = y[j + 2 * s] - y[j + s]
        A1[j, j + s] = (a + b) / b
        B1[j, j] = -(3.0 * a + 2.0 * b) / (a * a + a * b)
        B1[j, j + s] = ((a + b) * (2.0 * b - a)) / (a * b * b)
        B1[j, j + 2 * s] = a * a / (b * b * a + b ** 3)
    D1 = np.linalg.solve(A1, B1)
    # D2 with closure (meanUevol.c:254-329)
    A2 = M.copy()
    K2 = K.copy()
    for (j, s) in ((0, 1), (N - 1, -1)):
        a = y[j + s] - y[j]
        b = y[j + 2 * s] - y[j]
        A2[j, j] = 1.0
        A2[j, j + s] = (a + b) / (2.0 * a - b)
        Ac = 6.0 / ((a - b) * (2.0 * a - b))
        Bc = -6.0 * a / ((a * b - b * b) * (2.0 * a - b))
        K2[j, j], K2[j, j + s], K2[j, j + 2 * s] = -Ac - Bc, Ac, Bc
    D2 = np.linalg.solve(A2, K2)
    return YOps(y, A1, B1, D1, M, K, D2, flux_weights(y))


def flux_weights(y: np.ndarray) -> np.ndarray:
    """Cubic-exact quadrature weights (per-interval 4-point Lagrange interpolant, Gauss-Legendre)."""
    N = len(y)
    w = np.zeros(N)
    g = 1.0 / math.sqrt(3.0)
    for j in range(N - 1):
        s = min(max(j - 1, 0), N - 4)
        a, b = y[j], y[j + 1]
        for xq in (0.5 * (a + b) - 0.5 * (b - a) * g, 0.5 * (a + b) + 0.5 * (b - a) * g):
            for m in range(4):
                lag = 1.0
                for n in range(4):
                    if n != m:
                        lag *= (xq - y[s + n]) / (y[s + m] - y[s + n])
                w[s + m] += 0.5 * (b - a) * lag
    return w


def _walls_identity(A: np.ndarray) -> np.ndarray:
    A = A.copy()
    A[..., 0, :] = 0.0
    A[..., -1, :] = 0.0
    A[..., 0, 0] = 1.0
    A[..., -1, -1] = 1.0
    return A


def helm_matrix(ops: YOps, k2: np.ndarray) -> np.ndarray:
    k2 = np.asarray(k2, dtype=float)
    return _walls_identity(ops.K[None] - k2[:, None, None] * ops.M[None])


def impl_matrix(ops: YOps, k2: np.ndarray, c: float) -> np.ndarray:
    k2 = np.asarray(k2, dtype=float)
    return _walls_identity((1.0 + c * k2)[:, None, None] * ops.M[None] - c * ops.K[None])


# operators on line batches x[y, line] (complex), per-line k2
def op_d1(ops: YOps, x: np.ndarray) -> np.ndarray:
    return ops.D1 @ x


def op_M(ops: YOps, x: np.ndarray) -> np.ndarray:
    return ops.M @ x


def op_K(ops: YOps, x: np.ndarray) -> np.ndarray:
    return ops.K @ x


def _bsolve(A: np.ndarray, rhs: np.ndarray) -> np.ndarray:
    # A [L, N, N] (tridiagonal), rhs [N, L] -> [N, L]; vectorised Thomas over the L lines
    N = A.shape[-1]
    idx = np.arange(N)
    d = A[:, idx, idx].T.copy()                       # [N, L]
    lo = np.zeros_like(d)
    up = np.zeros_like(d)
    lo[1:] = A[:, idx[1:], idx[:-1]].T
    up[:-1] = A[:, idx[:-1], idx[1:]].T
    return tri_solve(lo, d, up, rhs)


def tri_solve(lo: np.ndarray, d: np.ndarray, up: np.ndarray, rhs: np.ndarray) -> np.ndarray:
    """Thomas algorithm on [N, L] coefficient/RHS arrays (vectorised over the L lines)."""
    N = d.shape[0]
    rhs = np.asarray(rhs)
    cp = np.empty_like(d)
    dp = np.empty(rhs.shape, dtype=np.result_type(rhs, d))
    cp[0] = up[0] / d[0]
    dp[0] = rhs[0] / d[0]
    for j in range(1, N):
        m = d[j] - lo[j] * cp[j - 1]
        cp[j] = up[j] / m
        dp[j] = (rhs[j] - lo[j] * dp[j - 1]) / m
    x = np.empty_like(dp)
    x[-1] = dp[-1]
    for j in range(N - 2, -1, -1):
        x[j] = dp[j] - cp[j] * x[j + 1]
    return x


def op_helm(ops: YOps, x: np.ndarray, k2: np.ndarray) -> np.ndarray:
    return _bsolve(helm_matrix(ops, k2), ops.M @ x)


def op_impl(ops: YOps, x: np.ndarray, k2: np.ndarray, c: float) -> np.ndarray:
    return _bsolve(impl_matrix(ops, k2, c), ops.M @ x)


# --------------------------------------------------------------------------------------------
# decomposition helpers (mirror of csrc/core/plan.cpp)
# --------------------------------------------------------------------------------------------
def balanced_split(n: int, parts: int) -> tuple[list[int], list[int]]:
    base, rem = divmod(n, parts)
    count = [base + (1 if p < rem else 0) for p in range(parts)]
    start = [sum(count[:p]) for p in range(parts)]
    return start, count


@dataclasses.dataclass
class OraclePlan:
    """Decomposition of the retained modes over P = Pr x Pc ranks (rank = prow * Pc + pcol).

    Slab (Pr = 1): kx split over P, physical y split over P.  Pencil (Pr > 1): kx and y split
    over the Pc columns, kz and physical x split over the Pr rows (csrc/include/channel/plan.hpp).
    """
    NX: int
    NY: int
    NZ: int
    P: int = 1
    rank: int = 0
    LX: float = 2 * math.pi
    LZ: float = math.pi
    Pr: int = 1

    def __post_init__(self):
        self.Nzp = 2 * self.NZ - 2
        self.Kx = self.NX // 3
        self.nkx = 2 * self.Kx + 1
        self.Kz = self.Nzp // 3
        self.nkz = self.Kz + 1
        if self.P % self.Pr:
            raise ValueError(f"Pr={self.Pr} does not divide P={self.P}")
        self.Pc = self.P // self.Pr
        self.prow, self.pcol = divmod(self.rank, self.Pc)
        self.kx_start, self.kx_count = balanced_split(self.nkx, self.Pc)
        self.y_start, self.y_count = balanced_split(self.NY, self.Pc)
        self.kz_start, self.kz_count = balanced_split(self.nkz, self.Pr)
        self.x_start, self.x_count = balanced_split(self.NX, self.Pr)
        self.kx0, self.nkx_loc = self.kx_start[self.pcol], self.kx_count[self.pcol]
        self.y0, self.ny_loc = self.y_start[self.pcol], self.y_count[self.pcol]
        self.kz0, self.nkz_loc = self.kz_start[self.prow], self.kz_count[self.prow]
        self.x0, self.nx_loc = self.x_start[self.prow], self.x_count[self.prow]
        self.ax = 2 * math.pi / self.LX
        self.az = 2 * math.pi / self.LZ

    def rank_of(self, row: int, col: int) -> int:
        return row * self.Pc + col

    def kx_of(self, i: np.ndarray | int):
        i = np.asarray(i)
        return np.where(i <= self.Kx, i, i - self.nkx)

    def kx_pos(self, i: np.ndarray | int):
        i = np.asarray(i)
        return np.where(i <= self.Kx, i, self.NX - (self.nkx - i))

    def local_wavenumbers(self):
        ig = self.kx0 + np.arange(self.nkx_loc)
        kx = self.kx_of(ig).astype(float)
        kz = self.kz0 + np.arange(self.nkz_loc, dtype=float)
        al = self.ax * np.repeat(kx, self.nkz_loc)
        be = self.az * np.tile(kz, self.nkx_loc)
        return al, be


# --------------------------------------------------------------------------------------------
# transforms
# --------------------------------------------------------------------------------------------
def spec_to_phys_full(f: np.ndarray, plan: OraclePlan) -> np.ndarray:
    """f[..., y, nkx, nkz] (global kx) -> physical [..., y, NX, Nzp] real."""
    shp = f.shape[:-2]
    F = np.zeros(shp + (plan.NX, plan.NZ), dtype=complex)
    F[..., plan.kx_pos(np.arange(plan.nkx)), : plan.nkz] = f
    G = np.fft.ifft(F, axis=-2, norm="forward")
    return np.fft.irfft(G, n=plan.Nzp, axis=-1, norm="forward")


def phys_to_spec_full(p: np.ndarray, plan: OraclePlan) -> np.ndarray:
    G = np.fft.rfft(p, axis=-1, norm="forward")[..., : plan.nkz]
    F = np.fft.fft(G, axis=-2, norm="forward")
    return F[..., plan.kx_pos(np.arange(plan.nkx)), :]


def rotational_product(phys6: np.ndarray) -> np.ndarray:
    u, v, w, wx, wy, wz = phys6
    return np.stack([v * wz - w * wy, w * wx - u * wz, u * wy - v * wx])


# --------------------------------------------------------------------------------------------
# the solver
# --------------------------------------------------------------------------------------------
class OracleSolver:
    """fp64 NumPy DNS.  State layout per rank: [y][kx_local][kz] (the GPU layout).

    ``comm`` (optional) is a ``torch.distributed`` process group handle for gloo slab runs; the
    physical stage then operates on y-slabs after an all-to-all, exactly like the GPU path.
    """

    def __init__(self, NX, NY, NZ, Re=3250.0, Q=1.8, LX=2 * math.pi, LZ=math.pi, stretch=2.0, cfl=0.5,
                 dt_max=0.05, dt_fixed=0.0, P=1, rank=0, dist=None, Pr=1, explicit_d2="compact",
                 influence="discrete"):
        self.plan = OraclePlan(NX, NY, NZ, P, rank, LX, LZ, Pr)
        self.ops = build_ops(NY, stretch)
        self.Re, self.nu, self.Q = Re, 1.0 / Re, Q
        self.cfl, self.dt_max, self.dt_fixed = cfl, dt_max, dt_fixed
        self.dist = dist
        # reference-parity switches: explicit D2 as D1 o D1 (RK3_kernels.cu:160-164) and analytic
        # cosh/sinh influence functions (bilplacSolver_double.cu:56-250, l1/l2 typo fixed)
        self.explicit_d2, self.influence = explicit_d2, influence
        p = self.plan
        shape = (NY, p.nkx_loc, p.nkz_loc)
        self.phi = np.zeros(shape, complex)
        self.om = np.zeros(shape, complex)
        self.Rphi = np.zeros(shape, complex)
        self.Rom = np.zeros(shape, complex)
        self.U = 0.75 * Q * (1.0 - self.ops.y ** 2)
        self.NU = np.zeros(NY)          # M * N_mean of the previous substep
        self.t = 0.0
        self.dt = 0.0
        self.maxima = np.zeros(4)
        al, be = p.local_wavenumbers()
        self.al, self.be, self.k2 = al, be, al * al + be * be
        self.mean_line = 0 if (p.kx0 == 0 and p.kz0 == 0) else None
        self.fields = None              # 6 prepared fields [6, y, nkx_loc, nkz]
        y = self.ops.y
        h = np.empty(NY)
        h[0], h[-1] = y[1] - y[0], y[-1] - y[-2]
        h[1:-1] = 0.5 * (y[2:] - y[:-2])
        self.inv_dy = 1.0 / h

    # ---- state -----------------------------------------------------------------------------
    def lines(self, f):
        return f.reshape(self.plan.NY, -1)

    def set_state(self, phi, om, U=None):
        self.phi = np.array(phi, complex).reshape(self.phi.shape)
        self.om = np.array(om, complex).reshape(self.om.shape)
        if U is not None:
            self.U = np.array(U, float)
        self.Rphi[:] = 0
        self.Rom[:] = 0
        self.fields = None

    # ---- velocity / vorticity from the state ------------------------------------------------
    def _prepare(self, phi_l, om_l, v_l, U):
        ops, k2, al, be = self.ops, self.k2, self.al, self.be
        dv = ops.D1 @ v_l
        Dom = ops.D1 @ om_l
        DDv = phi_l + k2 * v_l
        ik2 = np.where(k2 > 0, 1.0 / np.where(k2 > 0, k2, 1.0), 0.0)
        u = 1j * (al * dv - be * om_l) * ik2
        w = 1j * (be * dv + al * om_l) * ik2
        Du = 1j * (al * DDv - be * Dom) * ik2
        Dw = 1j * (be * DDv + al * Dom) * ik2
        wx = Dw - 1j * be * v_l
        wy = om_l.copy()
        wz = 1j * al * v_l - Du
        v = v_l.copy()
        if self.mean_line is not None:
            m = self.mean_line
            u[:, m] = U
            w[:, m] = 0
            v[:, m] = 0
            wx[:, m] = 0
            wy[:, m] = 0
            wz[:, m] = -(ops.D1 @ U)
        sh = self.phi.shape
        return np.stack([f.reshape(sh) for f in (u, v, w, wx, wy, wz)])

    def prepare(self):
        phi_l, om_l = self.lines(self.phi), self.lines(self.om)
        v_l = _bsolve(helm_matrix(self.ops, self.k2), self.ops.M @ phi_l)
        zero = self.k2 == 0
        v_l[:, zero] = 0
        phi_l = phi_l.copy()
        phi_l[:, zero] = 0
        self.fields = self._prepare(phi_l, om_l, v_l, self.U)

    # ---- physical stage (optionally distributed) ----------------------------------------------
    def _a2a(self, send: dict, recv_shapes: dict):
        """Variable all-to-all on the world group; peers missing from ``send``/``recv_shapes``
        exchange nothing (the pencil row/column exchanges, like the GPU's alltoallv)."""
        import torch
        import torch.distributed as dist

        P = self.plan.P
        flat = [torch.from_numpy(np.ascontiguousarray(send[g]).view(np.float64)).reshape(-1) if g in send
                else torch.zeros(0, dtype=torch.float64) for g in range(P)]
        in_splits = [t.numel() for t in flat]
        out_splits = [2 * int(np.prod(recv_shapes[g])) if g in recv_shapes else 0 for g in range(P)]
        out = torch.empty(sum(out_splits), dtype=torch.float64)
        dist.all_to_all_single(out, torch.cat(flat), out_splits, in_splits, group=self.dist)
        parts = torch.split(out, out_splits)
        return {g: parts[g].numpy().view(complex).reshape(recv_shapes[g]) for g in recv_shapes}

    def transforms(self, compute_dt: bool):
        p = self.plan
        F = self.fields
        if p.P == 1:
            phys = spec_to_phys_full(F, p)
            H = rotational_product(phys)
            self._maxima(phys, p.y0)
            self.H = phys_to_spec_full(H, p)
        else:
            cols = [p.rank_of(p.prow, c) for c in range(p.Pc)]   # A exchange: kx <-> y
            rows = [p.rank_of(r, p.pcol) for r in range(p.Pr)]   # B exchange: kz <-> x
            nf = F.shape[0]
            recv = self._a2a({g: F[:, p.y_start[c]:p.y_start[c] + p.y_count[c]] for c, g in enumerate(cols)},
                             {g: (nf, p.ny_loc, p.kx_count[c], p.nkz_loc) for c, g in enumerate(cols)})
            full = np.concatenate([recv[g] for g in cols], axis=2)  # [6, ny_loc, nkx, nkz_loc]
            X = np.zeros(full.shape[:2] + (p.NX, p.nkz_loc), complex)
            X[:, :, p.kx_pos(np.arange(p.nkx))] = full
            X = np.fft.ifft(X, axis=2, norm="forward")             # [6, ny_loc, NX, nkz_loc]
            recv = self._a2a({g: X[:, :, p.x_start[r]:p.x_start[r] + p.x_count[r]] for r, g in enumerate(rows)},
                             {g: (nf, p.ny_loc, p.nx_loc, p.kz_count[r]) for r, g in enumerate(rows)})
            Z = np.zeros((nf, p.ny_loc, p.nx_loc, p.NZ), complex)
            Z[..., :p.nkz] = np.concatenate([recv[g] for g in rows], axis=3)
            phys = np.fft.irfft(Z, n=p.Nzp, axis=-1, norm="forward")  # [6, ny_loc, nx_loc, Nzp]
            self._maxima(phys, p.y0)
            Hk = np.fft.rfft(rotational_product(phys), axis=-1, norm="forward")[..., :p.nkz]
            recv = self._a2a({g: Hk[..., p.kz_start[r]:p.kz_start[r] + p.kz_count[r]] for r, g in enumerate(rows)},
                             {g: (3, p.ny_loc, p.x_count[r], p.nkz_loc) for r, g in enumerate(rows)})
            Xh = np.fft.fft(np.concatenate([recv[g] for g in rows], axis=2), axis=2, norm="forward")
            Hs = Xh[:, :, p.kx_pos(np.arange(p.nkx))]              # [3, ny_loc, nkx, nkz_loc]
            recv = self._a2a({g: Hs[:, :, p.kx_start[c]:p.kx_start[c] + p.kx_count[c]] for c, g in enumerate(cols)},
                             {g: (3, p.y_count[c], p.nkx_loc, p.nkz_loc) for c, g in enumerate(cols)})
            self.H = np.concatenate([recv[g] for g in cols], axis=1)
            if compute_dt:
                import torch
                import torch.distributed as dist

                t = torch.from_numpy(self.maxima.copy())
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.dist)
                self.maxima = t.numpy()
        if compute_dt:
            self._update_dt()

    def _maxima(self, phys, y0):
        p = self.plan
        u, v, w = np.abs(phys[0]), np.abs(phys[1]), np.abs(phys[2])
        cx, cz = p.ax * p.Kx, p.az * p.Kz
        iy = self.inv_dy[y0:y0 + phys.shape[1]][:, None, None]
        self.maxima = np.array([u.max(), v.max(), w.max(), (u * cx + v * iy + w * cz).max()])

    def _update_dt(self):
        cs = self.maxima[3]
        dt_c = self.cfl / cs if cs > 0 else self.dt_max
        self.dt = self.dt_fixed if self.dt_fixed > 0 else min(dt_c, self.dt_max)
        self.t += self.dt

    # ---- one substep (K-SPEC equivalent) -------------------------------------------------------
    def substep(self, n: int):
        ops, k2, al, be = self.ops, self.k2, self.al, self.be
        dt, nu = self.dt, self.nu
        Hx, Hy, Hz = (self.lines(h) for h in self.H)
        X = -1j * al * Hx - 1j * be * Hz
        G = 1j * be * Hx - 1j * al * Hz
        m = self.mean_line
        if m is not None:
            G[:, m] = Hx[:, m].real
        Nphi = ops.D1 @ X - k2 * Hy
        RPn = ops.M @ Nphi
        RWn = ops.M @ G
        phi_l, om_l = self.lines(self.phi), self.lines(self.om).copy()
        if m is not None:
            om_l[:, m] = self.U
        Rp_prev, Rw_prev = self.lines(self.Rphi), self.lines(self.Rom)

        def rhs(q, Rn, Rp):
            Kq = ops.K @ q
            if self.explicit_d2 == "dd":
                Kdd = ops.M @ (ops.D1 @ (ops.D1 @ q))
                Kdd[0] = Kdd[-1] = 0.0  # interior rows only, like K
                if m is not None:
                    Kdd[:, m] = Kq[:, m]  # the mean profile keeps the compact D2
                Kq = Kdd
            return ops.M @ q + dt * (ALPHA[n] * nu * (Kq - k2 * (ops.M @ q)) + GAMMA[n] * Rn + ZETA[n] * Rp)

        rP = rhs(phi_l, RPn, Rp_prev)
        rW = rhs(om_l, RWn, Rw_prev)
        c = BETA[n] * dt * nu
        Aimp = impl_matrix(ops, k2, c)
        om_new = _bsolve(Aimp, rW)
        if m is not None:
            U1 = np.linalg.solve(Aimp[m], ops.M @ np.ones(ops.N))
            fU = ops.trap @ om_new[:, m].real
            C = (self.Q - fU) / (ops.trap @ U1)
            om_new[:, m] = om_new[:, m].real + C * U1
            self.U = om_new[:, m].real.copy()
            self.mean_C = C
        phi_p = _bsolve(Aimp, rP)
        L = phi_l.shape[1]
        e0 = np.zeros((ops.N, L))
        e0[0] = 1.0
        eN = np.zeros((ops.N, L))
        eN[-1] = 1.0
        ph1, ph2 = _bsolve(Aimp, e0), _bsolve(Aimp, eN)
        Ah = helm_matrix(ops, k2)
        vp = _bsolve(Ah, ops.M @ phi_p)
        vh1, vh2 = _bsolve(Ah, ops.M @ ph1), _bsolve(Ah, ops.M @ ph2)
        dvp, dvh1, dvh2 = ops.D1 @ vp, ops.D1 @ vh1, ops.D1 @ vh2
        if self.influence == "analytic" and dt > 1e-14:
            ph1, ph2, vh1, vh2, dvh1, dvh2 = analytic_influence(ops.y, k2, BETA[n] * dt * nu)
        det = dvh1[0] * dvh2[-1] - dvh2[0] * dvh1[-1]
        ok = (k2 > 0) & (dt > 1e-14) & (det != 0)
        dets = np.where(ok, det, 1.0)
        C1 = np.where(ok, (-dvp[0] * dvh2[-1] + dvh2[0] * dvp[-1]) / dets, 0)
        C2 = np.where(ok, (-dvh1[0] * dvp[-1] + dvh1[-1] * dvp[0]) / dets, 0)
        phi = phi_p + C1 * ph1 + C2 * ph2
        v = vp + C1 * vh1 + C2 * vh2
        zero = k2 == 0
        phi[:, zero] = 0
        v[:, zero] = 0
        sh = self.phi.shape
        self.Rphi = RPn.reshape(sh)
        self.Rom = RWn.reshape(sh)
        om_store = om_new.copy()
        self.phi = phi.reshape(sh)
        if m is not None:
            om_store[:, m] = 0
        self.om = om_store.reshape(sh)
        om_for_prep = om_new.copy()
        if m is not None:
            om_for_prep[:, m] = self.U
        self.fields = self._prepare(phi, om_for_prep, v, self.U)

    def step(self):
        if self.fields is None:
            self.prepare()
        for n in range(3):
            self.transforms(compute_dt=(n == 0))
            self.substep(n)

    # ---- diagnostics -------------------------------------------------------------------------
    def dUdy_walls(self):
        d = self.ops.D1 @ self.U
        return d[0], d[-1]

    def utau(self):
        lo, hi = self.dUdy_walls()
        a, b = math.sqrt(self.nu * abs(lo)), math.sqrt(self.nu * abs(hi))
        return math.sqrt(0.5 * (a * a + b * b))

    def plane_stats(self):
        """[4, NY]: <u'u'>, <v'v'>, <w'w'>, <u'v'> (plane averages, fluctuations only)."""
        p = self.plan
        u, v, w = (self.lines(f) for f in self.fields[:3])
        wgt = np.where(np.tile(p.kz0 + np.arange(p.nkz_loc), p.nkx_loc) == 0, 1.0, 2.0)
        if self.mean_line is not None:
            wgt = wgt.copy()
            wgt[self.mean_line] = 0
        return np.stack([(np.abs(u) ** 2) @ wgt, (np.abs(v) ** 2) @ wgt, (np.abs(w) ** 2) @ wgt,
                         (u.real * v.real + u.imag * v.imag) @ wgt])


def _chs(l, y):
    """cosh(l y)/cosh(l), sinh(l y)/sinh(l) and their y-derivatives, overflow-safe (l > 0)."""
    ep, em, e2 = np.exp(l * (y - 1.0)), np.exp(-l * (y + 1.0)), np.exp(-2.0 * l)
    return (ep + em) / (1 + e2), (ep - em) / (1 - e2), l * (ep - em) / (1 + e2), l * (ep + em) / (1 - e2)


def analytic_influence(y: np.ndarray, k2: np.ndarray, c: float):
    """Analytic homogeneous solutions of the phi-v system for each line (reference
    bilplacSolver_double.cu:56-217 with the l1/l2 typo fixed): phi1,2 = (C_l1 -+ S_l1)/2 with
    l1^2 = k^2 + 1/c (c = beta dt nu), v1,2 = D [(C_l1 -+ S_l1)/2 - (C_l2 -+ S_l2)/2] with l2 = k,
    D = 1/(l1^2 - l2^2); returns (phi1, phi2, v1, v2, dv1, dv2) as [NY, lines] (dv: analytic, only the
    wall rows are used).  Lines with k = 0 get zeros."""
    yy = y[:, None]
    ok = k2 > 0
    l2 = np.sqrt(np.where(ok, k2, 1.0))[None, :]
    l1 = np.sqrt(np.where(ok, k2, 1.0) + 1.0 / c)[None, :]
    D = 1.0 / (l1 * l1 - l2 * l2)
    C1, S1, dC1, dS1 = _chs(l1, yy)
    C2, S2, dC2, dS2 = _chs(l2, yy)
    ph1, ph2 = 0.5 * (C1 - S1), 0.5 * (C1 + S1)
    v1 = D * (0.5 * (C1 - S1) - 0.5 * (C2 - S2))
    v2 = D * (0.5 * (C1 + S1) - 0.5 * (C2 + S2))
    dv1 = D * (0.5 * (dC1 - dS1) - 0.5 * (dC2 - dS2))
    dv2 = D * (0.5 * (dC1 + dS1) - 0.5 * (dC2 + dS2))
    z = ~ok
    for a in (ph1, ph2, v1, v2, dv1, dv2):
        a[:, z] = 0.0
    return ph1, ph2, v1, v2, dv1, dv2


def random_state(plan: OraclePlan, ops: YOps, seed: int = 1, amp: float = 0.1, kscale: float = 32.0):
    """Divergence-free random state (v with (1-y^2)^2, omega_y with (1-y^2)), Hermitian kz=0."""
    rng = np.random.default_rng(seed)
    N = ops.N
    y = ops.y
    gphi = np.zeros((N, plan.nkx, plan.nkz), complex)
    gom = np.zeros_like(gphi)
    for i in range(plan.nkx):
        kx = int(plan.kx_of(i))
        if kx < 0:
            continue
        for kz in range(plan.nkz):
            if kx == 0 and kz == 0:
                continue
            al, be = plan.ax * kx, plan.az * kz
            k2 = al * al + be * be
            env = math.exp(-k2 / kscale)
            v = amp * env * (1 - y ** 2) ** 2 * (rng.uniform(-1, 1, N) + 1j * rng.uniform(-1, 1, N))
            om = amp * env * (1 - y ** 2) * (rng.uniform(-1, 1, N) + 1j * rng.uniform(-1, 1, N))
            if kz == 0 and kx == 0:
                v, om = v.real, om.real
            phi = ops.D2 @ v - k2 * v
            gphi[:, i, kz], gom[:, i, kz] = phi, om
            if kz == 0 and kx > 0:
                j = plan.nkx - kx
                gphi[:, j, 0], gom[:, j, 0] = np.conj(phi), np.conj(om)
    return gphi, gom
