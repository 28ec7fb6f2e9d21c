"""Time-averaged turbulence statistics of the channel in wall units.

The reference only appends instantaneous profiles to text files (MEANPROFILE.dat every step,
URMS/VRMS/WRMS/RSTRSS.dat every 10 steps: meanUevol.c:489-560, statistics.cu:161-243) and leaves
averaging and wall scaling to the user.  This accumulator takes the same quantities the solver
reduces on the device — U(y), the plane mean squares <u'u'>, <v'v'>, <w'w'>, <u'v'> (Parseval
plane sums, all ranks reduced) and the wall friction velocities — and produces the standard
wall-unit profiles folded over the two channel halves: U+(y+), u'+, v'+, w'+ r.m.s., -<u'v'>+,
plus the scalar checks of a statistically steady Re_tau~180 channel (Re_tau, U+_c, the u'+ peak
and its y+).
"""
from __future__ import annotations

import json

import numpy as np


class TurbulenceStatistics:
    def __init__(self, y: np.ndarray, nu: float):
        self.y = np.asarray(y, float)
        self.nu = float(nu)
        self.reset()

    def reset(self):
        n = self.y.size
        self.n = 0
        self.U = np.zeros(n)
        self.ms = np.zeros((4, n))  # uu, vv, ww, uv
        self.tau = 0.0              # mean wall shear velocity squared (both walls)
        self.t0 = None
        self.t1 = None

    def add(self, U, stats, utau_lo: float, utau_hi: float, t: float | None = None):
        """One sample: U(y) [NY], stats [4*NY] (uu, vv, ww, uv plane means), u_tau at both walls."""
        n = self.y.size
        st = np.asarray(stats, float).reshape(4, n)
        self.U += np.asarray(U, float)
        self.ms += st
        self.tau += 0.5 * (utau_lo ** 2 + utau_hi ** 2)
        self.n += 1
        if t is not None:
            self.t0 = t if self.t0 is None else self.t0
            self.t1 = t

    # ---- averaged results ------------------------------------------------------------------------
    def utau(self) -> float:
        return float(np.sqrt(self.tau / max(self.n, 1)))

    def profiles(self) -> dict:
        """Averaged profiles folded onto the lower half (y+ from the nearest wall)."""
        if self.n == 0:
            raise ValueError("no samples")
        n = self.y.size
        ut = self.utau()
        U = self.U / self.n
        ms = self.ms / self.n
        h = (n + 1) // 2  # lower half incl. the centre point for odd NY
        lo = np.arange(h)
        hi = n - 1 - lo  # mirror points
        fold = lambda a, s=1.0: 0.5 * (a[lo] + s * a[hi])  # noqa: E731
        yplus = (1.0 + self.y[lo]) * ut / self.nu
        return {
            "y": self.y[lo],
            "yplus": yplus,
            "Uplus": fold(U) / ut,
            "urms": np.sqrt(np.maximum(fold(ms[0]), 0.0)) / ut,
            "vrms": np.sqrt(np.maximum(fold(ms[1]), 0.0)) / ut,
            "wrms": np.sqrt(np.maximum(fold(ms[2]), 0.0)) / ut,
            # <u'v'> is antisymmetric about the centreline
            "uvplus": -fold(ms[3], -1.0) / ut ** 2,
        }

    def summary(self) -> dict:
        p = self.profiles()
        ut = self.utau()
        U = self.U / self.n
        yb = self.y
        Ub = float(np.trapz(U, yb) / (yb[-1] - yb[0]))
        i = int(np.argmax(p["urms"]))
        return {
            "samples": self.n,
            "t_start": self.t0,
            "t_end": self.t1,
            "utau": ut,
            "Re_tau": ut / self.nu,
            "Uc_plus": float(p["Uplus"][-1]),
            "Ub_plus": Ub / ut,
            "Cf": 2.0 * ut ** 2 / Ub ** 2,
            "urms_peak": float(p["urms"][i]),
            "urms_peak_yplus": float(p["yplus"][i]),
            "vrms_max": float(p["vrms"].max()),
            "wrms_max": float(p["wrms"].max()),
            "uv_max": float(p["uvplus"].max()),
        }

    def write(self, path: str):
        """Profiles as whitespace columns (y, y+, U+, u'+, v'+, w'+, -u'v'+) with a JSON summary header."""
        p = self.profiles()
        cols = np.column_stack([p["y"], p["yplus"], p["Uplus"], p["urms"], p["vrms"], p["wrms"], p["uvplus"]])
        with open(path, "w") as f:
            f.write("# " + json.dumps(self.summary()) + "\n")
            f.write("# y yplus Uplus urms_plus vrms_plus wrms_plus minus_uv_plus\n")
            np.savetxt(f, cols, fmt="%.6e")
