"""Slab decomposition math (Python mirror of csrc/core/plan.cpp, used by tests and tools).

Spectral state per rank: [y (all NY)][kx_local][kz]; physical per rank: [y_local][x][kz].
Every split is balanced (counts differ by at most one), so NY = 385 at P = 8 works — the
reference required NX == NY, NY % P == 0 and NX/P % 64 == 0.
"""
from __future__ import annotations

import dataclasses


def balanced_split(n: int, parts: int) -> tuple[list[int], list[int]]:
    if parts < 1 or n < parts:
        raise ValueError(f"cannot split {n} items over {parts} parts")
    base, rem = divmod(n, parts)
    count = [base + (1 if p < rem else 0) for p in range(parts)]
    start, off = [], 0
    for c in count:
        start.append(off)
        off += c
    return start, count


@dataclasses.dataclass(frozen=True)
class SlabDecomposition:
    NX: int
    NY: int
    NZ: int
    P: int

    @property
    def Kx(self) -> int:
        return self.NX // 3

    @property
    def nkx(self) -> int:
        return 2 * self.Kx + 1

    @property
    def nkz(self) -> int:
        return (2 * self.NZ - 2) // 3 + 1

    def kx_split(self):
        return balanced_split(self.nkx, self.P)

    def y_split(self):
        return balanced_split(self.NY, self.P)

    def a2a_backward_bytes(self, rank: int, esz: int = 8) -> list[int]:
        """bytes rank sends to each peer in one backward (spectral -> physical) all-to-all."""
        ks, kc = self.kx_split()
        ys, yc = self.y_split()
        return [yc[q] * kc[rank] * self.nkz * esz for q in range(self.P)]

    def a2a_bytes_per_peer_per_step(self, rank: int, esz: int = 8) -> list[int]:
        """bytes ``rank`` sends to each peer per RK3 step: per substep 6 backward fields (its kx
        columns of the peer's y rows) and 3 forward fields (its y rows of the peer's kx columns);
        the entry for ``rank`` itself is the on-device self copy."""
        ks, kc = self.kx_split()
        ys, yc = self.y_split()
        return [3 * (6 * yc[q] * kc[rank] + 3 * yc[rank] * kc[q]) * self.nkz * esz for q in range(self.P)]

    def a2a_off_rank_bytes_per_step(self, esz: int = 8) -> int:
        """off-rank bytes per RK3 step for the busiest rank (6 backward + 3 forward per substep)."""
        worst = 0
        for r in range(self.P):
            b = sum(x for q, x in enumerate(self.a2a_backward_bytes(r, esz)) if q != r)
            worst = max(worst, b)
        return 3 * 9 * worst


def auto_pencil_grid(P: int, NX: int, NY: int, NZ: int) -> tuple[int, int]:
    """The Pr x Pc pencil grid (Pr, Pc > 1) with the fewest bytes on the busiest link
    (Plan::auto_grid): per substep a rank sends (NY/Pc)(nkx/Pc)(nkz/Pr) complex values to each
    column-group peer (A) and (NY/Pc)(NX/Pr)(nkz/Pr) to each row-group peer (B, x-expanded rows);
    ties go to the squarer grid with Pr <= Pc.  (1, P) when P has no such factorisation."""
    nkx, nkz = 2 * (NX // 3) + 1, (2 * NZ - 2) // 3 + 1
    best, grid = None, (1, P)
    for r in range(2, min(8, P - 1) + 1):
        if P % r:
            continue
        c = P // r
        if c > 8 or c > nkx or c > NY or r > nkz or r > NX:
            continue
        ny, kz = NY / c, nkz / r
        link = max(ny * (nkx / c) * kz, ny * (NX / r) * kz)
        squarer = abs(r - c) < abs(grid[0] - grid[1]) or (abs(r - c) == abs(grid[0] - grid[1]) and r <= c)
        if best is None or link < best * (1 - 1e-9) or (link <= best * (1 + 1e-9) and squarer):
            best, grid = link, (r, c)
    return grid


@dataclasses.dataclass(frozen=True)
class PencilDecomposition:
    """Pr x Pc pencil grid (Python mirror of Plan for decomposition = "pencil").

    rank = prow * Pc + pcol.  Spectral [y][kx in KX_pcol][kz in KZ_prow]; the A exchange
    (column group, Pc ranks) swaps kx <-> y, the B exchange (row group, Pr ranks) swaps kz <-> x;
    the z stage sees [y in Y_pcol][x in X_prow][kz (all)].  Pr = 1 is the slab.
    """
    NX: int
    NY: int
    NZ: int
    Pr: int
    Pc: int

    @property
    def P(self) -> int:
        return self.Pr * self.Pc

    @property
    def nkx(self) -> int:
        return 2 * (self.NX // 3) + 1

    @property
    def nkz(self) -> int:
        return (2 * self.NZ - 2) // 3 + 1

    def coords(self, rank: int) -> tuple[int, int]:
        return divmod(rank, self.Pc)

    def local(self, rank: int) -> dict:
        prow, pcol = self.coords(rank)
        ks, kc = balanced_split(self.nkx, self.Pc)
        ys, yc = balanced_split(self.NY, self.Pc)
        zs, zc = balanced_split(self.nkz, self.Pr)
        xs, xc = balanced_split(self.NX, self.Pr)
        return dict(kx0=ks[pcol], nkx_loc=kc[pcol], y0=ys[pcol], ny_loc=yc[pcol], kz0=zs[prow], nkz_loc=zc[prow],
                    x0=xs[prow], nx_loc=xc[prow])

    def exchange_bytes_per_substep(self, rank: int, esz: int = 8) -> dict:
        """off-rank bytes sent by ``rank`` per substep: A (6 backward + 3 forward fields over the
        column group) and B (6 + 3 over the row group; 0 for the slab)."""
        L = self.local(rank)
        prow, pcol = self.coords(rank)
        ys, yc = balanced_split(self.NY, self.Pc)
        xs, xc = balanced_split(self.NX, self.Pr)
        a = sum(yc[c] for c in range(self.Pc) if c != pcol) * L["nkx_loc"] * L["nkz_loc"] * esz
        b = sum(xc[r] for r in range(self.Pr) if r != prow) * L["ny_loc"] * L["nkz_loc"] * esz
        return {"A": 9 * a, "B": 9 * b}
