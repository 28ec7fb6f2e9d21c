"""Slab decomposition math: C++ Plan vs the Python mirror; limits of the reference lifted
(NX != NY, NY % P != 0, NY = 385 at P = 8)."""
import pytest

from channel_gpu_amd.parallel.decomposition import (PencilDecomposition, SlabDecomposition, auto_pencil_grid,
                                                    balanced_split)


def cfg(native, **kw):
    c = native.Config()
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_plan_matches_python(native, P):
    c = cfg(native, NX=1024, NY=385, NZ=513)
    d = SlabDecomposition(1024, 385, 513, P)
    ks, kc = d.kx_split()
    ys, yc = d.y_split()
    for r in range(P):
        p = native.Plan.make(c, P, r)
        assert (p.nkx, p.nkz, p.Kx, p.Kz) == (683, 342, 341, 341)
        assert p.kx0 == ks[r] and p.nkx_loc == kc[r]
        assert p.y0 == ys[r] and p.ny_loc == yc[r]
        assert p.R == 7
    assert sum(kc) == 683 and sum(yc) == 385 and max(yc) - min(yc) <= 1


def test_mean_mode_on_rank0(native):
    c = cfg(native, NX=128, NY=129, NZ=65)
    p = native.Plan.make(c, 4, 0)
    assert p.kx0 == 0 and p.kx_of(0) == 0


def test_kx_maps(native):
    c = cfg(native, NX=128, NY=129, NZ=65)
    p = native.Plan.make(c, 1, 0)
    assert p.nkx == 85 and p.Kx == 42
    assert p.kx_of(42) == 42 and p.kx_of(43) == -42 and p.kx_of(84) == -1
    assert p.kx_fft_pos(43) == 128 - 42 and p.kx_fft_pos(84) == 127


def test_balanced_split_properties():
    for n in (33, 385, 683):
        for parts in (1, 2, 3, 7, 8):
            s, c = balanced_split(n, parts)
            assert sum(c) == n and s[0] == 0 and max(c) - min(c) <= 1
            assert all(s[i] + c[i] == s[i + 1] for i in range(parts - 1))


def test_too_many_ranks(native):
    c = cfg(native, NX=32, NY=33, NZ=17)
    with pytest.raises(RuntimeError):
        native.Plan.make(c, 64, 0)


def test_a2a_volume_model():
    d = SlabDecomposition(1024, 385, 1024 // 2 + 1, 8)
    b = d.a2a_off_rank_bytes_per_step(esz=8)
    # per rank and step: 27 transposes of 7/8 of its retained-field slab (0.72 GB / 8 per field)
    # ~= 2.1 GB; at ~7 x 153 GB/s of xGMI per GPU that is ~2 ms of ideal all-to-all per step
    assert 1.5e9 < b < 3.0e9


@pytest.mark.parametrize("P,pr", [(4, 2), (8, 2), (8, 4), (6, 3), (8, 0)])
def test_pencil_plan_matches_python(native, P, pr):
    c = cfg(native, NX=1024, NY=385, NZ=513, decomposition="pencil", pr=pr)
    Pr, Pc = (pr, P // pr) if pr else auto_pencil_grid(P, 1024, 385, 513)
    d = PencilDecomposition(1024, 385, 513, Pr, Pc)
    seen = set()
    for r in range(P):
        p = native.Plan.make(c, P, r)
        assert (p.Pr, p.Pc) == (Pr, Pc) and p.pencil() == (Pr > 1)
        L = d.local(r)
        got = dict(kx0=p.kx0, nkx_loc=p.nkx_loc, y0=p.y0, ny_loc=p.ny_loc, kz0=p.kz0, nkz_loc=p.nkz_loc, x0=p.x0,
                   nx_loc=p.nx_loc)
        assert got == L
        assert p.owns_mean() == (r == 0) if hasattr(p, "owns_mean") else True
        seen.update((kx, kz) for kx in range(p.kx0, p.kx0 + p.nkx_loc) for kz in range(p.kz0, p.kz0 + p.nkz_loc))
    assert len(seen) == 683 * 342   # every retained mode owned exactly once


def test_pencil_grid_mismatch(native):
    c = cfg(native, NX=64, NY=65, NZ=33, decomposition="pencil", pr=3)
    with pytest.raises(RuntimeError):
        native.Plan.make(c, 4, 0)


@pytest.mark.parametrize("P,per_peer_mb", [(2, 180.0), (4, 45.0), (8, 11.2)])
def test_a2a_per_peer_bytes_match_survey_model(P, per_peer_mb):
    """Per-peer exchange volume of the slab pipeline vs SURVEY §5.8's truncated model at Re_tau~950
    (1024x385x1024, fp32): one field of one transpose to one peer is (NY/P)(nkx/P)nkz x 8 B; a
    step moves 27 such blocks (9 fields x 3 substeps) to every peer."""
    d = SlabDecomposition(1024, 385, 513, P)
    ys, yc = d.y_split()
    ks, kc = d.kx_split()
    one = [yc[q] * kc[0] * d.nkz * 8 for q in range(1, P)]  # rank 0 -> q, one field, backward
    # SURVEY §5.8 lists 45 MB per peer at P=4 and 11.2 MB at P=8 (truncated); P=2 is 4x the P=4 block
    assert abs(max(one) / 1e6 - per_peer_mb) / per_peer_mb < 0.03
    per_step = d.a2a_bytes_per_peer_per_step(0)
    for q in range(1, P):
        assert per_step[q] == 3 * (6 * yc[q] * kc[0] + 3 * yc[0] * kc[q]) * d.nkz * 8
        assert abs(per_step[q] / (27 * one[q - 1]) - 1) < 0.03


def test_bench_refuses_work_skipping_env(tmp_path):
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CHANNEL_FFT_DIAG="1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "work-skipping" in (r.stderr + r.stdout)


def test_ny_cap_lifted_to_1536(native):
    """The reference's one-thread-per-y-point solver caps NY at 1024 (main.c:79-82); the register-
    resident y-line kernels go to R = 24 rows per lane (NY <= 1536), beyond which Plan refuses."""
    assert native.Plan.make(cfg(native, NX=32, NY=1201, NZ=17), 1, 0).R == 19
    assert native.Plan.make(cfg(native, NX=32, NY=1536, NZ=17), 1, 0).R == 24
    with pytest.raises(Exception, match="1536"):
        native.Plan.make(cfg(native, NX=32, NY=1537, NZ=17), 1, 0)


def test_auto_pencil_grid_minimises_the_busiest_link():
    """--decomposition pencil without pr/pc picks the factorisation with the fewest bytes on the
    busiest link: 4 x 2 at 8 ranks of the headline grid (the B exchange carries x-expanded rows,
    NX = 1.5 nkx, so the most square 2 x 4 loads a row-group link 1.5x more)."""
    assert auto_pencil_grid(8, 1024, 385, 513) == (4, 2)
    assert auto_pencil_grid(4, 1024, 385, 513) == (2, 2)
    assert auto_pencil_grid(7, 1024, 385, 513) == (1, 7)
    for P in (4, 6, 8):
        Pr, Pc = auto_pencil_grid(P, 1024, 385, 513)
        d = PencilDecomposition(1024, 385, 513, Pr, Pc)
        link = max(max(d.exchange_bytes_per_substep(r)["A"] // max(1, Pc - 1),
                       d.exchange_bytes_per_substep(r)["B"] // max(1, Pr - 1)) for r in range(P))
        for r2 in range(2, P):
            if P % r2 == 0 and r2 != Pr and P // r2 > 1:
                d2 = PencilDecomposition(1024, 385, 513, r2, P // r2)
                link2 = max(max(d2.exchange_bytes_per_substep(r)["A"] // max(1, P // r2 - 1),
                                d2.exchange_bytes_per_substep(r)["B"] // max(1, r2 - 1)) for r in range(P))
                assert link <= link2 * 1.01, (P, (Pr, Pc), (r2, P // r2))
