"""Orr-Sommerfeld eigen-solver (in-repo Chebyshev collocation) used by the linear-stability test."""
import numpy as np

from channel_gpu_amd.models import orr_sommerfeld as osm


def test_orszag_eigenvalue():
    c, _, _ = osm.least_stable(10000.0, 1.0, N=120)
    assert abs(c - osm.ORSZAG_RE10000) < 1e-7


def test_ts_unstable_at_7500_and_stable_at_5000():
    c75, _, _ = osm.least_stable(7500.0, 1.0, N=100)
    c50, _, _ = osm.least_stable(5000.0, 1.0, N=100)
    assert c75.imag > 0 > c50.imag  # critical Reynolds number 5772 lies in between
    assert abs(c75.real - 0.2498915) < 1e-5


def test_mode_interpolation_on_dns_grid():
    from channel_gpu_amd.reference import oracle as ora

    ops = ora.build_ops(129)
    c, v = osm.ts_mode_on_grid(ops.y, 7500.0)
    assert abs(v[0]) < 1e-12 and abs(v[-1]) < 1e-12
    assert abs(np.abs(v).max() - 1.0) < 1e-12
    # clamped: v'(+-1) ~ 0 on the DNS grid
    dv = ops.D1 @ v
    assert abs(dv[0]) < 1e-3 and abs(dv[-1]) < 1e-3
