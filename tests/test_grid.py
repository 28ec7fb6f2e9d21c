"""Grid and compact-scheme coefficient tables: C++ tables vs an independent NumPy re-derivation,
polynomial exactness and measured convergence order (SURVEY §4.2 tier 'Unit: grid and coefficients')."""
import numpy as np
import pytest

from channel_gpu_amd.reference import oracle as ora


@pytest.mark.parametrize("N", [33, 129, 385])
def test_tables_match_numpy(native, N):
    g = native.YGrid.build(N)
    o = ora.build_ops(N)
    assert np.max(np.abs(np.asarray(g.y) - o.y)) < 1e-15
    idx = np.arange(1, N - 1)
    assert np.allclose(np.asarray(g.d1_lo)[idx], o.A1[idx, idx - 1], rtol=1e-12, atol=0)
    assert np.allclose(np.asarray(g.d1_up)[idx], o.A1[idx, idx + 1], rtol=1e-12, atol=0)
    assert np.allclose(np.asarray(g.d1_rm)[idx], o.B1[idx, idx - 1], rtol=1e-12, atol=0)
    assert np.allclose(np.asarray(g.m_lo)[idx], o.M[idx, idx - 1], rtol=1e-12, atol=0)
    assert np.allclose(np.asarray(g.k_up)[idx], o.K[idx, idx + 1], rtol=1e-12, atol=0)
    assert np.allclose(g.d1_w0, o.B1[0, :3], rtol=1e-12)
    assert abs(np.asarray(g.d1_up)[0] - o.A1[0, 1]) < 1e-12
    assert np.allclose(np.asarray(g.trap), o.trap, rtol=1e-12, atol=1e-15)


def test_d1_polynomial_exactness():
    o = ora.build_ops(65)
    y = o.y
    for p in range(0, 4):
        f = y ** p
        df = p * y ** (p - 1) if p > 0 else 0 * y
        assert np.max(np.abs(o.D1 @ f - df)) < 1e-10 * max(1, p), p


def test_d2_exact_for_cubics():
    o = ora.build_ops(65)
    y = o.y
    for p in range(0, 4):
        f = y ** p
        d2 = p * (p - 1) * y ** max(p - 2, 0) if p > 1 else 0 * y
        # interior compact relation M f'' = K f
        res = (o.M @ d2 - o.K @ f)[1:-1]
        assert np.max(np.abs(res)) < 1e-9, p


def test_convergence_order():
    errs = []
    for N in (33, 65, 129, 257):
        o = ora.build_ops(N)
        f = np.sin(1.3 * o.y) + np.cos(2.1 * o.y)
        df = 1.3 * np.cos(1.3 * o.y) - 2.1 * np.sin(2.1 * o.y)
        errs.append(np.max(np.abs(o.D1 @ f - df)))
    orders = np.log2(np.array(errs[:-1]) / np.array(errs[1:]))
    assert orders.min() > 2.8, orders  # 3rd-order wall closure, 4th-order interior


def test_flux_weights_exact_for_cubics():
    o = ora.build_ops(129)
    for p in range(4):
        exact = (1 - (-1) ** (p + 1)) / (p + 1)
        assert abs(o.trap @ o.y ** p - exact) < 1e-13


def test_helmholtz_manufactured():
    """(D2 - k^2) v = phi with v(+-1)=0 for v = (1-y^2)^2 cos(pi y/2): solution error converges."""
    errs = []
    for N in (65, 129, 257):
        o = ora.build_ops(N)
        y = o.y
        c, s = np.cos(np.pi * y / 2), np.sin(np.pi * y / 2)
        v = (1 - y * y) ** 2 * c
        # v'' of (1-y^2)^2 cos(pi y/2), analytic
        g, dg, d2g = (1 - y * y) ** 2, -4 * y * (1 - y * y), -4 + 12 * y * y
        d2v = d2g * c + 2 * dg * (-np.pi / 2 * s) + g * (-(np.pi / 2) ** 2 * c)
        k2 = np.array([9.0])
        phi = (d2v - k2[0] * v)[:, None]
        vr = ora.op_helm(o, phi, k2)[:, 0]
        errs.append(np.max(np.abs(vr - v)))
    orders = np.log2(np.array(errs[:-1]) / np.array(errs[1:]))
    assert orders.min() > 3.5, (errs, orders)


def test_helmholtz_solve_consistency():
    o = ora.build_ops(129)
    y = o.y
    k2 = np.array([0.0, 4.0, 100.0])
    v = np.stack([(1 - y * y) ** 2 * np.cos(np.pi * y / 2)] * 3, axis=1)
    phi = o.D2 @ v - k2 * v
    vr = ora.op_helm(o, phi, k2)
    assert np.max(np.abs(vr - v)) < 1e-12
