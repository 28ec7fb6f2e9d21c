"""Physics of the CPU reference path (NumPy fp64 oracle): BASELINE config 1 (laminar Poiseuille,
32x33x32, Re=100), divergence-free velocity recovery, influence-matrix wall conditions."""
import numpy as np
import pytest

from channel_gpu_amd.reference import oracle as ora


def random_solver(NX=32, NY=33, NZ=17, Re=400.0, dt=0.01, amp=0.3, seed=3):
    o = ora.OracleSolver(NX, NY, NZ, Re=Re, dt_fixed=dt)
    phi, om = ora.random_state(o.plan, o.ops, seed=seed, amp=amp)
    o.set_state(phi, om, 0.75 * 1.8 * (1 - o.ops.y ** 2))
    return o


def test_continuity_of_recovered_velocity():
    o = random_solver()
    o.prepare()
    u, v, w = (o.lines(f) for f in o.fields[:3])
    div = 1j * o.al * u + o.ops.D1 @ v + 1j * o.be * w
    assert np.abs(div).max() < 1e-12 * max(1.0, np.abs(v).max())


def test_wall_conditions_after_steps():
    o = random_solver()
    for _ in range(3):
        o.step()
    vl = ora._bsolve(ora.helm_matrix(o.ops, o.k2), o.ops.M @ o.lines(o.phi))
    dv = o.ops.D1 @ vl
    nz = o.k2 > 0
    assert np.abs(vl[[0, -1]]).max() < 1e-12
    assert np.abs(dv[[0, -1]][:, nz]).max() < 1e-11
    assert abs(o.ops.trap @ o.U - 1.8) < 1e-12


def test_hermitian_kz0_preserved():
    o = random_solver()
    for _ in range(2):
        o.step()
    p = o.plan
    phi = o.phi
    for i in range(1, p.Kx + 1):
        assert np.allclose(phi[:, i, 0], np.conj(phi[:, p.nkx - i, 0]), atol=1e-12)


def test_poiseuille_cpu_reference_path():
    """BASELINE config 1: 32x33x32, Re=100 relaxes to U = 1.35 (1 - y^2), u_tau^2 = 2.7 nu."""
    o = ora.OracleSolver(32, 33, 17, Re=100.0, dt_fixed=2.0)
    y = o.ops.y
    U0 = 1.0 - y ** 8
    U0 *= 1.8 / (o.ops.trap @ U0)
    z = np.zeros_like(o.phi)
    o.set_state(z, z, U0)
    for _ in range(300):
        o.step()
    assert np.max(np.abs(o.U - 1.35 * (1 - y * y))) < 1e-6
    assert abs(o.utau() ** 2 - 2.7 / 100.0) < 1e-7


def test_perturbations_decay_at_low_re():
    o = random_solver(Re=100.0, dt=0.02, amp=0.05)
    e0 = np.sum(np.abs(o.om) ** 2) + np.sum(np.abs(o.phi) ** 2)
    for _ in range(20):
        o.step()
    e1 = np.sum(np.abs(o.om) ** 2) + np.sum(np.abs(o.phi) ** 2)
    assert e1 < 0.5 * e0


def test_plane_stats_nonnegative():
    o = random_solver()
    o.prepare()
    st = o.plane_stats()
    assert (st[:3] >= 0).all() and np.isfinite(st).all()


def test_parity_modes_differ_from_default_but_stay_close():
    """CPU oracle: explicit D1 o D1 and analytic influence functions (the reference's semantics) give
    trajectories close to the default (compact D2, discrete Green's functions) but not identical; the
    analytic influence only satisfies v'(+-1) = 0 to truncation error, the discrete one to round-off."""
    NX, NY, NZ = 16, 33, 9
    base = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=0.01)
    phi, om = ora.random_state(base.plan, base.ops, seed=2, amp=0.3)
    U = 0.75 * 1.8 * (1 - base.ops.y ** 2)
    res = {}
    for key in [("compact", "discrete"), ("dd", "discrete"), ("compact", "analytic")]:
        o = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=0.01, explicit_d2=key[0], influence=key[1])
        o.set_state(phi, om, U)
        for _ in range(2):
            o.step()
        res[key] = o
    ref = res[("compact", "discrete")].phi
    for key in [("dd", "discrete"), ("compact", "analytic")]:
        d = np.linalg.norm(res[key].phi - ref) / np.linalg.norm(ref)
        assert 1e-12 < d < 0.2, (key, d)
    # wall derivative of v after the step: discrete influence -> round-off
    o = res[("compact", "discrete")]
    v = ora._bsolve(ora.helm_matrix(o.ops, o.k2), o.ops.M @ o.lines(o.phi))
    dv = o.ops.D1 @ v
    assert np.abs(dv[[0, -1]]).max() < 1e-9 * max(1.0, np.abs(v).max())
