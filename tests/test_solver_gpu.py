"""End-to-end GPU solver tests against the NumPy fp64 oracle and analytic solutions."""
import math
import os

import numpy as np
import pytest
import torch

from channel_gpu_amd.reference import oracle as ora
from channel_gpu_amd.utils.config import default_config

pytestmark = pytest.mark.gpu


def rel(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(np.asarray(b)), 1e-300)


def make_solver(native, **kw):
    cfg = default_config(**kw)
    return native.Solver(cfg, 0, 1, 0, b"")


@pytest.mark.parametrize("NX,NY,NZ", [(32, 33, 17), (32, 65, 33), (96, 97, 97), (48, 33, 41), (112, 33, 73),
                                      (240, 33, 57), (176, 33, 105)])
def test_gpu_matches_oracle_fp64(native, NX, NY, NZ):
    """(96, 97, 97): NX = 96 and 2NZ-2 = 192 run the radix-3 transform plans; (48, 33, 41): 48 and 80;
    (112, 33, 73): 7*2^k and 9*2^k (2NZ-2 = 144); (240, 33, 57): 15*2^k and 7*2^k (112);
    (176, 33, 105): 11*2^k and 13*2^k (208).
    The fixed step shrinks with the grid so the random state stays within the CFL limit."""
    dt = 0.01 * min(1.0, 32.0 / NX)
    kw = dict(NX=NX, NY=NY, NZ=NZ, Re=400.0, precision="fp64", dt_fixed=dt, stats_every=0, log_every=0,
              symmetry_every=0, ic="zero")
    s = make_solver(native, **kw)
    o = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=dt)
    phi, om = ora.random_state(o.plan, o.ops, seed=3, amp=0.3)
    U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
    o.set_state(phi, om, U)
    s.set_state(phi, om, U)
    s.prepare()
    for it in range(3):
        o.step()
        s.step(False)
        gphi, gom, gU = s.get_state()
        assert rel(gphi, o.phi) < 1e-9, f"phi step {it}"
        assert rel(gom, o.om) < 1e-9, f"omega step {it}"
        assert rel(gU, o.U) < 1e-11, f"U step {it}"


@pytest.mark.parametrize("precision,NY", [("fp32", 129), ("fp64", 129), ("fp32", 225), ("fp64", 225), ("fp32", 257),
                                          ("fp64", 257), ("fp32", 385), ("fp64", 481),
                                          ("fp32", 633), ("fp64", 633), ("fp32", 769), ("fp32", 1201),
                                          ("fp64", 1409)])
def test_gpu_matches_oracle_large_ny(native, precision, NY):
    """Tall lines: R = 3, 4 (address-only prefetch slots), R = 7 (register prefetch slots),
    R = 10 and 13->16 (deferred slots, LDS-staged tables), 17->24 (NY up to 1536: the lifted
    NY <= 1024 cap of the reference, main.c:79-82)."""
    NX, NZ, dt = 16, 9, 1e-4
    kw = dict(NX=NX, NY=NY, NZ=NZ, Re=400.0, precision=precision, dt_fixed=dt, stats_every=0, log_every=0,
              symmetry_every=0, ic="zero")
    s = make_solver(native, **kw)
    o = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=dt)
    phi, om = ora.random_state(o.plan, o.ops, seed=5, amp=0.05)
    if precision == "fp32":
        phi = phi.astype(np.complex64).astype(np.complex128)
        om = om.astype(np.complex64).astype(np.complex128)
    # fp32 storage round-off grows with NY (omega at NY = 1201: 1.2e-4)
    tol, tolU = (1e-9, 1e-11) if precision == "fp64" else (1e-4 * max(1.0, NY / 600), 1e-5)
    U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
    o.set_state(phi, om, U)
    s.set_state(phi, om, U)
    s.prepare()
    for it in range(2):
        o.step()
        s.step(False)
        gphi, gom, gU = s.get_state()
        assert rel(gphi, o.phi) < tol, f"phi step {it}: {rel(gphi, o.phi):.3e}"
        assert rel(gom, o.om) < tol, f"omega step {it}: {rel(gom, o.om):.3e}"
        assert rel(gU, o.U) < tolU, f"U step {it}: {rel(gU, o.U):.3e}"


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_blocked_layout_nx1024_matches_oracle(native, monkeypatch, precision):
    """The one-rank blocked spectral layout forced on (CHANNEL_SPEC_KZB=1) at NX = 1024, the
    headline's x length: fp32 runs the plane-tile x kernels with 16-byte accesses
    (xfft_*_kernel<1024, float, false, 1, 0, 2, 2>), fp64 the one-plane tiles; both against the
    dense fp64 oracle for 3 steps."""
    monkeypatch.setenv("CHANNEL_SPEC_KZB", "1")
    NX, NY, NZ, dt = 1024, 65, 33, 3e-4
    kw = dict(NX=NX, NY=NY, NZ=NZ, Re=400.0, precision=precision, dt_fixed=dt, stats_every=0, log_every=0,
              symmetry_every=0, ic="zero")
    s = make_solver(native, **kw)
    assert s.spec_kzb() == 8
    o = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=dt)
    phi, om = ora.random_state(o.plan, o.ops, seed=11, amp=0.3)
    if precision == "fp32":
        phi = phi.astype(np.complex64).astype(np.complex128)
        om = om.astype(np.complex64).astype(np.complex128)
    # fp32: the fp32 round-off of the physical-space product (~1e-7 of the peak) fills the modes the
    # random state leaves near zero, and at |kx| up to 341 phi = D2 v - k^2 v weighs that noise by
    # k^2 (measured 1.8e-4 over all modes at step 0): the fp32 bound is taken on the lines holding
    # >= 1e-6 of the peak line energy, as in test_fp32_tracks_fp64_on_resolved_modes
    tol, tolU = (1e-9, 1e-11) if precision == "fp64" else (1e-4, 1e-5)

    def err(g, w):
        if precision == "fp64":
            return rel(g, w)
        e = np.sum(np.abs(w) ** 2, axis=0)
        keep = e >= 1e-6 * e.max()
        return np.sqrt(np.sum(np.abs(g - w) ** 2, axis=0)[keep].sum() / e[keep].sum())

    U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
    o.set_state(phi, om, U)
    s.set_state(phi, om, U)
    s.prepare()
    for it in range(3):
        o.step()
        s.step(False)
        gphi, gom, gU = s.get_state()
        assert err(gphi, o.phi) < tol, f"phi step {it}: {err(gphi, o.phi):.3e} (all modes {rel(gphi, o.phi):.3e})"
        assert err(gom, o.om) < tol, f"omega step {it}: {err(gom, o.om):.3e} (all modes {rel(gom, o.om):.3e})"
        assert rel(gU, o.U) < tolU, f"U step {it}: {rel(gU, o.U):.3e}"


def test_blocked_layout_equals_plain_headline_ny(native, monkeypatch):
    """CHANNEL_SPEC_KZB=1 vs =0 at 1024 x 385 x 17 (the headline's NX and NY; R = 7): the layouts
    change only addressing and tiling, so the states after 3 steps agree to fp32 round-off."""
    kw = dict(NX=1024, NY=385, NZ=17, Re=20700.0, precision="fp32", ic="random", ic_amplitude=0.05, stats_every=0,
              log_every=0, symmetry_every=0, dt_fixed=5e-4)
    res = {}
    for kzb in ("0", "1"):
        monkeypatch.setenv("CHANNEL_SPEC_KZB", kzb)
        s = make_solver(native, **kw)
        assert s.spec_kzb() == (8 if kzb == "1" else 0)
        s.init_ic()
        s.prepare()
        for _ in range(3):
            s.step(False)
        res[kzb] = s.get_state()
        del s
    for f in range(3):
        a, b = res["1"][f], res["0"][f]
        print(f"field {f}: bitwise {np.array_equal(a, b)}, rel {rel(a, b):.3e}")
        assert rel(a, b) < 1e-6, f


@pytest.mark.parametrize("NY", [289, 385, 449])
def test_kspec_halves_matches_oracle(native, monkeypatch, NY):
    """The opt-in two-wave K-SPEC lines (CHANNEL_KSPEC_HALVES=1: R = 4 on 2 x 64 lanes for
    256 + 2 < NY <= 512, fp32 storage) against the fp64 oracle, at the tolerance of the one-wave
    fp32 path of test_gpu_matches_oracle_large_ny."""
    monkeypatch.setenv("CHANNEL_KSPEC_HALVES", "1")
    NX, NZ, dt = 16, 9, 1e-4
    kw = dict(NX=NX, NY=NY, NZ=NZ, Re=400.0, precision="fp32", dt_fixed=dt, stats_every=0, log_every=0,
              symmetry_every=0, ic="zero")
    s = make_solver(native, **kw)
    o = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=dt)
    phi, om = ora.random_state(o.plan, o.ops, seed=5, amp=0.05)
    phi = phi.astype(np.complex64).astype(np.complex128)
    om = om.astype(np.complex64).astype(np.complex128)
    U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
    o.set_state(phi, om, U)
    s.set_state(phi, om, U)
    s.prepare()
    for it in range(2):
        o.step()
        s.step(False)
        gphi, gom, gU = s.get_state()
        assert rel(gphi, o.phi) < 1e-4, f"phi step {it}: {rel(gphi, o.phi):.3e}"
        assert rel(gom, o.om) < 1e-4, f"omega step {it}: {rel(gom, o.om):.3e}"
        assert rel(gU, o.U) < 1e-5, f"U step {it}: {rel(gU, o.U):.3e}"


def test_poiseuille_steady(native):
    """BASELINE config 1 on the GPU path: the laminar profile 1.35(1-y^2) is a steady state."""
    s = make_solver(native, NX=32, NY=33, NZ=17, Re=100.0, precision="fp64", ic="laminar", stats_every=0,
                    log_every=0, symmetry_every=0)
    s.init_ic()
    s.prepare()
    for _ in range(20):
        s.step(False)
    y = np.asarray(s.grid.y)
    U = np.asarray(s.mean_profile())
    assert np.max(np.abs(U - 1.35 * (1 - y * y))) < 1e-10
    L = s.log()
    assert abs(L.utau ** 2 - 2.7 / 100.0) < 1e-8
    assert L.health == 0


def test_poiseuille_relaxation(native):
    """From a blunt profile with the same flux, the mean flow relaxes to the parabola."""
    s = make_solver(native, NX=32, NY=33, NZ=17, Re=100.0, precision="fp64", ic="zero", stats_every=0,
                    log_every=0, symmetry_every=0, dt_fixed=2.0)
    y = np.asarray(s.grid.y)
    U0 = 1.0 - y ** 8
    U0 *= 1.8 / np.trapz(U0, y)
    n = s.plan.NY * s.plan.nkx_loc * s.plan.nkz
    z = np.zeros(n, complex)
    s.set_state(z, z, U0)
    s.prepare()
    for _ in range(300):
        s.step(False)
    U = np.asarray(s.mean_profile())
    assert np.max(np.abs(U - 1.35 * (1 - y * y))) < 1e-6


def test_graph_equals_eager_fp32(native):
    kw = dict(NX=64, NY=65, NZ=33, Re=1000.0, precision="fp32", ic="random", ic_amplitude=0.2, stats_every=0,
              log_every=0, symmetry_every=0)
    a = make_solver(native, **kw)
    b = make_solver(native, **kw)
    b.set_use_graph(False)
    for s in (a, b):
        s.init_ic()
        s.prepare()
        for _ in range(4):
            s.step(False)
    pa, oa, ua = a.get_state()
    pb, ob, ub = b.get_state()
    assert np.array_equal(pa, pb) and np.array_equal(oa, ob) and np.array_equal(ua, ub)
    assert np.isfinite(pa).all() and a.health() == 0


@pytest.mark.parametrize("chunk,streams", [(1, 1), (7, 1), (16, 1), (7, 2), (8, 2)])
def test_ychunk_pipeline_equals_whole_slab(native, monkeypatch, chunk, streams):
    """The y-chunked x->z->x pipeline (P = 1) is bitwise the whole-slab one, ragged last chunk included."""
    kw = dict(NX=64, NY=65, NZ=33, Re=1000.0, precision="fp32", ic="random", ic_amplitude=0.2, stats_every=0,
              log_every=0, symmetry_every=0)
    monkeypatch.setenv("CHANNEL_YCHUNK", "0")
    a = make_solver(native, **kw)
    monkeypatch.setenv("CHANNEL_YCHUNK", str(chunk))
    monkeypatch.setenv("CHANNEL_YSTREAMS", str(streams))
    b = make_solver(native, **kw)
    for s in (a, b):
        s.init_ic()
        s.prepare()
        for _ in range(3):
            s.step(False)
    pa, oa, ua = a.get_state()
    pb, ob, ub = b.get_state()
    assert np.array_equal(pa, pb) and np.array_equal(oa, ob) and np.array_equal(ua, ub)
    assert a.log().dt == b.log().dt and np.isfinite(pa).all()


def test_turbulent_smoke_128(native, tmp_path):
    """Reference grid 128x129x128 (Re_tau~180 box) in fp32: finite, flux held, stats files written."""
    s = make_solver(native, NX=128, NY=129, NZ=65, Re=3250.0, precision="fp32", ic="random", ic_amplitude=0.3,
                    stats_every=2, log_every=2, path=str(tmp_path) + "/")
    s.init_ic()
    s.run(6, False)
    L = s.log()
    assert L.health == 0 and L.dt > 0 and np.isfinite(L.utau)
    assert abs(L.flux - 1.8) < 0.05  # flux before the correction of the last substep
    for f in ["MEANPROFILE.dat", "UTAU.dat", "STATISTICS.dat", "URMS.dat", "RSTRSS.dat"]:
        assert (tmp_path / f).exists(), f


def test_t_end_stops_run(native):
    """run() stops at the first step whose end time reaches t_end.  Far from t_end the decision reads
    the previous step's (dt, time) from pinned memory (no per-step host sync); near it, the device
    time after a sync.  A second run() continues to a later t_end the same way."""
    s = make_solver(native, NX=32, NY=33, NZ=17, Re=400.0, precision="fp64", ic="random", stats_every=0,
                    log_every=0, symmetry_every=0, dt_fixed=0.01, t_end=0.055)
    s.init_ic()
    s.run(100, False)
    assert s.steps_done() == 6
    assert abs(s.time() - 0.06) < 1e-12
    s2 = make_solver(native, NX=32, NY=33, NZ=17, Re=400.0, precision="fp64", ic="random", stats_every=0,
                     log_every=0, symmetry_every=0, dt_fixed=0.01, t_end=0.405)
    s2.init_ic()
    s2.run(100, False)
    assert s2.steps_done() == 41 and abs(s2.time() - 0.41) < 1e-12


def test_t_end_with_cfl_dt_at_dt_max(native):
    """Variable dt (no dt_fixed): a laminar start whose CFL step exceeds dt_max runs at dt_max from the
    first step; the host-side t_end decision uses dt_max as its margin (a multiple of the
    previous dt is no bound), so the run still stops at the first step that reaches t_end."""
    s = make_solver(native, NX=32, NY=33, NZ=17, Re=400.0, precision="fp64", ic="laminar", stats_every=0,
                    log_every=0, symmetry_every=0, dt_max=0.01, t_end=0.035)
    s.init_ic()
    s.run(100, False)
    assert s.steps_done() == 4 and abs(s.time() - 0.04) < 1e-12


def test_phase_times_add_up(native):
    """Per-phase event timing (serialised chunked pipeline) accounts for the whole step."""
    s = make_solver(native, NX=512, NY=257, NZ=257, Re=11150.0, precision="fp32", ic="random", stats_every=0,
                    log_every=0, symmetry_every=0)
    s.init_ic()
    s.prepare()
    for _ in range(3):
        s.step(False)
    s.set_phase_timing(True)
    s.set_step_timing(True)
    for _ in range(4):
        s.step(False)
    steps = s.step_times_ms()
    s.set_phase_timing(False)
    ph = s.phase_times_ms()
    assert sum(ph[:4]) > 0.8 * sum(steps) and sum(ph[:4]) <= 1.001 * sum(steps)


def test_restart_roundtrip(native, tmp_path):
    if not native.hdf5_available():
        pytest.skip("libhdf5 unavailable")
    kw = dict(NX=32, NY=33, NZ=17, Re=400.0, precision="fp32", ic="random", stats_every=0, log_every=0)
    a = make_solver(native, **kw)
    a.init_ic()
    a.prepare()
    a.step(False)
    g, d, u = str(tmp_path / "G.h5"), str(tmp_path / "DDV.h5"), str(tmp_path / "U.bin")
    a.write_restart(g, d, u)
    b = make_solver(native, **kw)
    b.read_restart(g, d, u)
    pa, oa, ua = a.get_state()
    pb, ob, ub = b.get_state()
    assert rel(pb, pa) < 1e-6 and rel(ob, oa) < 1e-6 and rel(ub, ua) < 1e-6
    assert abs(b.time() - a.time()) < 1e-12


def test_restart_fp64_resume_is_bitwise(native, tmp_path):
    """fp64 storage writes float64 datasets (+ U at full precision): the restored state is bitwise
    the written one, and the resumed run tracks the continuous one to round-off (zeta_0 = 0 needs no
    R; the only difference is that the first transform inputs are re-derived from the state: v from
    a Helmholtz solve instead of the influence-matrix combination of the step that produced it)."""
    if not native.hdf5_available():
        pytest.skip("libhdf5 unavailable")
    kw = dict(NX=32, NY=33, NZ=17, Re=400.0, precision="fp64", ic="random", ic_amplitude=0.2, stats_every=0,
              log_every=0, symmetry_every=0)
    a = make_solver(native, **kw)
    a.init_ic()
    a.prepare()
    for _ in range(3):
        a.step(False)
    g, d, u = str(tmp_path / "G.h5"), str(tmp_path / "DDV.h5"), str(tmp_path / "U.bin")
    a.write_restart(g, d, u)
    b = make_solver(native, **kw)
    b.read_restart(g, d, u)
    b.prepare()
    pa, oa, ua = a.get_state()
    pb, ob, ub = b.get_state()
    assert np.array_equal(pa, pb) and np.array_equal(oa, ob) and np.array_equal(ua, ub)
    for s in (a, b):
        for _ in range(3):
            s.step(False)
    pa, oa, ua = a.get_state()
    pb, ob, ub = b.get_state()
    assert rel(pb, pa) < 1e-11 and rel(ob, oa) < 1e-11 and rel(ub, ua) < 1e-13
    assert abs(a.time() - b.time()) < 1e-14


def test_async_checkpoints(native, tmp_path):
    """checkpoint_every with checkpoint_async: files written by a background thread from a host copy
    taken at the step boundary, while stepping continues; every checkpoint reads back exactly."""
    if not native.hdf5_available():
        pytest.skip("libhdf5 unavailable")
    out = str(tmp_path) + "/"
    s = make_solver(native, NX=32, NY=33, NZ=17, Re=400.0, precision="fp64", ic="random", ic_amplitude=0.2,
                    stats_every=0, log_every=0, symmetry_every=0, checkpoint_every=2, checkpoint_async=True,
                    out_G=out + "G.h5", out_DDV=out + "DDV.h5", out_UMEAN=out + "U.bin", path=out)
    s.init_ic()
    s.run(4, False)
    p4, o4, u4 = s.get_state()
    import os

    assert all(os.path.exists(out + f) for f in ["G.h5.2", "DDV.h5.2", "G.h5.4", "DDV.h5.4", "U.bin.4"])
    assert not any(f.endswith(".turn") for f in os.listdir(out))
    r = make_solver(native, NX=32, NY=33, NZ=17, Re=400.0, precision="fp64", ic="zero", stats_every=0, log_every=0)
    r.read_restart(out + "G.h5.4", out + "DDV.h5.4", out + "U.bin.4")
    pr, orr, ur = r.get_state()
    assert np.array_equal(pr, p4) and np.array_equal(orr, o4) and np.array_equal(ur, u4)
    assert r.steps_done() == 4


def test_symmetrize_with_communicator_matches_single_rank(native):
    """Distributed kz=0 symmetrisation (column exchange) on a real 1-rank RCCL communicator equals the
    single-rank kernel bitwise and leaves the kz=0 plane Hermitian."""
    kw = dict(NX=32, NY=33, NZ=17, Re=400.0, precision="fp64", ic="zero", stats_every=0, log_every=0,
              symmetry_every=0)
    o = ora.OracleSolver(32, 33, 17, Re=400.0)
    phi, om = ora.random_state(o.plan, o.ops, seed=7, amp=0.3)
    rng = np.random.default_rng(3)
    phi[:, :, 0] += 0.01 * (rng.standard_normal(phi[:, :, 0].shape) + 1j * rng.standard_normal(phi[:, :, 0].shape))
    U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
    res = []
    for uid in (b"", native.new_unique_id()):
        s = native.Solver(default_config(**kw), 0, 1, 0, uid)
        s.set_state(phi, om, U)
        s.symmetrize()
        res.append(s.get_state())
    (pa, oa, _), (pb, ob, _) = res
    assert np.array_equal(pa, pb) and np.array_equal(oa, ob)
    nkx = pa.shape[1]
    for k in range(1, nkx):
        assert np.array_equal(pa[:, k, 0], np.conj(pa[:, nkx - k, 0]))
    assert not np.any(pa[:, 0, 0].imag)


@pytest.mark.parametrize("explicit_d2,influence", [("dd", "discrete"), ("compact", "analytic"), ("dd", "analytic")])
@pytest.mark.parametrize("NX,NY,NZ", [(32, 33, 17), (32, 65, 33), (16, 257, 9), (16, 385, 9), (16, 633, 9)])
def test_reference_parity_modes_match_oracle(native, explicit_d2, influence, NX, NY, NZ):
    """Reference-parity switches: explicit_d2 = dd (D1 o D1, RK3_kernels.cu:160-164) and
    influence = analytic (cosh/sinh Green's functions, bilplacSolver_double.cu:56-250) on the GPU vs
    the NumPy oracle implementing the same semantics, up to the production wall-normal resolutions
    (NY = 257, 385, 633: the R = 5, 7, 10 kernels).  The explicit D1 o D1 viscous term of the
    reference scheme limits the step near the stretched walls, so the tall grids take a small one."""
    dt = 0.01 if NY <= 65 else 2e-4
    kw = dict(NX=NX, NY=NY, NZ=NZ, Re=400.0, precision="fp64", dt_fixed=dt, stats_every=0, log_every=0,
              symmetry_every=0, ic="zero", explicit_d2=explicit_d2, influence=influence)
    s = make_solver(native, **kw)
    o = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=dt, explicit_d2=explicit_d2, influence=influence)
    phi, om = ora.random_state(o.plan, o.ops, seed=3, amp=0.3)
    U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
    o.set_state(phi, om, U)
    s.set_state(phi, om, U)
    s.prepare()
    for it in range(3):
        o.step()
        s.step(False)
        gphi, gom, gU = s.get_state()
        assert rel(gphi, o.phi) < 1e-9, f"phi step {it}: {rel(gphi, o.phi):.3e}"
        assert rel(gom, o.om) < 1e-9, f"omega step {it}"
        assert rel(gU, o.U) < 1e-11, f"U step {it}"


def test_fp64_2048_point_transforms_run(native):
    """fp64 storage at 2048-point x and z transforms (Re_tau~2000 on 8 GPUs in fp64).

    The seeded IC is band-limited (exp(-k^2/32) envelope) and does not depend on the grid, so after
    two steps the 2048 x 2048 run must agree with the (oracle-tested) 1024 x 1024 run on every mode
    the smaller grid retains, and hold only round-off noise above it.  (An fp32-vs-fp64 comparison
    is no use here: at NY = 33 the wall influence correction amplifies fp32 round-off in the
    nonlinear term of the unresolved high modes by ~1e8; fp64 keeps it at ~1e-8.)"""
    kw = dict(NY=33, Re=2000.0, ic="random", ic_amplitude=0.02, stats_every=0, log_every=0,
              symmetry_every=0, dt_fixed=1e-4, precision="fp64")
    res = []
    for NX, NZ in ((2048, 1025), (1024, 513)):
        s = make_solver(native, NX=NX, NZ=NZ, **kw)
        s.init_ic()
        s.prepare()
        for _ in range(2):
            s.step(False)
        assert s.health() == 0
        res.append(s.get_state())
        del s
    big, small = res
    nkx1, nkz1 = small[0].shape[1], small[0].shape[2]
    nkx2 = big[0].shape[1]
    kx1 = (nkx1 - 1) // 2
    idx = np.r_[0:kx1 + 1, nkx2 - kx1:nkx2]
    for f in range(2):
        sub = big[f][:, idx, :nkz1]
        assert rel(sub, small[f]) < 1e-7, f"field {f}"  # the ~1e-8 noise floor of the high modes
        rest = np.linalg.norm(big[f]) ** 2 - np.linalg.norm(sub) ** 2
        assert math.sqrt(max(rest, 0.0)) < 1e-6 * np.linalg.norm(sub), f"field {f} high modes"


def test_fp32_tracks_fp64_on_resolved_modes(native):
    """fp32 storage (fp64 y-solves, the reference's precision split) vs fp64 storage from the same
    band-limited random IC over 20 steps at the headline NY = 385 (Re = 20700, stretched grid).

    The fp32 round-off of the nonlinear term seeds every mode at ~1e-7 of the peak; the wall
    influence correction amplifies it in modes the IC leaves empty (README, "fp32 storage and the
    high wavenumbers").  This bounds the drift where it matters: on the resolved modes (lines
    holding >= 1e-6 of the most energetic line's energy) the two trajectories agree to 2e-5
    (relative L2), and U to 1e-6."""
    kw = dict(NX=64, NY=385, NZ=33, Re=20700.0, ic="random", ic_amplitude=0.05, stats_every=0, log_every=0,
              symmetry_every=0, dt_fixed=5e-4)
    res = {}
    for prec in ("fp64", "fp32"):
        s = make_solver(native, precision=prec, **kw)
        s.init_ic()
        s.prepare()
        for _ in range(20):
            s.step(False)
        assert s.health() == 0
        res[prec] = s.get_state()
        del s
    worst = {}
    for f, name in ((0, "phi"), (1, "omega")):
        a, b = res["fp32"][f], res["fp64"][f]
        e = np.sum(np.abs(b) ** 2, axis=0)            # energy per (kx, kz) line
        keep = e >= 1e-6 * e.max()
        d = np.sqrt(np.sum(np.abs(a - b) ** 2, axis=0)[keep].sum() / e[keep].sum())
        worst[name] = d
        print(f"{name}: resolved lines {int(keep.sum())}/{keep.size}, rel L2 fp32-fp64 {d:.3e}")
    dU = rel(res["fp32"][2], res["fp64"][2])
    print(f"U: rel {dU:.3e}")
    assert worst["phi"] < 2e-5 and worst["omega"] < 2e-5, worst
    assert dU < 1e-6


def test_fp32_high_band_energy_bounded(native):
    """fp32 storage round-off in the wavenumber bands the band-limited random IC leaves empty
    (README, "fp32 storage and the high wavenumbers"; headline time series in
    profiles/r05/highband_1024x385x1024_table.txt): from the same IC, 400 steps of fp32 and fp64
    storage at 128 x 129 x 128 (Re = 3130), kinetic energy at three planes.  In the bands the IC
    leaves empty (kz >= nkz/2, |kx| >= Kx/2) fp32 may only carry noise at the level of fp32
    round-off (<= 1e-12 of the energy, ~300 eps^2) or the physical content fp64 finds there, and
    the energy itself and the filled low band must agree."""
    kw = dict(NX=128, NY=129, NZ=65, Re=3130.0, ic="random", ic_amplitude=0.05, stats_every=0, log_every=0,
              symmetry_every=0, dt_fixed=2e-3, spectra_planes="3,16,64")
    res = {}
    for prec in ("fp64", "fp32"):
        s = make_solver(native, precision=prec, **kw)
        s.init_ic()
        s.prepare()
        for _ in range(400):
            s.step(False)
        assert s.health() == 0
        sp = s.spectra()
        ekz = np.asarray(sp["ekz"]).sum(axis=(0, 1))
        ekx = np.asarray(sp["ekx"]).sum(axis=(0, 1))
        res[prec] = (ekz.sum(), ekz[ekz.size // 2:].sum() / ekz.sum(), ekx[ekx.size // 2:].sum() / ekx.sum(),
                     ekz[:8].sum() / ekz.sum())
        del s
    (E64, z64, x64, lo64), (E32, z32, x32, lo32) = res["fp64"], res["fp32"]
    print(f"E {E32:.6e} / {E64:.6e}; kz>=nkz/2 {z32:.3e} / {z64:.3e}; kx>=Kx/2 {x32:.3e} / {x64:.3e}")
    assert abs(E32 - E64) <= 1e-4 * E64
    assert abs(lo32 - lo64) <= 1e-4
    assert z32 <= max(100 * z64, 1e-12), (z32, z64)
    assert x32 <= max(100 * x64, 1e-12), (x32, x64)


@pytest.mark.parametrize("precision,NX,NY,NZ", [("fp32", 32, 33, 17), ("fp32", 64, 385, 33), ("fp64", 32, 129, 17),
                                                ("fp32", 48, 97, 41)])
def test_lds_poison_mode_is_bitwise(native, precision, NX, NY, NZ):
    """LDS poison-fill debug mode: K-SPEC, the x transforms and the z stage fill their
    shared memory with NaN bit patterns before use.  A kernel that read a slot it never wrote would
    turn NaN (or at least differ); the run must equal the normal one bitwise."""
    kw = dict(NX=NX, NY=NY, NZ=NZ, Re=2000.0, precision=precision, ic="random", ic_amplitude=0.05,
              stats_every=1, log_every=0, symmetry_every=0, dt_fixed=2e-4)
    res = []
    try:
        for poison in (False, True):
            native.set_lds_poison(poison)
            assert native.lds_poison_enabled() == poison
            s = make_solver(native, **kw)
            s.init_ic()
            s.prepare()
            for _ in range(3):
                s.step(True)
            assert s.health() == 0
            res.append((s.get_state(), np.asarray(s.stats())))
            del s
    finally:
        native.set_lds_poison(False)
    (a, sa), (b, sb) = res
    for f in range(3):
        assert np.all(np.isfinite(b[f]))
        assert np.array_equal(a[f], b[f]), f"field {f}"
    assert np.allclose(sa, sb, rtol=1e-12, atol=0)  # (plane sums: atomic order may differ)


@pytest.mark.parametrize("NX,NY,NZ,precision", [(64, 385, 33, "fp32"), (96, 129, 49, "fp64")])
def test_nontemporal_spectral_access_is_bitwise(native, monkeypatch, NX, NY, NZ, precision):
    """Non-temporal spectral reads (x-backward) and writes (x-forward), on by default only for grids
    whose spectral fields exceed the Infinity Cache: forced on for small grids (the tiled layout at
    NY = 385, the plain one at 129), the run equals the cached-access run bitwise."""
    kw = dict(NX=NX, NY=NY, NZ=NZ, Re=2000.0, precision=precision, ic="random", ic_amplitude=0.05,
              stats_every=0, log_every=0, symmetry_every=0, dt_fixed=2e-4)
    res = []
    for nt in ("0", "1"):
        monkeypatch.setenv("CHANNEL_XNT", nt)
        s = make_solver(native, **kw)
        s.init_ic()
        s.prepare()
        for _ in range(3):
            s.step(False)
        assert s.health() == 0
        res.append(s.get_state())
        del s
    for f in range(3):
        assert np.array_equal(res[0][f], res[1][f]), f"field {f}"


@pytest.mark.parametrize("precision,NY", [("fp64", 65), ("fp64", 385), ("fp32", 385), ("fp32", 1201)])
def test_combine_mode_matches_oracle(native, monkeypatch, precision, NY):
    """The combine mode of P > 1 (K-SPEC writes D1 v, v, D1 omega; the x-backward forms u, w,
    omega_x, omega_z per element, fp32 arithmetic at fp32 storage) forced at one rank
    (CHANNEL_COMBINE=1) against the fp64 oracle: fp64 at the 1e-9 of the six-output mode; fp32 U at
    NY = 1201 measured 1.26e-5 (the six-output mode: < 1e-5)."""
    monkeypatch.setenv("CHANNEL_COMBINE", "1")
    NX, NZ, dt = 16, 9, 1e-4
    kw = dict(NX=NX, NY=NY, NZ=NZ, Re=400.0, precision=precision, dt_fixed=dt, stats_every=0, log_every=0,
              symmetry_every=0, ic="zero")
    s = make_solver(native, **kw)
    assert s.combine()
    o = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=dt)
    phi, om = ora.random_state(o.plan, o.ops, seed=5, amp=0.05)
    if precision == "fp32":
        phi = phi.astype(np.complex64).astype(np.complex128)
        om = om.astype(np.complex64).astype(np.complex128)
    tol, tolU = (1e-9, 1e-11) if precision == "fp64" else (1e-4 * max(1.0, NY / 600), 1e-5 * max(1.0, NY / 600))
    U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
    o.set_state(phi, om, U)
    s.set_state(phi, om, U)
    s.prepare()
    for it in range(2):
        o.step()
        s.step(False)
        gphi, gom, gU = s.get_state()
        assert rel(gphi, o.phi) < tol, f"phi step {it}: {rel(gphi, o.phi):.3e}"
        assert rel(gom, o.om) < tol, f"omega step {it}: {rel(gom, o.om):.3e}"
        assert rel(gU, o.U) < tolU, f"U step {it}: {rel(gU, o.U):.3e}"
