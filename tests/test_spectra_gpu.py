"""Runtime energy spectra (the reference's dead calcSpectra, statistics.cu:245-326, made live) vs a
NumPy evaluation of the oracle's u, v, w fields at the same planes."""
import numpy as np
import pytest

from channel_gpu_amd.reference import oracle as ora
from channel_gpu_amd.utils.config import default_config

pytestmark = pytest.mark.gpu


def _numpy_spectra(o, planes):
    p = o.plan
    F = o.fields[:3]                                     # [3, NY, nkx, nkz]
    kx = np.asarray(p.kx_of(np.arange(p.nkx)))
    kz = np.arange(p.nkz)
    w = np.where(kz == 0, 1.0, 2.0)[None, :] * np.ones((p.nkx, 1))
    w[(kx == 0), 0] = 0.0                                # mean line excluded
    ekx = np.zeros((3, len(planes), p.Kx + 1))
    ekz = np.zeros((3, len(planes), p.nkz))
    for i, j in enumerate(planes):
        e = np.abs(F[:, j]) ** 2 * w                     # [3, nkx, nkz]
        ekz[:, i] = e.sum(axis=1)
        for ig in range(p.nkx):
            ekx[:, i, abs(kx[ig])] += e[:, ig].sum(axis=-1)
    return ekx, ekz


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_spectra_match_numpy(native, precision):
    G = dict(NX=32, NY=33, NZ=17)
    cfg = default_config(**G, Re=400.0, precision=precision, ic="zero", stats_every=0, log_every=0,
                         symmetry_every=0, spectra_planes="16, 4")
    s = native.Solver(cfg, 0, 1, 0, b"")
    o = ora.OracleSolver(**G, Re=400.0)
    phi, om = ora.random_state(o.plan, o.ops, seed=9, amp=0.3)
    U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
    o.set_state(phi, om, U)
    o.prepare()
    s.set_state(phi, om, U)
    s.prepare()
    sp = s.spectra()
    assert list(sp["planes"]) == [16, 4]
    ekx, ekz = _numpy_spectra(o, [16, 4])
    tol = 1e-10 if precision == "fp64" else 1e-5
    assert np.allclose(sp["ekx"], ekx, rtol=tol, atol=tol * ekx.max())
    assert np.allclose(sp["ekz"], ekz, rtol=tol, atol=tol * ekz.max())
    # Parseval: both 1-D spectra sum to the same plane energy
    assert np.allclose(sp["ekx"].sum(-1), sp["ekz"].sum(-1), rtol=1e-9)
    m = np.abs(o.fields[:3, 16]) ** 2
    m[:, 0, 0] = 0.0
    assert np.allclose(sp["map"], m, rtol=tol, atol=tol * m.max())


def test_spectra_files_written(native, tmp_path):
    cfg = default_config(NX=32, NY=33, NZ=17, Re=1000.0, precision="fp32", ic="random", ic_amplitude=0.2,
                         stats_every=0, log_every=2, symmetry_every=0, spectra_every=2,
                         path=str(tmp_path) + "/", log_json=str(tmp_path / "run.jsonl"))
    s = native.Solver(cfg, 0, 1, 0, b"")
    s.init_ic()
    s.run(4, False)
    u = np.loadtxt(tmp_path / "Uspec.dat")
    assert u.shape == (32, 17) and np.isfinite(u).all() and u.max() > 0
    kx = (tmp_path / "SPECTRA_KX.dat").read_text().strip().splitlines()
    assert len(kx) == 2 * 3                      # 2 calls x 1 plane x 3 components
    assert len(kx[0].split()) == 4 + 32 // 3 + 1
    import json

    recs = [json.loads(l) for l in (tmp_path / "run.jsonl").read_text().splitlines()]
    assert [r["step"] for r in recs] == [2, 4]
    assert all(r["health"] == 0 and r["ms_per_step"] > 0 and r["dt"] > 0 for r in recs)
