"""Physics validation on the GPU: Tollmien-Schlichting growth rate vs the Orr-Sommerfeld
eigenvalue (Re = 7500, alpha = 1; SURVEY §4.2 'Physics: linear stability')."""
import numpy as np
import pytest

from channel_gpu_amd.models import orr_sommerfeld as osm
from channel_gpu_amd.reference import oracle as ora
from channel_gpu_amd.utils.config import default_config

pytestmark = pytest.mark.gpu


def test_ts_wave_growth_rate(native):
    NX, NY, NZ, Re, dt = 16, 129, 9, 7500.0, 0.02
    cfg = default_config(NX=NX, NY=NY, NZ=NZ, Re=Re, Q=4.0 / 3.0, precision="fp64", dt_fixed=dt, ic="zero",
                         stats_every=0, log_every=0, symmetry_every=0)
    s = native.Solver(cfg, 0, 1, 0, b"")
    plan = ora.OraclePlan(NX, NY, NZ)
    ops = ora.build_ops(NY)
    phi, om, U, c = osm.ts_initial_state(plan, ops, Re, eps=1e-6)
    s.set_state(phi, om, U)
    s.prepare()
    amps, ts = [], []
    for i in range(1500):
        s.step(False)
        if i % 250 == 249:
            p, _, _ = s.get_state()
            amps.append(np.linalg.norm(p[:, 1, 0]))
            ts.append((i + 1) * dt)
    rates = np.diff(np.log(amps)) / np.diff(ts)
    sigma = c.imag  # alpha = 1
    assert np.all(np.abs(rates - sigma) < 0.01 * sigma), (rates, sigma)
    assert s.health() == 0


@pytest.mark.slow
def test_turbulent_retau180_statistics(native):
    """BASELINE config 2 regression: a developed Re_tau~180 state (seed committed from the long
    validation run in profiles/r02_turbulence_retau180: Re_tau 179.5, U+_c 18.2, u'+ peak 2.70 at
    y+ 14.4, 250k averaging steps) stays on the turbulent attractor.  Short average (2.5k steps after
    1k steps of recovery of the truncated seed modes), so the bands are loose; no reference output
    covers these numbers (parity unpinned), they are the published Re_tau=180 channel values."""
    import os

    from channel_gpu_amd.models.statistics import TurbulenceStatistics
    from channel_gpu_amd.utils.snapshots import load_seed

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    phi, om, U = load_seed(os.path.join(root, "tests", "data", "retau180_seed.npz"))
    cfg = default_config(NX=128, NY=129, NZ=65, Re=3130.0, precision="fp64", ic="zero", stats_every=0, log_every=0,
                         symmetry_every=0)
    s = native.Solver(cfg, 0, 1, 0, b"")
    s.set_state(phi, om, U)
    s.prepare()
    for _ in range(1000):
        s.step(False)
    st = TurbulenceStatistics(np.asarray(s.grid.y), 1.0 / cfg.Re)
    for _ in range(250):
        for i in range(10):
            s.step(i == 9)
        L = s.log()
        st.add(np.asarray(s.mean_profile()), np.asarray(s.stats()), L.utau_lo, L.utau_hi, L.time)
    sm = st.summary()
    assert s.health() == 0
    assert 165 < sm["Re_tau"] < 195, sm
    assert 16.5 < sm["Uc_plus"] < 20.0, sm
    assert 2.3 < sm["urms_peak"] < 3.1 and 8 < sm["urms_peak_yplus"] < 25, sm
    assert 0.6 < sm["uv_max"] < 0.9, sm
    y = np.asarray(s.grid.y)
    assert abs(float(np.asarray(s.grid.trap) @ np.asarray(s.mean_profile())) - cfg.Q) < 1e-10
