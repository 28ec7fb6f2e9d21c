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
