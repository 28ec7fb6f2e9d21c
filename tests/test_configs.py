"""Every shipped configs/*.conf (one per BASELINE.json config) parses, validates and decomposes on
the GPU counts it is meant for; the physical parameters match the BASELINE targets
(SURVEY Appendix C Re table).  CPU only."""
import glob
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFS = sorted(glob.glob(os.path.join(ROOT, "configs", "*.conf")))

# name -> (NX, NY, Nz_physical, Re, GPU counts it must decompose onto)
EXPECTED = {
    "poiseuille_32x33x32": (32, 33, 32, 100.0, [1, 2]),
    "retau180_128x129x128": (128, 129, 128, 3130.0, [1, 2]),
    "retau550_512x257x512": (512, 257, 512, 11150.0, [1, 2]),
    "retau950_1024x385x1024": (1024, 385, 1024, 20700.0, [1, 2, 4, 8]),
    "retau2000_2048x633x2048": (2048, 633, 2048, 48300.0, [1, 8]),
}


def test_every_baseline_config_shipped():
    names = {os.path.splitext(os.path.basename(c))[0] for c in CONFS}
    assert set(EXPECTED) <= names


@pytest.mark.parametrize("path", CONFS, ids=lambda p: os.path.basename(p))
def test_config_parses_and_plans(native, path):
    from channel_gpu_amd.utils.config import load_config

    c = load_config(path)
    c.validate()
    name = os.path.splitext(os.path.basename(path))[0]
    if name not in EXPECTED:
        return
    NX, NY, NZP, Re, gpus = EXPECTED[name]
    assert (c.NX, c.NY, 2 * c.NZ - 2) == (NX, NY, NZP)
    assert c.Re == Re and c.Q == 1.8
    for P in gpus:
        lines = 0
        for r in range(P):
            p = native.Plan.make(c, P, r)
            lines += p.nkx_loc * p.nkz_loc
            assert p.R * 64 >= NY
        p0 = native.Plan.make(c, P, 0)
        assert lines == p0.nkx * p0.nkz


@pytest.mark.parametrize("preset,conf", [("retau180", "retau180_128x129x128"), ("retau550", "retau550_512x257x512"),
                                         ("retau950", "retau950_1024x385x1024"), ("retau2000", "retau2000_2048x633x2048")])
def test_presets_match_shipped_configs(native, preset, conf):
    """The Python presets and the configs/*.conf files name the same physical case."""
    from channel_gpu_amd.utils.config import load_config, reference_preset

    p = reference_preset(preset)
    c = load_config(os.path.join(ROOT, "configs", conf + ".conf"))
    assert (p.NX, p.NY, p.NZ, p.Re, p.Q) == (c.NX, c.NY, c.NZ, c.Re, c.Q)
