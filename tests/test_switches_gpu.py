"""Opt-in kernel variants behind environment switches, each checked in a fresh child process (the
switches are read once per process): CHANNEL_ZFFT (z-stage row plans, incl. the paired-row H_z of
ZFFT=4 on odd row counts) against NumPy, CHANNEL_KSPEC_W8 (K-SPEC at 8 lines, two waves per SIMD)
against the fp64 oracle, CHANNEL_XSEGROWS=0 (per-element exchange-segment lookups of the P > 1 x
kernels) bitwise against the single-rank fast path.  README "Environment switches" lists them."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ZSTAGE_SCRIPT = r"""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.environ["CHANNEL_ROOT"])
from channel_gpu_amd import require_native
C = require_native()
rng = np.random.default_rng(7)
Nzp = 1024
nkz = Nzp // 3 + 1
for dtype, tol in ((torch.complex64, 5e-6), (torch.complex128, 1e-12)):
    # rows = ny * NX (a multiple of the block's 4 rows): 48 and 40 rows give every wave of the
    # persistent grid one row (ZFFT=4: the unpaired tail path), 3072 rows more groups than the
    # grid holds (blocks walk one or two groups: paired and unpaired waves)
    for NX, ny in ((16, 3), (8, 5), (64, 48)):
        f = rng.standard_normal((6, ny, NX, nkz)) + 1j * rng.standard_normal((6, ny, NX, nkz))
        f[..., 0] = f[..., 0].real
        H, m = C.zphys(torch.tensor(f, dtype=dtype, device="cuda"), Nzp, torch.ones(ny, dtype=torch.float64), 1.0, 1.0)
        phys = np.fft.irfft(np.concatenate([f, np.zeros(f.shape[:-1] + (Nzp // 2 + 1 - nkz,))], -1), n=Nzp,
                            axis=-1, norm="forward")
        u, v, w, wx, wy, wz = phys
        Hp = np.stack([v * wz - w * wy, w * wx - u * wz, u * wy - v * wx])
        Href = np.fft.rfft(Hp, axis=-1, norm="forward")[..., :nkz] / NX
        e = np.linalg.norm(H.cpu().numpy() - Href) / np.linalg.norm(Href)
        assert e < tol, (dtype, NX, ny, e)
        assert abs(m.cpu().numpy()[0] - np.abs(u).max()) < 1e-4 * np.abs(u).max()
print("ZSTAGE_OK")
"""


def _child(script, env_extra, token, timeout=300):
    env = dict(os.environ, CHANNEL_ROOT=ROOT, **env_extra)
    r = subprocess.run([sys.executable, "-c", script], env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0 and token in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


@pytest.mark.parametrize("mode", ["0", "1", "2", "4"])
def test_zfft_row_plans(mode):
    """CHANNEL_ZFFT = 0 (LDS twiddles), 1 (register twiddles), 2 (16 x 16 x 4 with pad-per-32 rows),
    4 (paired-row H_z: two rows' H_z as one transform, the odd row of a wave through hzbuf, alone);
    the default 3 runs in test_kernels_gpu.py::test_zphys."""
    _child(ZSTAGE_SCRIPT, {"CHANNEL_ZFFT": mode}, "ZSTAGE_OK")


W8_SCRIPT = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.environ["CHANNEL_ROOT"])
from channel_gpu_amd import require_native
from channel_gpu_amd.reference import oracle as ora
from channel_gpu_amd.utils.config import default_config
C = require_native()
NX, NY, NZ, dt = 16, 385, 9, 1e-4
cfg = default_config(NX=NX, NY=NY, NZ=NZ, Re=400.0, precision="fp32", dt_fixed=dt, stats_every=0, log_every=0,
                     symmetry_every=0, ic="zero")
s = C.Solver(cfg, 0, 1, 0, b"")
o = ora.OracleSolver(NX, NY, NZ, Re=400.0, dt_fixed=dt)
phi, om = ora.random_state(o.plan, o.ops, seed=5, amp=0.05)
phi = phi.astype(np.complex64).astype(np.complex128)
om = om.astype(np.complex64).astype(np.complex128)
U = 0.75 * 1.8 * (1 - o.ops.y ** 2)
o.set_state(phi, om, U)
s.set_state(phi, om, U)
s.prepare()
rel = lambda a, b: np.linalg.norm(a - b) / np.linalg.norm(b)
for it in range(2):
    o.step()
    s.step(False)
    gphi, gom, gU = s.get_state()
    assert rel(gphi, o.phi) < 1e-4 and rel(gom, o.om) < 1e-4 and rel(gU, o.U) < 1e-5, (it, rel(gphi, o.phi), rel(gom, o.om), rel(gU, o.U))
print("W8_OK")
"""


def test_kspec_w8_matches_oracle():
    """CHANNEL_KSPEC_W8=1: the R = 7 fp32 K-SPEC at 8 lines per workgroup (LEAN 2-RHS solves, async
    LDS staging) against the fp64 oracle at the one-wave kernel's fp32 tolerance
    (test_solver_gpu.py::test_gpu_matches_oracle_large_ny[fp32-385])."""
    _child(W8_SCRIPT, {"CHANNEL_KSPEC_W8": "1"}, "W8_OK")


SEGROWS_SCRIPT = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.environ["CHANNEL_ROOT"])
from channel_gpu_amd import require_native
from channel_gpu_amd.utils.config import default_config
C = require_native()
res = []
for uid in (b"", C.new_unique_id()):
    cfg = default_config(NX=64, NY=65, NZ=33, Re=1000.0, precision="fp64", ic="random", ic_amplitude=0.2,
                         stats_every=0, log_every=0, symmetry_every=0)
    s = C.Solver(cfg, 0, 1, 0, uid)
    s.init_ic()
    s.prepare()
    for _ in range(3):
        s.step(False)
    res.append(s.get_state())
    del s
for a, b in zip(res[0], res[1]):
    assert np.array_equal(a, b)
print("SEGROWS_OK")
"""


@pytest.mark.parametrize("combine", ["0", "1"])
def test_xsegrows_off_is_bitwise(combine):
    """CHANNEL_XSEGROWS=0: the P > 1 x kernels (1-rank RCCL communicator, 4 kx sub-blocks = 4
    exchange segments incl. the self blocks) with per-element segment lookups instead of the
    per-thread row tables, bitwise against the single-rank fast path; with K-SPEC's six outputs
    and in the combine mode (CHANNEL_COMBINE=1 on both sides)."""
    _child(SEGROWS_SCRIPT, {"CHANNEL_XSEGROWS": "0", "CHANNEL_COMBINE": combine}, "SEGROWS_OK")
