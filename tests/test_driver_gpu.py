"""Driver programs (C++ bin/channel_mi355x and python -m channel_gpu_amd.driver): run.conf in,
reference-format restart + statistics files out; multi-rank launch; restart continuation."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "channel_mi355x")

CONF = """application:
{{
  NX = 32; NY = 33; NZ = 17;
  input: {{ G = "{gin}"; DDV = "{din}"; UMEAN = "{uin}"; }};
  output: {{ G = "{d}/G.h5"; DDV = "{d}/DDV.h5"; UMEAN = "{d}/Umean.bin"; }};
  path = "{d}/";
  Re = 400.0; nsteps = {n}; stats_every = 2; log_every = 1; precision = "fp64"; dt_fixed = 0.01;
  ic = "{ic}"; ic_amplitude = 0.3;
}};
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _write_conf(d, n=4, ic="random", gin="-", din="-", uin="-"):
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, "run.conf")
    with open(p, "w") as f:
        f.write(CONF.format(d=d, n=n, ic=ic, gin=gin, din=din, uin=uin))
    return p


def _read_field(native, path, NX=32):
    data, dims = native.h5_read_planes(path, list(range(NX)))
    return np.asarray(data), dims


def test_cpp_driver_single_rank(native, tmp_path):
    if not os.path.exists(BIN):
        pytest.skip("driver not built")
    d = str(tmp_path / "one")
    conf = _write_conf(d)
    r = subprocess.run([BIN, conf], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "MEAN_PROFILE_STATISTICS" in r.stdout and "ms/step" in r.stdout
    for f in ["G.h5", "DDV.h5", "Umean.bin", "MEANPROFILE.dat", "UTAU.dat", "STATISTICS.dat", "RESOLUTION.dat",
              "URMS.dat", "VRMS.dat", "WRMS.dat", "RSTRSS.dat", "MEANREAYNOLDS.dat"]:
        assert os.path.exists(os.path.join(d, f)), f
    assert len(open(os.path.join(d, "UTAU.dat")).read().split()) == 4  # one record per step
    if native.hdf5_available():
        g, dims = _read_field(native, os.path.join(d, "G.h5"))
        assert dims == [32, 33, 34] and np.isfinite(g).all() and np.abs(g).max() > 0


def test_cpp_driver_two_ranks_equal_one(native, tmp_path):
    if not os.path.exists(BIN) or not native.hdf5_available():
        pytest.skip("driver or hdf5 missing")
    d1, d2 = str(tmp_path / "p1"), str(tmp_path / "p2")
    c1, c2 = _write_conf(d1), _write_conf(d2)
    # (the one-rank run in the combine mode the two ranks use: the same arithmetic)
    assert subprocess.run([BIN, c1, "--quiet"], capture_output=True, timeout=300,
                          env=dict(os.environ, CHANNEL_COMBINE="1")).returncode == 0
    port = _port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CHANNEL_COMM="shm")
        procs.append(subprocess.Popen([BIN, c2, "--quiet"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    for p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err.decode()
    for f in ["G.h5", "DDV.h5"]:
        a, _ = _read_field(native, os.path.join(d1, f))
        b, _ = _read_field(native, os.path.join(d2, f))
        assert np.array_equal(a, b), f  # identical per-line / per-row arithmetic at any P


def test_restart_continuation(native, tmp_path):
    if not os.path.exists(BIN) or not native.hdf5_available():
        pytest.skip("driver or hdf5 missing")
    da, db, dc = str(tmp_path / "a"), str(tmp_path / "b"), str(tmp_path / "c")
    assert subprocess.run([BIN, _write_conf(da, n=6), "--quiet"], capture_output=True, timeout=300).returncode == 0
    assert subprocess.run([BIN, _write_conf(db, n=3), "--quiet"], capture_output=True, timeout=300).returncode == 0
    cc = _write_conf(dc, n=3, ic="file", gin=f"{db}/G.h5", din=f"{db}/DDV.h5", uin=f"{db}/Umean.bin")
    assert subprocess.run([BIN, cc, "--quiet"], capture_output=True, timeout=300).returncode == 0
    a, _ = _read_field(native, os.path.join(da, "DDV.h5"))
    c, _ = _read_field(native, os.path.join(dc, "DDV.h5"))
    # the restart files hold float32 (reference format): continuation agrees to fp32 round-off
    assert np.abs(a - c).max() < 1e-5 * np.abs(a).max()
    attrs = native.h5_read_attrs(os.path.join(dc, "G.h5"))
    assert attrs["step"] == 6.0 and abs(attrs["time"] - 0.06) < 1e-12


def test_python_driver(tmp_path):
    d = str(tmp_path / "py")
    conf = _write_conf(d, n=2)
    r = subprocess.run([sys.executable, "-m", "channel_gpu_amd.driver", conf, "--quiet"], capture_output=True,
                       text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    assert "grid-pts/s" in r.stdout
    assert os.path.exists(os.path.join(d, "DDV.h5"))
