"""Independent decode of the restart files against the solver state (the
reference's writers: hit_mpi.c:257-339, io.c:37-72, meanUevol.c:153-176).

The files are written by the solver (csrc/core/solver.cpp write_restart_job -> csrc/core/io.cpp)
and read back here WITHOUT that code: the HDF5 C library is called through ctypes only for the
dataset's metadata (dims, stored type, layout, filters, file offset), and the values are taken as
raw bytes from the file at the dataset's offset with numpy.  A consistent mistake on both sides of
io.cpp (kz and y swapped, a wrong scale, a wrong plane order) would pass the round-trip tests but
fails here: the decoded planes are compared with N2 * get_state() in the reference's logical order
[kx plane in FFT order][kz][y][re, im], and the same bytes read in the swapped [y][kz] order must
NOT match.
"""
import ctypes
import os
import socket
import subprocess

import numpy as np
import pytest

from channel_gpu_amd.utils.config import default_config

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "channel_mi355x")
H5T_FLOAT, H5T_ORDER_LE, H5D_CONTIGUOUS = 1, 0, 1


def _h5lib():
    for c in (os.environ.get("CHANNEL_HDF5_LIB"), "libhdf5.so.103", "/opt/conda/lib/libhdf5.so.103", "libhdf5.so",
              "/opt/conda/lib/libhdf5.so"):
        if not c:
            continue
        try:
            return ctypes.CDLL(c)
        except OSError:
            pass
    return None


def read_dataset_raw(path, name="u"):
    """(values with the declared dims, stored item size) of a contiguous, unfiltered little-endian
    float dataset, taken from the file's bytes at the dataset's offset."""
    L = _h5lib()
    if L is None:
        pytest.skip("libhdf5 not available")
    hid, herr = ctypes.c_int64, ctypes.c_int
    L.H5open.restype = herr
    L.H5Fopen.restype, L.H5Fopen.argtypes = hid, [ctypes.c_char_p, ctypes.c_uint, hid]
    L.H5Dopen2.restype, L.H5Dopen2.argtypes = hid, [hid, ctypes.c_char_p, hid]
    L.H5Dget_space.restype, L.H5Dget_space.argtypes = hid, [hid]
    L.H5Dget_type.restype, L.H5Dget_type.argtypes = hid, [hid]
    L.H5Dget_create_plist.restype, L.H5Dget_create_plist.argtypes = hid, [hid]
    L.H5Dget_offset.restype, L.H5Dget_offset.argtypes = ctypes.c_uint64, [hid]
    L.H5Sget_simple_extent_ndims.restype, L.H5Sget_simple_extent_ndims.argtypes = ctypes.c_int, [hid]
    L.H5Sget_simple_extent_dims.restype = ctypes.c_int
    L.H5Sget_simple_extent_dims.argtypes = [hid, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    L.H5Tget_class.restype, L.H5Tget_class.argtypes = ctypes.c_int, [hid]
    L.H5Tget_size.restype, L.H5Tget_size.argtypes = ctypes.c_size_t, [hid]
    L.H5Tget_order.restype, L.H5Tget_order.argtypes = ctypes.c_int, [hid]
    L.H5Pget_layout.restype, L.H5Pget_layout.argtypes = ctypes.c_int, [hid]
    L.H5Pget_nfilters.restype, L.H5Pget_nfilters.argtypes = ctypes.c_int, [hid]
    for f in ("H5Tclose", "H5Sclose", "H5Pclose", "H5Dclose", "H5Fclose"):
        getattr(L, f).argtypes = [hid]
    assert L.H5open() >= 0
    H5P_DEFAULT, H5F_ACC_RDONLY = 0, 0
    fid = L.H5Fopen(path.encode(), H5F_ACC_RDONLY, H5P_DEFAULT)
    assert fid >= 0, path
    did = L.H5Dopen2(fid, name.encode(), H5P_DEFAULT)
    assert did >= 0, name
    sid, tid, pid = L.H5Dget_space(did), L.H5Dget_type(did), L.H5Dget_create_plist(did)
    nd = L.H5Sget_simple_extent_ndims(sid)
    dims = (ctypes.c_uint64 * nd)()
    L.H5Sget_simple_extent_dims(sid, dims, None)
    dims = tuple(int(d) for d in dims)
    cls, size, order = L.H5Tget_class(tid), L.H5Tget_size(tid), L.H5Tget_order(tid)
    layout, nfilt, off = L.H5Pget_layout(pid), L.H5Pget_nfilters(pid), L.H5Dget_offset(did)
    for f, h in (("H5Tclose", tid), ("H5Sclose", sid), ("H5Pclose", pid), ("H5Dclose", did), ("H5Fclose", fid)):
        getattr(L, f)(h)
    assert cls == H5T_FLOAT and order == H5T_ORDER_LE and size in (4, 8), (cls, order, size)
    assert layout == H5D_CONTIGUOUS and nfilt == 0, (layout, nfilt)  # plain bytes: no chunks, no filters
    raw = np.fromfile(path, dtype="<f4" if size == 4 else "<f8", count=int(np.prod(dims)), offset=int(off))
    return raw.reshape(dims), size


def decode_planes(u, NX, NY, NZ):
    """Appendix B1: dims {NX, NY, 2NZ} declared; logical order [kx plane][kz][y][re, im]."""
    assert u.shape == (NX, NY, 2 * NZ)
    c = u.reshape(NX, NZ, NY, 2)
    return c[..., 0] + 1j * c[..., 1]  # [plane][kz][y]


def expected_planes(q, NX, Kx, N2):
    """N2 * q (get_state layout [y][retained kx][kz]) placed at FFT-order planes [plane][kz][y]."""
    NY, nkx, nkz = q.shape
    out = np.zeros((NX, nkz, NY), complex)
    for i in range(nkx):
        kx = i if i <= Kx else i - nkx
        out[kx % NX] = (N2 * q[:, i, :]).T
    return out


def check_file(path, q, NX, NY, NZ, fp64):
    u, size = read_dataset_raw(path)
    assert size == (8 if fp64 else 4)
    got = decode_planes(u, NX, NY, NZ)
    Kx, Kz = NX // 3, (2 * NZ - 2) // 3
    N2 = NX * (2 * NZ - 2)
    want = np.zeros((NX, NZ, NY), complex)
    want[:, :q.shape[2], :] = expected_planes(q, NX, Kx, N2)
    if not fp64:  # the writer stores float32(N2 q): round the expectation the same way
        want = want.astype(np.complex64).astype(complex)
    scale = np.abs(want).max()
    assert scale > 0
    assert np.abs(got - want).max() <= (1e-12 if fp64 else 1e-7) * scale
    # dealiased modes are zero: planes of |kx| > Kx and kz > Kz
    kx_fft = np.where(np.arange(NX) < NX // 2, np.arange(NX), np.arange(NX) - NX)
    assert np.all(got[np.abs(kx_fft) > Kx] == 0)
    assert np.all(got[:, Kz + 1:, :] == 0)
    # the same bytes in the swapped (y, kz) order do not decode to the state
    c = u.reshape(NX, NY, NZ, 2)
    swapped = np.transpose(c[..., 0] + 1j * c[..., 1], (0, 2, 1))
    assert np.abs(swapped - want).max() > 1e-3 * scale
    return got


def check_umean(path, U, NY, N2):
    """Appendix B2: NY records of {float32 U N2, float32 0}, no header."""
    assert os.path.getsize(path) == 8 * NY
    r = np.fromfile(path, dtype="<f4").reshape(NY, 2)
    assert np.all(r[:, 1] == 0)
    assert np.array_equal(r[:, 0], (N2 * np.asarray(U)).astype(np.float32))


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_restart_files_decode_to_state(native, tmp_path, precision):
    if not native.hdf5_available():
        pytest.skip("hdf5 missing")
    NX, NY, NZ = 32, 33, 17
    cfg = default_config(NX=NX, NY=NY, NZ=NZ, Re=400.0, precision=precision, ic="random", ic_amplitude=0.3,
                         stats_every=0, log_every=0, dt_fixed=0.005)
    s = native.Solver(cfg, 0, 1, 0, b"")
    s.init_ic()
    s.prepare()
    for _ in range(2):
        s.step(False)
    g, d, um = (str(tmp_path / f) for f in ("G.h5", "DDV.h5", "Umean.bin"))
    s.write_restart(g, d, um)
    phi, om, U = s.get_state()
    fp64 = precision == "fp64"
    check_file(g, om, NX, NY, NZ, fp64)
    check_file(d, phi, NX, NY, NZ, fp64)
    check_umean(um, U, NY, NX * (2 * NZ - 2))


CONF = """application:
{{
  NX = 32; NY = 33; NZ = 17;
  input: {{ G = "-"; DDV = "-"; UMEAN = "-"; }};
  output: {{ G = "{d}/G.h5"; DDV = "{d}/DDV.h5"; UMEAN = "{d}/Umean.bin"; }};
  path = "{d}/";
  Re = 400.0; nsteps = 3; stats_every = 0; log_every = 1; precision = "fp64"; dt_fixed = 0.005;
  ic = "random"; ic_amplitude = 0.3;
}};
"""


def test_two_rank_driver_files_decode(native, tmp_path):
    """The per-rank hyperslab writes of a 2-rank driver run (shared-memory loopback: each rank
    writes its kx planes) decode to the same planes as a 1-rank run, with the layout checks above
    (dims, stored type, zero dealiased planes) on the decoded data.  fp64 storage (float64
    datasets): the per-line / per-row arithmetic is then bitwise the same at any P, as in
    test_driver_gpu.py::test_cpp_driver_two_ranks_equal_one."""
    if not os.path.exists(BIN) or not native.hdf5_available():
        pytest.skip("driver or hdf5 missing")
    runs = {}
    for P in (1, 2):
        d = str(tmp_path / f"p{P}")
        os.makedirs(d)
        conf = os.path.join(d, "run.conf")
        with open(conf, "w") as f:
            f.write(CONF.format(d=d))
        if P == 1:  # (in the combine mode the two ranks use: the same arithmetic)
            r = subprocess.run([BIN, conf, "--quiet"], capture_output=True, text=True, timeout=300,
                               env=dict(os.environ, CHANNEL_COMBINE="1"))
            assert r.returncode == 0, r.stderr
        else:
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
            sk.close()
            procs = []
            for rank in range(2):
                env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                           MASTER_PORT=str(port), CHANNEL_COMM="shm")
                procs.append(subprocess.Popen([BIN, conf, "--quiet"], env=env, stdout=subprocess.PIPE,
                                              stderr=subprocess.PIPE))
            for p in procs:
                _, err = p.communicate(timeout=300)
                assert p.returncode == 0, err.decode()
        runs[P] = {f: read_dataset_raw(os.path.join(d, f))[0] for f in ("G.h5", "DDV.h5")}
        runs[P]["umean"] = np.fromfile(os.path.join(d, "Umean.bin"), dtype="<f4")
    for f in ("G.h5", "DDV.h5"):
        a, b = runs[1][f], runs[2][f]
        assert a.dtype == np.float64 and a.shape == (32, 33, 34)
        assert np.array_equal(a, b), f
        got = decode_planes(b, 32, 33, 17)
        kx_fft = np.where(np.arange(32) < 16, np.arange(32), np.arange(32) - 32)
        assert np.all(got[np.abs(kx_fft) > 32 // 3] == 0) and np.all(got[:, (2 * 17 - 2) // 3 + 1:, :] == 0)
        assert np.abs(got).max() > 0
    assert np.array_equal(runs[1]["umean"], runs[2]["umean"])
