"""Restart/UMEAN formats: HDF5 dataset "u", float32, dims {NX, NY, 2NZ},
planes in [kz][y][re,im] order; UMEAN raw {float U, float 0} records.  Runs on CPU."""
import os
import struct

import numpy as np
import pytest


@pytest.fixture()
def h5(native):
    if not native.hdf5_available():
        pytest.skip("libhdf5 not available")
    return native


def test_h5_planes_roundtrip(h5, tmp_path):
    NX, NY, NZ = 16, 9, 5
    path = str(tmp_path / "G.h5")
    h5.h5_create_field(path, NX, NY, NZ, False)
    rng = np.random.default_rng(0)
    planes = [0, 3, 15]
    data = rng.standard_normal(len(planes) * NY * 2 * NZ).astype(np.float32).astype(np.float64)
    h5.h5_write_planes(path, planes, list(data))
    got, dims = h5.h5_read_planes(path, planes)
    assert dims == [NX, NY, 2 * NZ]
    assert np.array_equal(np.asarray(got), data)
    # untouched planes read back as zeros
    z, _ = h5.h5_read_planes(path, [1, 2])
    assert not np.any(np.asarray(z))


def test_h5_attributes(h5, tmp_path):
    path = str(tmp_path / "DDV.h5")
    h5.h5_create_field(path, 8, 5, 3, False)
    h5.h5_write_attrs(path, {"time": 12.5, "dt": 1e-3, "step": 40.0})
    a = h5.h5_read_attrs(path)
    assert a["time"] == 12.5 and a["dt"] == 1e-3 and a["step"] == 40.0


def test_umean_format(native, tmp_path):
    path = str(tmp_path / "Umean.bin")
    U = [0.0, 1.5, 2.25, 0.0]
    native.umean_write(path, U)
    raw = open(path, "rb").read()
    assert len(raw) == 8 * len(U)
    vals = struct.unpack(f"<{2 * len(U)}f", raw)
    assert list(vals[0::2]) == U and not any(vals[1::2])
    assert native.umean_read(path, 4) == U


def test_missing_file_raises(h5, tmp_path):
    with pytest.raises(RuntimeError):
        h5.h5_read_planes(str(tmp_path / "nope.h5"), [0])


def test_truncated_checkpoint_raises(h5, tmp_path):
    """Fault injection: a checkpoint cut short (e.g. the writer died) must fail loudly, not load garbage."""
    NX, NY, NZ = 16, 9, 5
    path = str(tmp_path / "G.h5")
    h5.h5_create_field(path, NX, NY, NZ, False)
    h5.h5_write_planes(path, list(range(NX)), list(np.ones(NX * NY * 2 * NZ)))
    size = os.path.getsize(path)
    with open(path, "r+b") as f:
        f.truncate(size // 2)
    with pytest.raises(RuntimeError):
        h5.h5_read_planes(path, list(range(NX)))


def test_garbage_checkpoint_raises(h5, tmp_path):
    path = tmp_path / "DDV.h5"
    path.write_bytes(b"not an hdf5 file" * 64)
    with pytest.raises(RuntimeError):
        h5.h5_read_planes(str(path), [0])


def test_h5_fp64_dataset_roundtrip_exact(h5, tmp_path):
    """fp64 storage writes an H5T_NATIVE_DOUBLE dataset (hit_mpi.c:92-255 convention): bit-exact."""
    NX, NY, NZ = 16, 9, 5
    path = str(tmp_path / "G64.h5")
    h5.h5_create_field(path, NX, NY, NZ, True)
    rng = np.random.default_rng(1)
    data = rng.standard_normal(2 * NY * 2 * NZ)
    h5.h5_write_planes(path, [2, 7], list(data))
    got, dims = h5.h5_read_planes(path, [2, 7])
    assert np.array_equal(np.asarray(got), data)


def test_h5_create_writes_only_dealiased_planes(h5, tmp_path):
    """With Kx given, only the dealiased planes (|kx| > Kx) are zero-written at creation; unwritten
    retained planes still read as the zero fill value."""
    NX, NY, NZ, Kx = 32, 9, 5, 10
    path = str(tmp_path / "G.h5")
    h5.h5_create_field(path, NX, NY, NZ, False, Kx)
    z, dims = h5.h5_read_planes(path, list(range(NX)))
    assert dims == [NX, NY, 2 * NZ] and not np.any(np.asarray(z))


def test_h5_vector_dataset(h5, tmp_path):
    path = str(tmp_path / "G.h5")
    h5.h5_create_field(path, 8, 5, 3, False)
    v = np.linspace(0.1, 1.7, 5) / 3.0
    h5.h5_write_vector(path, "umean", list(v))
    ok, got = h5.h5_read_vector(path, "umean")
    assert ok and np.array_equal(np.asarray(got), v)
    ok2, _ = h5.h5_read_vector(path, "nothere")
    assert not ok2
