"""Slab- and pencil-decomposed GPU solver with P ranks sharing the one GPU of the test box.

RCCL refuses two ranks on one device, so these runs use the host shared-memory communicator
(ShmComm, "shm:" unique id), which drives exactly the same send/recv block addressing, x-transform
source/destination tables and reductions as the RCCL path.  The P-rank trajectory must equal the
NumPy oracle, and a restart written by P ranks must be readable by one rank.
"""
import os
import tempfile
import uuid

import numpy as np
import pytest
import torch.multiprocessing as mp

from channel_gpu_amd.reference import oracle as ora

pytestmark = pytest.mark.gpu

GRID = dict(NX=32, NY=33, NZ=17)


def _global_state():
    plan = ora.OraclePlan(**GRID)
    ops = ora.build_ops(GRID["NY"])
    phi, om = ora.random_state(plan, ops, seed=5, amp=0.3)
    return phi, om, 0.75 * 1.8 * (1 - ops.y ** 2)


def _worker(rank, world, shm, outdir, nsteps, pr=1):
    import torch  # noqa: F401

    from channel_gpu_amd import require_native
    from channel_gpu_amd.utils.config import default_config

    C = require_native()
    cfg = default_config(**GRID, Re=400.0, precision="fp64", dt_fixed=0.01, ic="zero", stats_every=0,
                         log_every=0, symmetry_every=0, decomposition="pencil" if pr > 1 else "slab", pr=pr)
    s = C.Solver(cfg, rank, world, 0, shm.encode())
    p = s.plan
    assert p.Pr == pr and p.Pr * p.Pc == world
    phi, om, U = _global_state()
    sl = slice(p.kx0, p.kx0 + p.nkx_loc)
    sz = slice(p.kz0, p.kz0 + p.nkz_loc)
    s.set_state(np.ascontiguousarray(phi[:, sl, sz]), np.ascontiguousarray(om[:, sl, sz]), U)
    s.prepare()
    for _ in range(nsteps):
        s.step(False)
    gphi, gom, gU = s.get_state()
    if C.hdf5_available():
        s.write_restart(os.path.join(outdir, "G.h5"), os.path.join(outdir, "DDV.h5"), os.path.join(outdir, "U.bin"))
        s.checkpoint_async(os.path.join(outdir, "Ga.h5"), os.path.join(outdir, "DDVa.h5"), "-")
        s.wait_checkpoint()
    s.symmetrize()  # distributed kz=0 column exchange
    sphi, som, _ = s.get_state()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), phi=gphi, om=gom, U=gU, sphi=sphi, som=som, health=s.health(),
             kx0=p.kx0, kz0=p.kz0)
    del s


def _assemble(parts, field):
    nkx = sum(q[field].shape[1] for q in parts if int(q["kz0"]) == 0)
    nkz = sum(q[field].shape[2] for q in parts if int(q["kx0"]) == 0)
    out = np.zeros((parts[0][field].shape[0], nkx, nkz), complex)
    for q in parts:
        a, b = int(q["kx0"]), int(q["kz0"])
        out[:, a:a + q[field].shape[1], b:b + q[field].shape[2]] = q[field]
    return out


@pytest.mark.parametrize("world,pr,chunk,self_mode,kzb", [(2, 1, "0", "direct", "0"), (3, 1, "0", "direct", "0"),
                                                          (3, 1, "4", "direct", "0"), (2, 1, "1", "direct", "0"),
                                                          (3, 1, "4", "copy", "0"), (2, 2, "0", "direct", "0"),
                                                          (4, 2, "0", "direct", "0"), (4, 2, "4", "direct", "0"),
                                                          (4, 2, "5", "copy", "0"), (6, 2, "3", "direct", "0"),
                                                          (6, 3, "4", "direct", "0"),
                                                          (3, 1, "8", "direct", "1"), (2, 1, "0", "copy", "1"),
                                                          (4, 2, "8", "direct", "1"), (6, 2, "8", "direct", "1")])
def test_multirank_matches_oracle(native, monkeypatch, world, pr, chunk, self_mode, kzb):
    """chunk: y planes per exchange chunk of the slab and pencil pipelines (0 = whole slab; 4 with
    NY=33 over 3 ranks gives uneven ranks a different number of non-empty chunks); self_mode: own
    block in place (direct) or copied inside the exchange (copy).  pr > 1: pencil grids pr x
    world/pr, the chunked software pipeline with the row-group (B) exchange on its own group
    communicator.  kzb = 1: the blocked spectral layout at P > 1 (CHANNEL_SPEC_KZB=1; the default at
    R = 7, 8): y split in whole 8-plane tiles (NY = 33 over 3: 8 / 16 / 9 rows), exchange blocks
    and segments in tiles, the distributed kz = 0 symmetrisation on blocked fields."""
    monkeypatch.setenv("CHANNEL_YCHUNK", chunk)
    monkeypatch.setenv("CHANNEL_A2A_SELF", self_mode)
    monkeypatch.setenv("CHANNEL_SPEC_KZB", kzb)
    nsteps = 2
    ref = ora.OracleSolver(**GRID, Re=400.0, dt_fixed=0.01)
    phi, om, U = _global_state()
    ref.set_state(phi, om, U)
    for _ in range(nsteps):
        ref.step()
    shm = f"shm:chtest_{uuid.uuid4().hex[:12]}"
    with tempfile.TemporaryDirectory() as d:
        # a turn marker left behind by a crashed earlier run of the same checkpoint path, in the
        # pre-nonce format "<serial> <turn>": it must not let rank 1 start writing before rank 0 has
        # created the file (the planes of rank 1 would be lost without an error)
        with open(os.path.join(d, "Ga.h5.turn"), "w") as f:
            f.write("1 1\n")
        mp.start_processes(_worker, args=(world, shm, d, nsteps, pr), nprocs=world, join=True,
                           start_method="spawn")
        parts = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
        gphi = _assemble(parts, "phi")
        gom = _assemble(parts, "om")
        assert all(int(q["health"]) == 0 for q in parts)
        assert np.abs(gphi - ref.phi).max() < 1e-9 * np.abs(ref.phi).max()
        assert np.abs(gom - ref.om).max() < 1e-9 * np.abs(ref.om).max()
        assert np.abs(parts[0]["U"] - ref.U).max() < 1e-11
        # distributed symmetrisation: 0.5 (q(kx) + conj q(-kx)) on the kz = 0 plane
        for f, sf in (("phi", "sphi"), ("om", "som")):
            g, sg = _assemble(parts, f), _assemble(parts, sf)
            nkx = g.shape[1]
            want = g.copy()
            neg = (-np.arange(nkx)) % nkx
            want[:, :, 0] = 0.5 * (g[:, :, 0] + np.conj(g[:, neg, 0]))
            assert np.allclose(sg, want, rtol=0, atol=1e-15 * np.abs(g).max())
        if native.hdf5_available():
            from channel_gpu_amd.utils.config import default_config

            cfg = default_config(**GRID, Re=400.0, precision="fp64", ic="zero", stats_every=0, log_every=0)
            s1 = native.Solver(cfg, 0, 1, 0, b"")
            # no UMEAN file named: U from the full-precision 'umean' dataset of the G file
            s1.read_restart(os.path.join(d, "G.h5"), os.path.join(d, "DDV.h5"), "-")
            rphi, rom, rU = s1.get_state()
            gphi, gom = _assemble(parts, "phi"), _assemble(parts, "om")
            # fp64 storage writes float64 datasets and U at full precision: exact
            assert np.array_equal(rphi, gphi) and np.array_equal(rom, gom)
            assert np.abs(rU - ref.U).max() < 1e-11
            # the companion UMEAN file (float32 records of the same profile): the full-precision copy
            s1.read_restart(os.path.join(d, "G.h5"), os.path.join(d, "DDV.h5"), os.path.join(d, "U.bin"))
            assert np.array_equal(s1.get_state()[2], rU)
            # an edited UMEAN file wins over the profile stored in G
            u_edit = np.fromfile(os.path.join(d, "U.bin"), dtype=np.float32)
            u_edit[2 * (len(u_edit) // 4)] *= 1.5  # U of the middle row (records are float32 pairs)
            u_edit.tofile(os.path.join(d, "U2.bin"))
            s1.read_restart(os.path.join(d, "G.h5"), os.path.join(d, "DDV.h5"), os.path.join(d, "U2.bin"))
            fU = s1.get_state()[2]
            assert not np.array_equal(fU, rU) and np.abs(fU - rU).max() > 0.1 * np.abs(rU).max()
            # the background writer (ranks passing the file by marker files) wrote the same data
            s2 = native.Solver(cfg, 0, 1, 0, b"")
            s2.read_restart(os.path.join(d, "Ga.h5"), os.path.join(d, "DDVa.h5"), "-")
            aphi, aom, _ = s2.get_state()
            assert np.array_equal(aphi, rphi) and np.array_equal(aom, rom)
            assert not any(f.endswith(".turn") for f in os.listdir(d))


def _worker_big(rank, world, shm, outdir, grid, nsteps, pr=1):
    import torch  # noqa: F401

    from channel_gpu_amd import require_native
    from channel_gpu_amd.utils.config import default_config

    C = require_native()
    cfg = default_config(**grid, Re=2000.0, precision="fp64", ic="random", ic_amplitude=0.05, stats_every=0,
                         log_every=0, symmetry_every=0, decomposition="pencil" if pr > 1 else "slab", pr=pr)
    s = C.Solver(cfg, rank, world, 0, shm.encode())
    s.init_ic()  # deterministic and independent of P
    s.prepare()
    for _ in range(nsteps):
        s.step(False)
    p = s.plan
    phi, om, U = s.get_state()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), phi=phi, om=om, U=U, kx0=p.kx0, kz0=p.kz0, dt=s.log().dt,
             health=s.health())
    del s


@pytest.mark.parametrize("pr", [1, 2])
def test_eight_ranks_uneven_realistic_shape(native, monkeypatch, pr):
    """8 ranks at an uneven split like the headline's, y-chunked exchanges with a ragged last chunk:
    bitwise the single-rank run (the arithmetic is identical; only the data movement differs).
    pr = 1: slab (NY = 385 over 8: 49/48 rows, 43 retained kx over 8: 6/5 columns); pr = 2: the
    2 x 4 pencil (97/96 rows and 11/10 kx columns per process row, 22 kz and 64 x split in two)."""
    grid = dict(NX=64, NY=385, NZ=33)
    monkeypatch.setenv("CHANNEL_YCHUNK", "16")
    monkeypatch.setenv("CHANNEL_SHM_SLOT_MB", "8")
    # the slab runs the combine mode (the P <= 4 default, forced here), the pencil the six-output
    # mode (the default at 8 ranks); the single-rank reference runs the same mode (spawned ranks
    # inherit the environment at spawn)
    combine = "1" if pr == 1 else "0"
    monkeypatch.setenv("CHANNEL_COMBINE", combine)
    world, nsteps = 8, 2
    shm = f"shm:chtest8_{uuid.uuid4().hex[:12]}"
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker_big, args=(world, shm, d, grid, nsteps, pr), nprocs=world, join=True,
                           start_method="spawn")
        parts = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    from channel_gpu_amd.utils.config import default_config

    cfg = default_config(**grid, Re=2000.0, precision="fp64", ic="random", ic_amplitude=0.05, stats_every=0,
                         log_every=0, symmetry_every=0)
    # the single-rank reference in the ranks' mode (combine: K-SPEC's D1 v / v / D1 omega outputs,
    # the combining x-backward), the arithmetic the 8 ranks run
    s1 = native.Solver(cfg, 0, 1, 0, b"")
    assert s1.combine() == (combine == "1")
    s1.init_ic()
    s1.prepare()
    for _ in range(nsteps):
        s1.step(False)
    rphi, rom, rU = s1.get_state()
    assert all(int(q["health"]) == 0 for q in parts)
    assert len({float(q["dt"]) for q in parts}) == 1 and float(parts[0]["dt"]) == s1.log().dt
    gphi, gom = _assemble(parts, "phi"), _assemble(parts, "om")
    assert np.array_equal(gphi, rphi) and np.array_equal(gom, rom)
    assert np.array_equal(parts[0]["U"], rU)
