"""Slab- and pencil-decomposed solver on CPU ranks (torch.distributed gloo): the same block
addressing as the GPU all-to-alls; P ranks must reproduce the P=1 trajectory.

Slab: world 2 and 3 (Pr = 1).  Pencil: 2 x 1 (only the kz <-> x exchange), 2 x 2 and 3 x 1
(uneven kz / x splits); the reference had the slab only."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from channel_gpu_amd.reference import oracle as ora

GRID = dict(NX=32, NY=33, NZ=17)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_state():
    plan = ora.OraclePlan(**GRID)
    ops = ora.build_ops(GRID["NY"])
    phi, om = ora.random_state(plan, ops, seed=11, amp=0.3)
    U = 0.75 * 1.8 * (1 - ops.y ** 2)
    return phi, om, U


def _worker(rank, world, port, outdir, nsteps, pr=1):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = ora.OracleSolver(**GRID, Re=400.0, dt_fixed=0.01, P=world, rank=rank, Pr=pr)
        phi, om, U = _global_state()
        p = o.plan
        sl = slice(p.kx0, p.kx0 + p.nkx_loc)
        sz = slice(p.kz0, p.kz0 + p.nkz_loc)
        o.set_state(phi[:, sl, sz], om[:, sl, sz], U)
        for _ in range(nsteps):
            o.step()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), phi=o.phi, om=o.om, U=o.U, kx0=p.kx0, kz0=p.kz0,
                 stats=o.plane_stats())
    finally:
        dist.destroy_process_group()


def _assemble(parts, field):
    nkx = sum(q[field].shape[1] for q in parts if int(q["kz0"]) == 0)
    nkz = sum(q[field].shape[2] for q in parts if int(q["kx0"]) == 0)
    out = np.zeros((parts[0][field].shape[0], nkx, nkz), complex)
    for q in parts:
        a, b = int(q["kx0"]), int(q["kz0"])
        out[:, a:a + q[field].shape[1], b:b + q[field].shape[2]] = q[field]
    return out


@pytest.mark.parametrize("world,pr", [(2, 1), (3, 1), (2, 2), (4, 2), (3, 3)])
def test_decomposition_equals_single_rank(world, pr):
    nsteps = 2
    ref = ora.OracleSolver(**GRID, Re=400.0, dt_fixed=0.01)
    phi, om, U = _global_state()
    ref.set_state(phi, om, U)
    for _ in range(nsteps):
        ref.step()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, nsteps, pr), nprocs=world, join=True,
                           start_method="spawn")
        parts = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    gphi = _assemble(parts, "phi")
    gom = _assemble(parts, "om")
    # plane statistics: the per-rank partial sums add up to the single-rank sums
    st = sum(q["stats"] for q in parts)
    assert np.allclose(st, ref.plane_stats(), rtol=1e-10, atol=1e-14)
    assert np.abs(gphi - ref.phi).max() < 1e-11 * np.abs(ref.phi).max()
    assert np.abs(gom - ref.om).max() < 1e-11 * np.abs(ref.om).max()
    assert np.abs(parts[0]["U"] - ref.U).max() < 1e-13
