"""Slab-decomposed solver on CPU ranks (torch.distributed gloo, world_size 2 and 3): the same
block addressing as the GPU all-to-alls; P ranks must reproduce the P=1 trajectory."""
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


def _worker(rank, world, port, outdir, nsteps):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = ora.OracleSolver(**GRID, Re=400.0, dt_fixed=0.01, P=world, rank=rank)
        phi, om, U = _global_state()
        p = o.plan
        sl = slice(p.kx0, p.kx0 + p.nkx_loc)
        o.set_state(phi[:, sl], om[:, sl], U)
        for _ in range(nsteps):
            o.step()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), phi=o.phi, om=o.om, U=o.U, kx0=p.kx0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_slab_equals_single_rank(world):
    nsteps = 2
    ref = ora.OracleSolver(**GRID, Re=400.0, dt_fixed=0.01)
    phi, om, U = _global_state()
    ref.set_state(phi, om, U)
    for _ in range(nsteps):
        ref.step()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, nsteps), nprocs=world, join=True,
                           start_method="spawn")
        parts = [np.load(os.path.join(d, f"r{r}.npz")) for r in range(world)]
    gphi = np.concatenate([q["phi"] for q in parts], axis=1)
    gom = np.concatenate([q["om"] for q in parts], axis=1)
    assert np.abs(gphi - ref.phi).max() < 1e-11 * np.abs(ref.phi).max()
    assert np.abs(gom - ref.om).max() < 1e-11 * np.abs(ref.om).max()
    assert np.abs(parts[0]["U"] - ref.U).max() < 1e-13
