"""Failure detection, rollback and fault injection.

The reference's only failure handling was printf + exit(1) on the failing rank (check.cu:3-79):
peers then blocked forever in the next MPI call, and NaNs went unnoticed into the statistics.
Here: a device health flag is reduced over all ranks every ``health_every`` steps; ``on_nan =
"abort"`` aborts every rank, ``on_nan = "rollback"`` restores the last in-memory snapshot and
retries with a smaller CFL; a dead peer makes the surviving ranks raise instead of hanging.
"""
import multiprocessing as mpc
import os
import time
import uuid

import numpy as np
import pytest

from channel_gpu_amd.utils.config import default_config

pytestmark = pytest.mark.gpu

BASE = dict(NX=32, NY=33, NZ=17, Re=1000.0, precision="fp32", ic="random", ic_amplitude=0.2, stats_every=0,
            log_every=0, symmetry_every=0)


def test_nan_aborts(native):
    s = native.Solver(default_config(**BASE, health_every=1), 0, 1, 0, b"")
    s.init_ic()
    s.run(2, False)
    assert s.health() == 0
    s.inject_nan()
    with pytest.raises(RuntimeError, match="health check failed"):
        s.run(3, False)


def test_nan_rollback_recovers(native):
    s = native.Solver(default_config(**BASE, health_every=2, on_nan="rollback", snapshot_every=2, max_rollbacks=2),
                      0, 1, 0, b"")
    s.init_ic()
    s.run(4, False)
    assert s.snapshot_step() == 4
    cfl0 = s.cfl()
    s.inject_nan()
    s.run(4, False)           # NaN found at step 6 -> back to step 4, then 4 more steps
    assert s.rollbacks() == 1
    assert s.cfl() == pytest.approx(0.5 * cfl0)
    assert s.steps_done() == 8
    assert s.health() == 0
    phi, om, U = s.get_state()
    assert np.isfinite(phi).all() and np.isfinite(om).all() and np.isfinite(U).all()


def test_rollback_limit_then_abort(native):
    s = native.Solver(default_config(**BASE, health_every=1, on_nan="rollback", max_rollbacks=0), 0, 1, 0, b"")
    s.init_ic()
    s.run(1, False)
    s.inject_nan()
    with pytest.raises(RuntimeError):
        s.run(2, False)


def _peer(rank, shm, q, decomposition="slab"):
    os.environ["CHANNEL_COMM_TIMEOUT_S"] = "5"
    from channel_gpu_amd import require_native

    C = require_native()
    s = C.Solver(default_config(**BASE, decomposition=decomposition, pr=2 if decomposition == "pencil" else 0),
                 rank, 2, 0, shm.encode())
    s.init_ic()
    s.run(2, False)
    if rank == 1:
        os._exit(3)           # simulated rank death: no clean-up, no further collectives
    t0 = time.time()
    try:
        s.run(5, False)
        q.put(("no-error", time.time() - t0))
    except RuntimeError as e:
        t1 = time.time()
        # every communicator (the pencil's per-axis groups too) was aborted: tearing the solver
        # down must not block on the dead exchange
        del s
        q.put(("raised", t1 - t0, str(e), time.time() - t1))


@pytest.mark.parametrize("decomposition", ["slab", "pencil"])
def test_dead_peer_raises_instead_of_hanging(native, decomposition):
    ctx = mpc.get_context("spawn")
    q = ctx.Queue()
    shm = f"shm:chfail_{uuid.uuid4().hex[:12]}"
    ps = [ctx.Process(target=_peer, args=(r, shm, q, decomposition)) for r in range(2)]
    for p in ps:
        p.start()
    res = q.get(timeout=240)
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert res[0] == "raised", res
    assert res[1] < 60
    assert res[3] < 30, f"solver teardown took {res[3]:.1f} s after the failure"
    assert ps[1].exitcode == 3
