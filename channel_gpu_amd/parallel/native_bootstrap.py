"""Torch-free process bootstrap of the solver's communicator (one process per GPU).

The launcher (torchrun / ``python -m torch.distributed.run``, mpirun, srun) only provides the
environment: RANK/WORLD_SIZE/LOCAL_RANK (or the PMI/Open MPI/SLURM equivalents) and
MASTER_ADDR/MASTER_PORT.  Rank 0 creates the 128-byte ncclUniqueId and a native TCP rendezvous
(``tcp_broadcast``, csrc/core/bootstrap.cpp, at MASTER_PORT+11) hands it to every rank; the solver
then builds its own RCCL communicator on its own streams.  Nothing here imports torch, so the
process runs on /opt/rocm's HIP runtime and RCCL (the same stack as the C++ driver binary).

``CHANNEL_COMM=shm`` selects the shared-memory loopback data plane (several ranks on one GPU);
``CHANNEL_FORCE_COMM=1`` gives a single rank a real 1-rank communicator (the P > 1 pipeline).
The reference bootstrapped MPI and broadcast nx/ny/nz and one path string (main.c:25-43, 106).
"""
from __future__ import annotations

import dataclasses
import os
import uuid

from .._native import require_core


@dataclasses.dataclass
class RankInfo:
    rank: int
    world: int
    local: int
    device: int
    uid: bytes  # communicator id ("" = single-rank fast path)


def _comm_kind() -> str:
    return os.environ.get("CHANNEL_COMM", "rccl").lower()


def init_native(force: bool | None = None, timeout_s: int = 300) -> RankInfo:
    """Rank/size from the launcher env, device = local rank, communicator id on every rank."""
    C = require_core()
    pi = C.ProcInfo.from_env()
    ndev = C.device_count()
    shm = _comm_kind() == "shm"
    if force is None:
        force = os.environ.get("CHANNEL_FORCE_COMM", "0") == "1"
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", pi.size))
    if pi.size > 1 and not shm and ndev > 0 and local_world > ndev:
        raise RuntimeError(
            f"{local_world} ranks on this node but only {ndev} visible GPU(s): RCCL needs one GPU per rank "
            f"(it refuses two ranks on one device: 'Duplicate GPU detected'). Use a node with >= {local_world} "
            "GPUs, or CHANNEL_COMM=shm to rehearse the multi-rank path over the shared-memory loopback.")
    if ndev < 1:
        raise RuntimeError("no GPU visible")
    device = pi.local_rank % ndev
    uid = b""
    if pi.size > 1 or force:
        if pi.rank == 0:
            if shm:
                port = os.environ.get("MASTER_PORT", "0")
                uid = f"shm:channel_{port}_{os.getpid()}_{uuid.uuid4().hex[:8]}".encode()
            else:
                uid = C.new_unique_id()
        uid = C.tcp_broadcast(pi, uid, timeout_s) if pi.size > 1 else uid
    return RankInfo(pi.rank, pi.size, pi.local_rank, device, bytes(uid))
