"""Bootstrap of the solver's RCCL communicator from torch.distributed.

One process per GPU (torchrun / torch.distributed.run).  The solver owns its own RCCL
communicator (created in C++ with ncclCommInitRank) so its all-to-alls can be enqueued on its own
streams and captured in its hipGraph; torch.distributed is only used to agree on the 128-byte
ncclUniqueId (rank 0 creates it, broadcast_object_list distributes it) and for host-side barriers
and timing reductions.  That control plane is gloo (CPU) by default: it moves a few bytes, and a
second, torch-owned RCCL communicator per GPU would only cost HBM and init time.

``CHANNEL_COMM=shm`` swaps the RCCL data plane for the shared-memory loopback communicator
(ShmComm): same block addressing, host-staged copies.  It lets several ranks share one GPU (RCCL
refuses that: "Duplicate GPU detected"), so the whole torchrun bench/driver path can be rehearsed
on a one-GPU box.  The reference bootstrapped nothing: it used host MPI for all data
movement (channel_cuda_mpi.c:64-128) and bound rank%2 to a device (main.c:87).
"""
from __future__ import annotations

import os
import uuid

import torch
import torch.distributed as dist

from .._native import require_native


def dist_info() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from torch.distributed or the torchrun environment."""
    if dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
    else:
        rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", rank))
    return rank, world, local


def force_comm() -> bool:
    """CHANNEL_FORCE_COMM=1: run the distributed (exchange-based) pipeline even on one rank."""
    return os.environ.get("CHANNEL_FORCE_COMM", "0") == "1"


def nccl_unique_id(force: bool | None = None) -> bytes:
    """Create the communicator id on rank 0 and share it with every rank.

    RCCL ncclUniqueId by default; a "shm:<name>" id when CHANNEL_COMM=shm.  One rank gets an empty
    id (the single-rank fast path) unless ``force`` (default: CHANNEL_FORCE_COMM=1): then it gets
    its own id and the solver builds a real 1-rank communicator and runs the P > 1 pipeline."""
    rank, world, _ = dist_info()
    if force is None:
        force = force_comm()
    shm = os.environ.get("CHANNEL_COMM", "rccl").lower() == "shm"
    if world == 1:
        if not force:
            return b""
        return f"shm:channel_{os.getpid()}_{uuid.uuid4().hex[:10]}".encode() if shm else require_native().new_unique_id()
    if not dist.is_initialized():
        raise RuntimeError("world_size > 1 requires torch.distributed to be initialised")
    if os.environ.get("CHANNEL_COMM", "rccl").lower() == "shm":
        uid = f"shm:channel_{os.getpid()}_{uuid.uuid4().hex[:10]}".encode() if rank == 0 else None
    else:
        uid = require_native().new_unique_id() if rank == 0 else None
    obj = [uid]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def init_distributed(backend: str | None = None) -> tuple[int, int, int]:
    """Initialise torch.distributed from the torchrun environment if needed; set the device."""
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("CHANNEL_DIST_BACKEND", "gloo")
        dist.init_process_group(backend=backend)
    rank, world, local = dist_info()
    ndev = torch.cuda.device_count()
    shm = os.environ.get("CHANNEL_COMM", "rccl").lower() == "shm"
    if world > 1 and ndev > 0 and not shm:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if local_world > ndev:
            raise RuntimeError(
                f"{local_world} ranks on this node but only {ndev} visible GPU(s): RCCL needs one GPU per rank "
                f"(it refuses two ranks on one device: 'Duplicate GPU detected'). Use a node with >= {local_world} "
                "GPUs, or CHANNEL_COMM=shm to rehearse the multi-rank path over the shared-memory loopback.")
    if torch.cuda.is_available():
        torch.cuda.set_device(local % max(1, ndev))
    return rank, world, local
