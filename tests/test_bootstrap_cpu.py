"""torch.distributed bootstrap of the solver communicator (channel_gpu_amd/parallel/bootstrap.py):
the control plane defaults to gloo, and every rank receives rank 0's communicator id.  With
CHANNEL_COMM=shm the id names a shared-memory loopback segment (several ranks per GPU, used to
rehearse the torchrun bench path on a one-GPU box).  CPU only: world size 2, 127.0.0.1."""
import os
import socket
import tempfile

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), CHANNEL_COMM="shm")
    import torch.distributed as dist

    from channel_gpu_amd.parallel.bootstrap import init_distributed, nccl_unique_id

    r, w, local = init_distributed()
    assert (r, w, local) == (rank, world, rank)
    assert dist.get_backend() == "gloo"
    uid = nccl_unique_id()
    with open(os.path.join(outdir, f"uid{rank}"), "wb") as f:
        f.write(uid)
    dist.barrier()
    dist.destroy_process_group()


def test_shm_uid_shared_over_gloo():
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        ids = [open(os.path.join(d, f"uid{r}"), "rb").read() for r in range(2)]
    assert ids[0] == ids[1] and ids[0].startswith(b"shm:channel_")
