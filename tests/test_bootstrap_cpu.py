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


_TCP_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.environ["CHANNEL_ROOT"])
from channel_gpu_amd import require_core
C = require_core()
pi = C.ProcInfo.from_env()
out = C.tcp_broadcast(pi, b"payload-from-0" if pi.rank == 0 else b"", int(os.environ.get("TMO", "30")))
print("GOT", out.decode(), flush=True)
"""


def _tcp_env(rank, world, port):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(port), CHANNEL_ROOT=root, CHANNEL_TORCH_FREE="1")


def test_native_tcp_broadcast_three_ranks():
    """The torch-free rendezvous of bench.py / the drivers: rank 0's payload reaches every rank."""
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, "-c", _TCP_SCRIPT], env=_tcp_env(r, 3, port), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(3)]
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert all("GOT payload-from-0" in o for o, _ in outs)


def test_native_tcp_broadcast_missing_peer_times_out():
    """Rank 0 waits a bounded time for its peers (a dead peer is an error, not a hang)."""
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(_tcp_env(0, 3, port), TMO="2")
    r = subprocess.run([sys.executable, "-c", _TCP_SCRIPT], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "peers connected" in r.stderr


def test_rank_imports_stay_torch_free():
    """bench.py's and the drivers' rank-side imports must not import torch: torch's bundled HIP
    runtime and RCCL share /opt/rocm's sonames, and a torch import ahead of the native core binds the
    solver to them (round 6: channel_gpu_amd.parallel imported its torch.distributed helpers eagerly,
    so bench.py ran on torch's HIP 7.0 runtime, where captured steps keep one compute stream)."""
    import subprocess
    import sys

    code = (
        "import os, sys\n"
        "os.environ['CHANNEL_TORCH_FREE'] = '1'\n"
        "from channel_gpu_amd import require_core\n"
        "from channel_gpu_amd.parallel.decomposition import PencilDecomposition, SlabDecomposition\n"
        "from channel_gpu_amd.parallel.native_bootstrap import init_native\n"
        "from channel_gpu_amd.utils.config import default_config\n"
        "import channel_gpu_amd.driver\n"
        "assert 'torch' not in sys.modules, sorted(m for m in sys.modules if m.startswith('torch'))[:5]\n"
        "from channel_gpu_amd.parallel import dist_info  # the lazy torch.distributed helpers still resolve\n"
        "print('TORCH_FREE_OK')\n"
    )
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    assert r.returncode == 0 and "TORCH_FREE_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
