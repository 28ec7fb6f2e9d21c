"""The distributed pipeline on a real RCCL communicator, on a one-GPU box.

A 1-rank RCCL communicator (ncclCommInitRank with nranks = 1, built when the solver is given a
unique id at P = 1) runs the P > 1 slab code path: the y-chunked batched exchanges
(RcclComm::alltoallv_batch), the x transforms gathering from exchange blocks, the CFL
allreduce (allreduce_max_f32), the statistics allreduce (allreduce_sum_f64), the health
allreduce (allreduce_max_u32) and the watchdog's ncclCommGetAsyncError polling — captured into
the step hipGraph.  Every result must be bitwise the single-rank fast path (same arithmetic, only
the data movement differs).  CHANNEL_A2A_SELF=rccl routes the self block through ncclSend/Recv
instead of a D2D copy, so RCCL's point-to-point path itself is exercised (and captured) — in a
torch-free process on ROCm's RCCL, the stack bench.py and the drivers run on.
"""
import numpy as np
import pytest

from channel_gpu_amd.utils.config import default_config

pytestmark = pytest.mark.gpu

KW = dict(NX=64, NY=65, NZ=33, Re=1000.0, precision="fp64", ic="random", ic_amplitude=0.2, stats_every=0,
          log_every=0, symmetry_every=0)


def _run(native, uid, nsteps=3, graph=True, stats=False, **kw):
    cfg = default_config(**{**KW, **kw})
    s = native.Solver(cfg, 0, 1, 0, uid)
    s.set_use_graph(graph)
    s.init_ic()
    s.prepare()
    for i in range(nsteps):
        s.step(stats and i == nsteps - 1)
    st = s.stats() if stats else None
    phi, om, U = s.get_state()
    L = s.log()
    return s, phi, om, U, L, st


def _same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a[1:4], b[1:4])) and a[4].dt == b[4].dt


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_rccl_1rank_equals_fast_path(native, precision):
    ref = _run(native, b"", precision=precision)
    got = _run(native, native.new_unique_id(), precision=precision)
    assert got[0].comm_kind() == "rccl" and ref[0].comm_kind() == "none"
    assert _same(ref, got)
    assert got[4].health == 0 and np.isfinite(got[1]).all()


def test_rccl_graph_capture(native):
    """RCCL exchanges inside the captured step graph: the graph is really used and bitwise eager."""
    uid_a, uid_b = native.new_unique_id(), native.new_unique_id()
    g = _run(native, uid_a, nsteps=4, graph=True)
    e = _run(native, uid_b, nsteps=4, graph=False)
    assert g[0].graph_active() and not e[0].graph_active()
    assert _same(g, e)


@pytest.mark.parametrize("chunk,self_mode", [("1", "direct"), ("4", "direct"), ("7", "direct"), ("0", "direct"),
                                             ("4", "copy"), ("0", "copy")])
def test_rccl_ychunks(native, monkeypatch, chunk, self_mode):
    """Chunked exchanges (ragged last chunk) are bitwise the whole-slab exchange and the fast path,
    with the own block accessed in place (direct) or copied inside the exchange (copy)."""
    ref = _run(native, b"")
    monkeypatch.setenv("CHANNEL_YCHUNK", chunk)
    monkeypatch.setenv("CHANNEL_A2A_SELF", self_mode)
    got = _run(native, native.new_unique_id())
    assert _same(ref, got)


SELF_P2P_SCRIPT = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.environ["CHANNEL_ROOT"])
from channel_gpu_amd import require_core
from channel_gpu_amd.utils.config import default_config
C = require_core()
kw = dict(NX=64, NY=65, NZ=33, Re=1000.0, precision="fp64", ic="random", ic_amplitude=0.2, stats_every=0,
          log_every=0, symmetry_every=0)
out = []
for uid in (b"", C.new_unique_id()):
    s = C.Solver(default_config(**kw), 0, 1, 0, uid)
    s.init_ic(); s.prepare()
    for _ in range(4):
        s.step(False)
    out.append((s.get_state(), s.graph_active(), s.comm_kind()))
(a, ga, ka), (b, gb, kb) = out
assert ka == "none" and kb == "rccl" and gb, (ka, kb, gb)
assert all(np.array_equal(x, y) for x, y in zip(a, b))
print("SELF_P2P_OK", flush=True)
"""


def test_rccl_self_block_through_p2p(native):
    """CHANNEL_A2A_SELF=rccl: the self block goes through grouped ncclSend/ncclRecv, captured in the
    step graph, bitwise the fast path.  Runs in a torch-free process (ROCm's RCCL, like bench.py and
    the drivers): torch's bundled RCCL 2.26 crashes capturing a 1-rank self send/recv."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CHANNEL_TORCH_FREE="1", CHANNEL_A2A_SELF="rccl", CHANNEL_YCHUNK="9", CHANNEL_ROOT=root)
    r = subprocess.run([sys.executable, "-c", SELF_P2P_SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "SELF_P2P_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])


def test_rccl_statistics_and_health(native):
    """Statistics step: plane sums go through the RCCL sum allreduce, health through the max."""
    ref = _run(native, b"", stats=True)
    got = _run(native, native.new_unique_id(), stats=True)
    # per-line contributions are accumulated with device atomics (order-dependent rounding): compare
    # against the scale of each statistic, not element by element (the Reynolds-stress row crosses 0)
    N = len(got[5]) // 4
    for q in range(4):
        g, r = got[5][q * N:(q + 1) * N], ref[5][q * N:(q + 1) * N]
        assert np.abs(g - r).max() <= 1e-13 * np.abs(r).max(), q
    assert np.abs(got[5]).max() > 0
    assert got[0].health() == 0
    got[0].barrier()


def test_rccl_phase_timing(native):
    """Per-phase events on both streams of the distributed pipeline (bench.py's exchange timing)."""
    cfg = default_config(**KW)
    s = native.Solver(cfg, 0, 1, 0, native.new_unique_id())
    s.init_ic()
    s.prepare()
    s.step(False)
    s.set_phase_timing(True)
    for _ in range(2):
        s.step(False)
    s.set_phase_timing(False)
    ph = s.phase_times_ms()
    assert ph[0] > 0 and ph[1] > 0 and ph[2] > 0 and ph[3] > 0 and ph[4] > 0
    s.set_step_timing(True)
    for _ in range(3):
        s.step(False)
    t = s.step_times_ms()
    assert len(t) == 3 and all(x > 0 for x in t)


@pytest.mark.parametrize("kblocks,self_mode,fsplit", [("1", "direct", "1"), ("2", "direct", "1"), ("3", "direct", "1"),
                                                      ("8", "direct", "1"), ("16", "direct", "1"), ("4", "copy", "1"),
                                                      ("4", "direct", "0")])
def test_rccl_kspec_blocks_overlap(native, monkeypatch, kblocks, self_mode, fsplit):
    """K-SPEC / exchange overlap: the spectral fields stored as kx
    sub-blocks, K-SPEC run block by block and each block's backward exchange issued behind it on
    the comm stream; the last chunk's forward exchange returns block by block and K-SPEC block b
    waits only for its own rows (fsplit = 1); 16 sub-blocks fill the 16 exchange segments of the
    x transforms.  State, statistics, the kz = 0 symmetrisation and the spectra equal the fast path
    bitwise (the arithmetic per line and per tile is unchanged), eager and captured."""
    monkeypatch.setenv("CHANNEL_A2A_SELF", self_mode)
    monkeypatch.setenv("CHANNEL_FWD_SPLIT", fsplit)
    monkeypatch.setenv("CHANNEL_YCHUNK", "7")
    res = []
    for uid, kb in ((b"", None), (native.new_unique_id(), kblocks)):
        if kb is not None:
            monkeypatch.setenv("CHANNEL_KBLOCKS", kb)
        cfg = default_config(**{**KW, "stats_every": 1, "spectra_planes": "0,10,32"})
        s = native.Solver(cfg, 0, 1, 0, uid)
        if kb is not None:
            assert s.kblocks() == int(kb)
        s.init_ic()
        s.prepare()
        for i in range(4):
            s.step(True)
        s.symmetrize()
        s.prepare()
        s.step(True)
        sp = s.spectra()
        res.append((s.get_state(), np.asarray(s.stats()), sp))
        del s
    (a, sa, pa), (b, sb, pb) = res
    for f in range(3):
        assert np.array_equal(a[f], b[f]), f"field {f}"
    assert np.allclose(sa, sb, rtol=1e-12, atol=0)
    for k in ("ekx", "ekz", "map"):
        assert np.allclose(pa[k], pb[k], rtol=1e-12, atol=0), k


def test_rccl_kspec_exchange_overlap_measured(native, monkeypatch):
    """Per-phase events on a common clock: with kx sub-blocks the backward exchange of block b
    (comm stream) runs while K-SPEC solves block b+1 (compute stream); slot 7 of the phase times is
    the measured intersection of the two.  The self block goes through the exchange (copy) so the
    exchange intervals have a duration on one rank."""
    monkeypatch.setenv("CHANNEL_A2A_SELF", "copy")
    monkeypatch.setenv("CHANNEL_KBLOCKS", "4")
    cfg = default_config(**{**KW, "NX": 128, "NY": 129, "NZ": 65, "precision": "fp32"})
    s = native.Solver(cfg, 0, 1, 0, native.new_unique_id())
    assert s.kblocks() == 4
    s.init_ic()
    s.prepare()
    s.step(False)
    s.reset_phase_times()
    s.set_phase_timing(True)
    for _ in range(2):
        s.step(False)
    s.set_phase_timing(False)
    ph = s.phase_times_ms()
    print("phase ms:", [round(x, 4) for x in ph])
    assert ph[0] > 0 and ph[4] > 0
    assert ph[7] > 0.0, "no K-SPEC / exchange overlap measured"


def test_capture_failure_agreement_falls_back_eagerly(native, monkeypatch, capfd):
    """A capture that fails on a rank (injected after the first substep has been recorded,
    CHANNEL_TEST_CAPTURE_FAIL=<rank>) goes through the cross-rank capture agreement: the failed
    capture is ended on every forked stream, the agreement allreduce runs on the communicator, and
    the rank steps eagerly -- bitwise the captured run.  CHANNEL_MARKERS=1 prints the per-rank
    progress lines bench.py enables at P > 1."""
    monkeypatch.setenv("CHANNEL_MARKERS", "1")
    ref = _run(native, native.new_unique_id(), nsteps=4, graph=True)
    err = capfd.readouterr().err
    assert ref[0].graph_active()
    for m in ("eager warm-up step done", "step graph captured", "first replay of the step graph done"):
        assert m in err, (m, err[-2000:])
    monkeypatch.setenv("CHANNEL_TEST_CAPTURE_FAIL", "0")
    got = _run(native, native.new_unique_id(), nsteps=4, graph=True)
    err = capfd.readouterr().err
    assert not got[0].graph_active()
    assert "capture failure injected" in err and "step graph not captured" in err, err[-2000:]
    assert _same(ref, got)
    got[0].barrier()


def test_capture_failure_keeps_presend_state(native, monkeypatch):
    """With kx sub-blocks (CHANNEL_KBLOCKS=4) every step ends by pre-sending blocks 0 .. NB-2 of the
    next substep 0, and substep 0 then exchanges only block NB-1.  A capture that fails part-way
    records some of that bookkeeping without running it; the abandoned graph must leave it as it
    was, so the eager steps that follow exchange exactly the blocks an eager-from-the-start run
    does (on a multi-rank job a mismatch would pair different exchange sizes between ranks).  The
    host count of issued backward block exchanges is compared, and the states bitwise."""
    monkeypatch.setenv("CHANNEL_KBLOCKS", "4")
    ref = _run(native, native.new_unique_id(), nsteps=4, graph=False)
    assert ref[0].kblocks() == 4
    n_ref = ref[0].bwd_blocks_issued()
    monkeypatch.setenv("CHANNEL_TEST_CAPTURE_FAIL", "0")
    got = _run(native, native.new_unique_id(), nsteps=4, graph=True)
    assert not got[0].graph_active()
    assert got[0].bwd_blocks_issued() == n_ref, (got[0].bwd_blocks_issued(), n_ref)
    assert _same(ref, got)


def test_rccl_two_compute_streams_bitwise(native, monkeypatch):
    """CHANNEL_PSTREAMS=2: the y chunks of the P > 1 pipeline alternate between two compute streams
    (each chunk waits for its own backward exchange; the forward exchange of chunk k waits for the
    stream that ran it).  Eager steps (inside a capture the second stream is used only on HIP
    runtimes >= 7.2, i.e. not in a torch process: see transforms_slab) are bitwise the fast path."""
    monkeypatch.setenv("CHANNEL_PSTREAMS", "2")
    monkeypatch.setenv("CHANNEL_YCHUNK", "16")
    ref = _run(native, b"")
    got = _run(native, native.new_unique_id(), graph=False)
    assert _same(ref, got)
    got2 = _run(native, native.new_unique_id(), graph=True)
    assert _same(ref, got2)


PSTREAMS_SCRIPT = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.environ["CHANNEL_ROOT"])
from channel_gpu_amd import require_core
from channel_gpu_amd.utils.config import default_config
C = require_core()
kw = dict(NX=64, NY=65, NZ=33, Re=1000.0, precision="fp64", ic="random", ic_amplitude=0.2, stats_every=0,
          log_every=0, symmetry_every=0)
kw.update(json.loads(os.environ.get("PSTREAMS_KW", "{}")))
out = []
for uid in (b"", C.new_unique_id()):
    s = C.Solver(default_config(**kw), 0, 1, 0, uid)
    s.init_ic(); s.prepare()
    for _ in range(4):
        s.step(False)
    out.append((s.get_state(), s.graph_active(), s.comm_kind()))
(a, ga, ka), (b, gb, kb) = out
assert ka == "none" and kb == "rccl" and gb, (ka, kb, gb)
assert all(np.array_equal(x, y) for x, y in zip(a, b))
print("PSTREAMS_OK", flush=True)
"""


@pytest.mark.parametrize("layout", ["plain", "blocked"])
def test_rccl_two_compute_streams_captured_torch_free(native, layout):
    """CHANNEL_PSTREAMS=2 inside the captured step graph, in a torch-free process (ROCm 7.2's
    runtime and RCCL, like bench.py and the drivers), bitwise the fast path.  Each exchange chunk's
    transforms run as two parts, one per compute stream (XArgs::seg_yoff): plain [y][line] layout
    with 16-plane chunks, and the blocked layout's plane tiles (NX = 512 fp32, 8-plane chunks split
    4 + 4 inside the 8-plane tiles)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CHANNEL_TORCH_FREE="1", CHANNEL_PSTREAMS="2", CHANNEL_YCHUNK="16", CHANNEL_ROOT=root)
    if layout == "blocked":
        env.update(CHANNEL_SPEC_KZB="1", CHANNEL_YCHUNK="8", CHANNEL_COMBINE="1",
                   PSTREAMS_KW=json.dumps(dict(NX=512, NY=65, NZ=129, precision="fp32", Re=2000.0)))
    r = subprocess.run([sys.executable, "-c", PSTREAMS_SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "PSTREAMS_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])


@pytest.mark.parametrize("kblocks,chunk,precision,combine", [("1", "8", "fp64", "0"), ("4", "16", "fp64", "0"),
                                                             ("16", "8", "fp64", "1"), ("4", "0", "fp32", "0"),
                                                             ("4", "16", "fp32", "1")])
def test_rccl_blocked_layout_equals_fast_path(native, monkeypatch, kblocks, chunk, precision, combine):
    """The blocked spectral layout ([y/8][line/8][y%8][line%8], the default at R = 7, 8) on the P > 1
    pipeline (CHANNEL_SPEC_KZB=1 on both sides): kx sub-blocks each blocked, exchange chunks of whole
    8-plane tiles, the x kernels addressing blocked exchange segments and self blocks (segblk).
    State and the kz = 0 symmetrisation equal the one-rank fast path on the same layout bitwise, the
    statistics and spectra to summation order."""
    monkeypatch.setenv("CHANNEL_SPEC_KZB", "1")
    monkeypatch.setenv("CHANNEL_YCHUNK", chunk)
    monkeypatch.setenv("CHANNEL_COMBINE", combine)  # (combine = 1: the P > 1 default, on both sides)
    res = []
    for uid, kb in ((b"", None), (native.new_unique_id(), kblocks)):
        if kb is not None:
            monkeypatch.setenv("CHANNEL_KBLOCKS", kb)
        cfg = default_config(**{**KW, "precision": precision, "stats_every": 1, "spectra_planes": "0,10,32"})
        s = native.Solver(cfg, 0, 1, 0, uid)
        assert s.spec_kzb() == 8
        if kb is not None:
            assert s.kblocks() == int(kb)
        s.init_ic()
        s.prepare()
        for i in range(3):
            s.step(True)
        s.symmetrize()
        s.prepare()
        s.step(True)
        sp = s.spectra()
        res.append((s.get_state(), np.asarray(s.stats()), sp))
        del s
    (a, sa, pa), (b, sb, pb) = res
    for f in range(3):
        assert np.array_equal(a[f], b[f]), f"field {f}"
    assert np.allclose(sa, sb, rtol=1e-12, atol=0)  # (atomic plane sums: summation order)
    for k in ("ekx", "ekz", "map"):
        assert np.allclose(pa[k], pb[k], rtol=1e-12, atol=0), k


@pytest.mark.parametrize("combine", ["0", "1"])
def test_rccl_blocked_plane_tiles_equal_fast_path(native, monkeypatch, combine):
    """The x kernels of the P > 1 pipeline on the blocked layout as plane tiles (two planes x one
    8-wide kz block per 128-B line, the one-rank fast path's tiles; WIDE = 1 at NX = 512 / 1024 fp32)
    with each row's exchange segment or own block from the per-thread row table: bitwise the
    one-rank fast path, and the launched variants are the plane-tile row-table ones."""
    monkeypatch.setenv("CHANNEL_SPEC_KZB", "1")
    monkeypatch.setenv("CHANNEL_YCHUNK", "8")
    monkeypatch.setenv("CHANNEL_COMBINE", combine)
    res = []
    for uid, kb in ((b"", None), (native.new_unique_id(), "4")):
        if kb is not None:
            monkeypatch.setenv("CHANNEL_KBLOCKS", kb)
        cfg = default_config(**{**KW, "NX": 512, "NY": 65, "NZ": 129, "precision": "fp32", "Re": 2000.0})
        s = native.Solver(cfg, 0, 1, 0, uid)
        assert s.spec_kzb() == 8
        s.init_ic()
        s.prepare()
        for _ in range(3):
            s.step(False)
        res.append(s.get_state())
        if kb is not None:
            assert s.comm_kind() == "rccl"
            assert native.xfft_last_variant() == "xfft_forward_kernel<512, float, false, 1, 3, 2, 2>", native.xfft_last_variant()
            bw = native.xfft_last_backward_variant()
            assert bw == f"xfft_backward_kernel<512, float, false, 1, 3, 2, 2, {'true' if combine == '1' else 'false'}>", bw
        del s
    a, b = res
    for f in range(3):
        assert np.array_equal(a[f], b[f]), f"field {f}"
