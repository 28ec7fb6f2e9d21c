"""Numerics of every HIP kernel against a NumPy fp64 reference of the same operator."""
import numpy as np
import pytest
import torch

from channel_gpu_amd.reference import oracle as ora

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("NY", [33, 65, 129, 257, 385, 633, 1100])
@pytest.mark.parametrize("dtype", [torch.complex128, torch.complex64])
def test_yline_operators(native, NY, dtype):
    rng = np.random.default_rng(NY)
    L = 37
    ops = ora.build_ops(NY)
    x = rng.standard_normal((NY, L)) + 1j * rng.standard_normal((NY, L))
    k2 = np.concatenate([[0.0], rng.uniform(0, 400.0, L - 1)])
    c = 3e-3
    Y = native.YLineOps(NY)
    xt = torch.tensor(x, dtype=dtype, device=DEV)
    k2t = torch.tensor(k2, dtype=torch.float64, device=DEV)
    tol = 1e-10 if dtype == torch.complex128 else 2e-5
    cases = {
        0: ora.op_d1(ops, x),
        1: ora.op_helm(ops, x, k2),
        2: ora.op_impl(ops, x, k2, c),
        3: ora.op_M(ops, x),
        4: ora.op_K(ops, x),
    }
    for op, ref in cases.items():
        got = Y.apply(op, xt, k2t, c).cpu().numpy()
        e = rel(got, ref)
        # fp32 storage: the input itself is rounded; Helmholtz at k=0 amplifies by cond(D2)
        t = tol * (50 if (op == 1 and dtype == torch.complex64) else 1)
        assert e < t, f"op {op} NY={NY} {dtype}: rel err {e:.3e}"


@pytest.mark.parametrize("NY", [259, 300, 385, 449, 512])
@pytest.mark.parametrize("dtype", [torch.complex128, torch.complex64])
def test_yline_operators_two_wave_lines(native, NY, dtype):
    """The operators on lines over two waves (K-SPEC's geometry for 258 < NY <= 512): each half
    solves locally with one spike right-hand side and the halves meet in the 2 x 2 interface solve;
    stencils exchange one halo row per side.  Same tolerances as the one-wave operators."""
    rng = np.random.default_rng(NY + 7)
    L = 29
    ops = ora.build_ops(NY)
    x = rng.standard_normal((NY, L)) + 1j * rng.standard_normal((NY, L))
    k2 = np.concatenate([[0.0], rng.uniform(0, 400.0, L - 1)])
    c = 3e-3
    Y = native.YLineOps(NY, 2.0, 2)
    xt = torch.tensor(x, dtype=dtype, device=DEV)
    k2t = torch.tensor(k2, dtype=torch.float64, device=DEV)
    tol = 1e-10 if dtype == torch.complex128 else 2e-5
    cases = {0: ora.op_d1(ops, x), 1: ora.op_helm(ops, x, k2), 2: ora.op_impl(ops, x, k2, c), 3: ora.op_M(ops, x),
             4: ora.op_K(ops, x)}
    for op, ref in cases.items():
        got = Y.apply(op, xt, k2t, c).cpu().numpy()
        e = rel(got, ref)
        t = tol * (50 if (op == 1 and dtype == torch.complex64) else 1)
        assert e < t, f"op {op} NY={NY} {dtype}: rel err {e:.3e}"


@pytest.mark.parametrize("NY", [33, 65, 129, 192])
def test_d1_dense_mfma(native, NY):
    """Dense D1 on the matrix cores (v_mfma_f64_16x16x4_f64) against the dense NumPy D1."""
    rng = np.random.default_rng(100 + NY)
    L = 37  # not a multiple of the 8 lines per block
    ops = ora.build_ops(NY)
    x = rng.standard_normal((NY, L)) + 1j * rng.standard_normal((NY, L))
    Y = native.YLineOps(NY)
    got = Y.d1_mfma(torch.tensor(x, dtype=torch.complex128, device=DEV)).cpu().numpy()
    assert rel(got, ora.op_d1(ops, x)) < 1e-10


@pytest.mark.parametrize("n", [16, 32, 64, 128, 256, 512, 1024, 2048,
                               48, 96, 192, 384, 768, 1536, 80, 160, 320, 640, 1280,
                               112, 224, 448, 896, 1792, 144, 288, 576, 1152, 240, 480, 960, 1920,
                               176, 352, 704, 1408, 208, 416, 832, 1664])
@pytest.mark.parametrize("dtype", [torch.complex64, torch.complex128])
def test_fft_c2c(native, n, dtype):
    """Batched C2C against numpy, powers of two and the radix-3/5/7/9/11/13/15 plans (m*2^k)."""
    rng = np.random.default_rng(n)
    x = rng.standard_normal((7, n)) + 1j * rng.standard_normal((7, n))
    xt = torch.tensor(x, dtype=dtype, device=DEV)
    tol = 1e-13 if dtype == torch.complex128 else 2e-6
    inv = native.fft_c2c(xt, 1).cpu().numpy()
    fwd = native.fft_c2c(xt, -1).cpu().numpy()
    assert rel(inv, np.fft.ifft(x, axis=-1) * n) < tol * np.log2(n)
    assert rel(fwd, np.fft.fft(x, axis=-1)) < tol * np.log2(n)


@pytest.mark.parametrize("NX,nkz", [(32, 11), (128, 43), (1024, 20), (2048, 9),
                                    (96, 13), (192, 11), (384, 20), (768, 9), (1536, 5), (80, 7), (1280, 6),
                                    (112, 9), (448, 13), (1792, 5), (144, 7), (1152, 6), (240, 11), (960, 7),
                                    (1920, 5), (176, 9), (1408, 5), (208, 7), (1664, 5)])
@pytest.mark.parametrize("dtype", [torch.complex64, torch.complex128])
def test_xfft(native, NX, nkz, dtype):
    rng = np.random.default_rng(NX)
    Kx = NX // 3
    nkx = 2 * Kx + 1
    F, ny = 3, 5
    s = rng.standard_normal((F, ny, nkx, nkz)) + 1j * rng.standard_normal((F, ny, nkx, nkz))
    st = torch.tensor(s, dtype=dtype, device=DEV)
    phys = native.xfft_backward(st, NX, Kx)
    pos = np.where(np.arange(nkx) <= Kx, np.arange(nkx), NX - (nkx - np.arange(nkx)))
    full = np.zeros((F, ny, NX, nkz), complex)
    full[:, :, pos, :] = s
    ref = np.fft.ifft(full, axis=2) * NX
    tol = 1e-12 if dtype == torch.complex128 else 3e-6
    assert rel(phys.cpu().numpy(), ref) < tol
    back = native.xfft_forward(phys, Kx).cpu().numpy() / NX
    assert rel(back, s) < tol


def _blocked_index(rows, nkx, nkz):
    """Element offsets spec_index(kzb = 8) of (y, ikx, kz) in one blocked field (kernels.hpp):
    [y / 8][line / 8][y % 8][line % 8], line = ikx * nkzs + kz, nkzs = nkz rounded up to 8."""
    nkzs = -(-nkz // 8) * 8
    lines = nkx * nkzs
    y = np.arange(rows)[:, None, None]
    line = np.arange(nkx)[None, :, None] * nkzs + np.arange(nkz)[None, None, :]
    idx = (y // 8) * 8 * lines + (y % 8) * 8 + (line // 8) * 64 + line % 8
    return idx, (-(-rows // 8) * 8) * lines


# The headline grid (1024 x 385 x 1024 fp32, one rank) runs the blocked spectral layout with plane
# tiles and 16-byte accesses: rocprofv3 names xfft_backward_kernel<1024, float, false, 1, 0, 2, 2> and
# xfft_forward_kernel<1024, float, false, 1, 0, 2, 2> (profiles/r04/final2/kernel_stats_1024x385x1024.csv).
# These cases run those instantiations (and the fp64 / odd-nkz / other-length variants of the same
# layout) against NumPy, on a plane range that starts and ends inside 8-plane tiles, with the
# non-temporal accesses on and off, and with field 4's mean line read as zero (omega_y's source).
@pytest.mark.parametrize("NX,nkz,dtype,nt,variant", [
    (1024, 342, torch.complex64, 1, "<1024, float, false, 1, 0, 2, 2>"),
    (1024, 342, torch.complex64, 0, "<1024, float, false, 1, 0, 2, 2>"),
    (1024, 341, torch.complex64, 1, "<1024, float, false, 1, 0, 1, 2>"),
    (1024, 342, torch.complex128, 1, "<1024, double, false, 0, 0, 1, 1>"),
    (512, 86, torch.complex64, 0, "<512, float, false, 1, 0, 2, 2>"),
    (2048, 20, torch.complex64, 1, "<2048, float, false, 0, 0, 2, 1>"),
    (768, 50, torch.complex64, 0, "<768, float, false, 0, 0, 2, 1>"),
])
def test_xfft_blocked_layout(native, NX, nkz, dtype, nt, variant):
    rng = np.random.default_rng(NX + nkz)
    Kx = NX // 3
    nkx = 2 * Kx + 1
    rows, y0, ny = 13, 3, 6
    F = 6
    s = rng.standard_normal((F, rows, nkx, nkz)) + 1j * rng.standard_normal((F, rows, nkx, nkz))
    idx, fstride = _blocked_index(rows, nkx, nkz)
    buf = np.zeros(F * fstride, complex)
    for f in range(F):
        buf[f * fstride + idx] = s[f]
    bt = torch.tensor(buf, dtype=dtype, device=DEV)
    phys = native.xfft_backward_blocked(bt, F, rows, y0, ny, NX, Kx, nkz, nt, 4)
    bvariant = variant[:-1] + ", false>"  # (the backward's combine argument)
    assert native.xfft_last_variant() == "xfft_backward_kernel" + bvariant, native.xfft_last_variant()
    pos = np.where(np.arange(nkx) <= Kx, np.arange(nkx), NX - (nkx - np.arange(nkx)))
    full = np.zeros((F, ny, NX, nkz), complex)
    full[:, :, pos, :] = s[:, y0:y0 + ny]
    full[4, :, 0, 0] = 0.0  # zero_mean_field = 4: (kx 0, kz 0) reads as zero
    ref = np.fft.ifft(full, axis=2) * NX
    tol = 1e-12 if dtype == torch.complex128 else 3e-6
    assert rel(phys.cpu().numpy(), ref) < tol
    # forward into fields pre-filled with a sentinel: only planes y0 .. y0 + ny - 1 change
    sent = torch.full((3 * fstride,), 7.0 + 7.0j, dtype=dtype, device=DEV)
    out = native.xfft_forward_blocked(phys[:3].contiguous(), sent, rows, y0, Kx, nt)
    assert native.xfft_last_variant() == "xfft_forward_kernel" + variant, native.xfft_last_variant()
    got = out.cpu().numpy()
    for f in range(3):
        g = got[f * fstride + idx]
        assert rel(g[y0:y0 + ny] / NX, s[f, y0:y0 + ny]) < tol, f
        assert np.all(g[:y0] == 7.0 + 7.0j) and np.all(g[y0 + ny:] == 7.0 + 7.0j), f


def _combine_ref(s, NX, Kx, ax, az, kz0):
    """The six physical-stage fields u, v, w, omega_x, omega_y, omega_z from the five K-SPEC outputs
    (D1 v, v, D1 omega, omega, phi) [5, ny, nkx, nkz], x-backward transformed (fft_impl.hpp cmb_pair)."""
    nkx, nkz = s.shape[2], s.shape[3]
    kxs = np.where(np.arange(nkx) <= Kx, np.arange(nkx), np.arange(nkx) - nkx)
    al = (ax * kxs)[None, :, None]
    be = (az * (kz0 + np.arange(nkz)))[None, None, :]
    k2 = al * al + be * be
    r = np.where(k2 > 0, 1.0 / np.where(k2 > 0, k2, 1.0), 0.0)
    dv, v, dom, om, phi = s
    mean = (k2 == 0).astype(float)
    u = 1j * (al * dv - be * om) * r + mean * om.real
    w = 1j * (be * dv + al * om) * r
    wx = 1j * (be * phi + al * dom) * r
    wz = 1j * (be * dom - al * phi) * r - mean * dom.real
    wy = om * (1.0 - mean)
    six = np.stack([u, v, w, wx, wy, wz])
    pos = np.where(np.arange(nkx) <= Kx, np.arange(nkx), NX - (nkx - np.arange(nkx)))
    full = np.zeros((6, s.shape[1], NX, nkz), complex)
    full[:, :, pos, :] = six
    return np.fft.ifft(full, axis=2) * NX


# Combine mode (the solver's x-backward): K-SPEC stores D1 v, v, D1 omega next to the omega and phi
# states, and the gather forms u, v, w, omega_x, omega_y, omega_z per element.  The blocked cases
# run the headline instantiation (1024-point fp32 plane tiles, 16-byte accesses) and the fp64 /
# odd-nkz / other-length variants; the plain cases the [y][kx][kz] layout of P > 1 (kz0 > 0: a
# pencil row's kz range).
@pytest.mark.parametrize("NX,nkz,dtype,nt,variant", [
    (1024, 342, torch.complex64, 1, "<1024, float, false, 1, 0, 2, 2, true>"),
    (1024, 341, torch.complex64, 0, "<1024, float, false, 1, 0, 1, 2, true>"),
    (1024, 342, torch.complex128, 1, "<1024, double, false, 0, 0, 1, 1, true>"),
    (512, 86, torch.complex64, 0, "<512, float, false, 1, 0, 2, 2, true>"),
    (2048, 20, torch.complex64, 1, "<2048, float, false, 0, 0, 2, 1, true>"),
    (768, 50, torch.complex128, 0, "<768, double, false, 0, 0, 1, 1, true>"),
])
def test_xfft_combine_blocked(native, NX, nkz, dtype, nt, variant):
    rng = np.random.default_rng(NX + nkz + 1)
    Kx = NX // 3
    nkx = 2 * Kx + 1
    rows, y0, ny = 13, 3, 6
    ax, az = 0.5, 2.0
    s = rng.standard_normal((5, rows, nkx, nkz)) + 1j * rng.standard_normal((5, rows, nkx, nkz))
    idx, fstride = _blocked_index(rows, nkx, nkz)
    buf = np.zeros(5 * fstride, complex)
    for f in range(5):
        buf[f * fstride + idx] = s[f]
    bt = torch.tensor(buf, dtype=dtype, device=DEV)
    phys = native.xfft_backward_blocked(bt, 5, rows, y0, ny, NX, Kx, nkz, nt, -1, combine=1, ax=ax, az=az)
    assert native.xfft_last_variant() == "xfft_backward_kernel" + variant, native.xfft_last_variant()
    ref = _combine_ref(s[:, y0:y0 + ny], NX, Kx, ax, az, 0)
    tol = 1e-12 if dtype == torch.complex128 else 3e-6
    assert rel(phys.cpu().numpy(), ref) < tol


@pytest.mark.parametrize("NX,nkz,kz0,dtype", [(1024, 20, 0, torch.complex64), (1024, 21, 5, torch.complex64),
                                              (128, 43, 0, torch.complex128), (96, 13, 3, torch.complex64),
                                              (2048, 9, 0, torch.complex128), (384, 20, 0, torch.complex64)])
def test_xfft_combine(native, NX, nkz, kz0, dtype):
    rng = np.random.default_rng(NX + kz0)
    Kx = NX // 3
    nkx = 2 * Kx + 1
    ny = 5
    ax, az = 1.0, 2.0
    s = rng.standard_normal((5, ny, nkx, nkz)) + 1j * rng.standard_normal((5, ny, nkx, nkz))
    st = torch.tensor(s, dtype=dtype, device=DEV)
    phys = native.xfft_backward(st, NX, Kx, combine=1, ax=ax, az=az, kz0=kz0)
    assert native.xfft_last_variant().endswith(", true>"), native.xfft_last_variant()
    ref = _combine_ref(s, NX, Kx, ax, az, kz0)
    tol = 1e-12 if dtype == torch.complex128 else 3e-6
    assert rel(phys.cpu().numpy(), ref) < tol


@pytest.mark.parametrize("NX,Nzp,dtype", [(32, 32, torch.complex128), (64, 128, torch.complex64),
                                          (16, 1024, torch.complex64), (16, 1024, torch.complex128),
                                          (32, 2048, torch.complex64), (8, 2048, torch.complex128),
                                          (16, 512, torch.complex128),
                                          (16, 96, torch.complex64), (8, 192, torch.complex128),
                                          (8, 384, torch.complex64), (4, 768, torch.complex64),
                                          (4, 768, torch.complex128), (2, 1536, torch.complex64),
                                          (4, 1536, torch.complex128), (4, 1280, torch.complex64),
                                          (8, 160, torch.complex128),
                                          (8, 112, torch.complex128), (4, 448, torch.complex64),
                                          (2, 1792, torch.complex64), (2, 1792, torch.complex128),
                                          (8, 144, torch.complex64), (4, 1152, torch.complex128),
                                          (8, 240, torch.complex128), (4, 960, torch.complex64),
                                          (2, 1920, torch.complex64), (2, 1920, torch.complex128),
                                          (8, 176, torch.complex128), (2, 1408, torch.complex64),
                                          (8, 208, torch.complex64), (2, 1664, torch.complex128),
                                          (1024, 1024, torch.complex64), (1024, 1024, torch.complex128),
                                          (512, 2048, torch.complex64)])
def test_zphys(native, NX, Nzp, dtype):
    """z stage vs NumPy (LDS-pass kernel; the register-resident one is covered in a subprocess).
    The 1024- and 2048-point cases have more row groups than the persistent grid holds, so blocks
    walk several groups and the next row's first field pair is prefetched across rows."""
    rng = np.random.default_rng(Nzp)
    nkz = Nzp // 3 + 1
    ny = 3
    f = rng.standard_normal((6, ny, NX, nkz)) + 1j * rng.standard_normal((6, ny, NX, nkz))
    f[..., 0] = f[..., 0].real  # kz=0 coefficient of a real z-row
    ft = torch.tensor(f, dtype=dtype, device=DEV)
    inv_dy = torch.ones(ny, dtype=torch.float64)
    H, maxima = native.zphys(ft, Nzp, inv_dy, 1.0, 1.0)
    phys = np.fft.irfft(np.concatenate([f, np.zeros(f.shape[:-1] + (Nzp // 2 + 1 - nkz,))], -1), n=Nzp,
                        axis=-1, norm="forward")
    u, v, w, wx, wy, wz = phys
    Hp = np.stack([v * wz - w * wy, w * wx - u * wz, u * wy - v * wx])
    Href = np.fft.rfft(Hp, axis=-1, norm="forward")[..., :nkz] / NX
    tol = 1e-12 if dtype == torch.complex128 else 5e-6
    assert rel(H.cpu().numpy(), Href) < tol
    m = maxima.cpu().numpy()
    assert abs(m[0] - np.abs(u).max()) < 1e-4 * np.abs(u).max()
    assert abs(m[1] - np.abs(v).max()) < 1e-4 * np.abs(v).max()
    assert abs(m[3] - (np.abs(u) + np.abs(v) + np.abs(w)).max()) < 1e-4 * m[3]


ZREG_SCRIPT = r"""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.environ["CHANNEL_ROOT"])
from channel_gpu_amd import require_native
C = require_native()
rng = np.random.default_rng(3)
for dtype, tol in ((torch.complex64, 5e-6), (torch.complex128, 1e-12)):
    NX, Nzp, ny = 16, 1024, 3
    nkz = Nzp // 3 + 1
    f = rng.standard_normal((6, ny, NX, nkz)) + 1j * rng.standard_normal((6, ny, NX, nkz))
    f[..., 0] = f[..., 0].real
    H, m = C.zphys(torch.tensor(f, dtype=dtype, device="cuda"), Nzp, torch.ones(ny, dtype=torch.float64), 1.0, 1.0)
    phys = np.fft.irfft(np.concatenate([f, np.zeros(f.shape[:-1] + (Nzp // 2 + 1 - nkz,))], -1), n=Nzp, axis=-1,
                        norm="forward")
    u, v, w, wx, wy, wz = phys
    Hp = np.stack([v * wz - w * wy, w * wx - u * wz, u * wy - v * wx])
    Href = np.fft.rfft(Hp, axis=-1, norm="forward")[..., :nkz] / NX
    e = np.linalg.norm(H.cpu().numpy() - Href) / np.linalg.norm(Href)
    assert e < tol, (dtype, e)
    assert abs(m.cpu().numpy()[0] - np.abs(u).max()) < 1e-4 * np.abs(u).max()
print("ZREG_OK")
"""


def test_zphys_register_kernel():
    """CHANNEL_ZREG=1: register-resident four-step z stage (Nzp = 1024, fp32/fp64) vs NumPy."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CHANNEL_ZREG="1", CHANNEL_ROOT=root)
    r = subprocess.run([sys.executable, "-c", ZREG_SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ZREG_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
