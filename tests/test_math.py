"""Host check of the kernels' fp64 sincos (gym-ctr-reach_amd/csrc/ctr_math.hpp): the same
source compiled with g++ must stay within 2 ulp of libm over the arguments the RHS sees."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib(tmp_path):
    src = tmp_path / "m.cpp"
    src.write_text('#include "ctr_math.hpp"\n'
                   'extern "C" void vsincos(const double* x, double* s, double* c, long n) {\n'
                   '  for (long i = 0; i < n; ++i) ctr_math::sincos_cw(x[i], s + i, c + i); }\n'
                   'extern "C" void vsincos_tab(const double* x, double* s, double* c, long n) {\n'
                   '  for (long i = 0; i < n; ++i) ctr_math::sincos_tab(x[i], ctr_math::TRIG_TAB, s[i], c[i]); }\n'
                   )
    so = tmp_path / "m.so"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC",
                           "-I", os.path.join(ROOT, "gym-ctr-reach_amd", "csrc"), str(src), "-o", str(so)])
    lib = ctypes.CDLL(str(so))
    lib.vsincos.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_long]
    lib.vsincos_tab.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_long]
    return lib


def _ulp_err(got, want):
    return np.abs(got - want) / np.spacing(np.maximum(np.abs(want), 1e-300))


import pytest


@pytest.mark.parametrize("fn", ["vsincos", "vsincos_tab"])
def test_sincos_accuracy(tmp_path, fn):
    lib = _lib(tmp_path)
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-np.pi, np.pi, 200000), rng.uniform(-300, 300, 200000),
                        rng.uniform(-1e5, 1e5, 50000), np.array([0.0, -0.0, 1e-300, np.pi / 2, -np.pi]),
                        np.arange(-40, 41) * (np.pi / 2), np.arange(-40, 41) * (np.pi / 2) + 1e-9,
                        np.arange(-400, 401) * (np.pi / 32), np.arange(-400, 401) * (np.pi / 32) + 1e-12,
                        np.arange(-1600, 1601) * (np.pi / 256), np.arange(-1600, 1601) * (np.pi / 512)])
    if fn == "vsincos":          # sincos_cw has the exact large-argument path; sincos_tab is |x| < 2^20
        x = np.concatenate([x, [1e6, 3e7]])
    s = np.empty_like(x)
    c = np.empty_like(x)
    getattr(lib, fn)(x.ctypes.data, s.ctypes.data, c.ctypes.data, len(x))
    # absolute error bound (values near zero crossings) + ulp bound elsewhere
    es = np.abs(s - np.sin(x))
    ec = np.abs(c - np.cos(x))
    assert es.max() < 4e-16 and ec.max() < 4e-16, (es.max(), ec.max())
    big = np.abs(np.sin(x)) > 1e-3
    assert _ulp_err(s[big], np.sin(x[big])).max() <= 2.0
    big = np.abs(np.cos(x)) > 1e-3
    assert _ulp_err(c[big], np.cos(x[big])).max() <= 2.0


def _lib2(tmp_path):
    src = tmp_path / "m2.cpp"
    src.write_text('#include "ctr_math.hpp"\n'
                   'extern "C" void vir10(const double* x, double* y, long n) {\n'
                   '  for (long i = 0; i < n; ++i) y[i] = ctr_math::inv_root10(x[i]); }\n'
                   'extern "C" void vsqrt(const double* x, double* y, long n) {\n'
                   '  for (long i = 0; i < n; ++i) y[i] = ctr_math::sqrt_rsq(x[i]); }\n')
    so = tmp_path / "m2.so"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC",
                           "-I", os.path.join(ROOT, "gym-ctr-reach_amd", "csrc"), str(src), "-o", str(so)])
    lib = ctypes.CDLL(str(so))
    lib.vir10.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_long]
    lib.vsqrt.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_long]
    return lib


def test_inv_root10_and_sqrt(tmp_path):
    """x^(-1/10) (RK45 step factor 0.9 en^-0.2 = 0.9 (en^2)^-0.1) within 2 ulp of libm pow over
    the whole positive double range, including subnormals."""
    lib = _lib2(tmp_path)
    rng = np.random.default_rng(1)
    x = np.concatenate([10.0 ** rng.uniform(-300, 300, 200000), rng.uniform(0.5, 2, 100000),
                        np.array([1.0, 2.0, 1024.0, 1e-310, 5e-324, 1.7e308, 18.0, 1e-30])])
    y = np.empty_like(x)
    lib.vir10(x.ctypes.data, y.ctypes.data, len(x))
    # reference: 50-digit decimal arithmetic (libm and numpy pow are themselves ~30 ulp off at the
    # extremes of the range); a subsample keeps the test fast
    from decimal import Decimal, getcontext
    getcontext().prec = 50
    idx = np.concatenate([np.arange(0, len(x), 97), np.arange(len(x) - 8, len(x))])
    want = np.array([float(Decimal(float(v)) ** Decimal("-0.1")) for v in x[idx]])
    assert _ulp_err(y[idx], want).max() <= 2.0, _ulp_err(y[idx], want).max()
    xs = 10.0 ** rng.uniform(-30, 30, 100000)
    s = np.empty_like(xs)
    lib.vsqrt(xs.ctypes.data, s.ctypes.data, len(xs))
    assert _ulp_err(s, np.sqrt(xs)).max() <= 2.0


def test_sampler_round_tables():
    """The wave sampler's per-round constants (ctr_device.hpp SampleTabs): for k = 1..64 unresolved
    lanes, x // k == (x * ceil(2^16 / k)) >> 16 for every 0 <= x <= 128 (the sampler divides
    lane, ctz(hit) - rank <= 63 and 64 - rank + k - 1 <= 127 by k), and stride[k] << rank is the
    set {rank, rank + k, ...} below 64 that the former loop built."""
    for k in range(1, 65):
        m = -(-65536 // k)
        for x in range(129):
            assert (x * m) >> 16 == x // k, (k, x)
        stride = sum(1 << i for i in range(0, 64, k))
        for rank in range(k):
            want = sum(1 << i for i in range(rank, 64, k))
            assert (stride << rank) & ((1 << 64) - 1) == want, (k, rank)


def test_gap_up_matches_nextafter(tmp_path):
    """ctr_math::gap_up(t) == nextafter(t, inf) - t bit for bit (the RK45 min_step, rk.py:114-119):
    normals, subnormals, signed zeros, negative powers of two (where the gap toward zero halves),
    the extremes and non-finite values."""
    src = tmp_path / "m3.cpp"
    src.write_text('#include "ctr_math.hpp"\n'
                   'extern "C" void vgap(const double* x, double* y, long n) {\n'
                   '  for (long i = 0; i < n; ++i) y[i] = ctr_math::gap_up(x[i]); }\n')
    so = tmp_path / "m3.so"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC",
                           "-I", os.path.join(ROOT, "gym-ctr-reach_amd", "csrc"), str(src), "-o", str(so)])
    lib = ctypes.CDLL(str(so))
    lib.vgap.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_long]
    rng = np.random.default_rng(2)
    p2 = np.ldexp(1.0, np.arange(-1074, 1024))
    x = np.concatenate([rng.uniform(-1, 1, 100000), rng.uniform(0, 0.6, 100000),
                        10.0 ** rng.uniform(-320, 308, 100000) * rng.choice([-1.0, 1.0], 100000),
                        p2, -p2, np.nextafter(p2, 0), -np.nextafter(p2, 0), np.nextafter(p2, np.inf),
                        np.array([0.0, -0.0, 5e-324, -5e-324, 1.7976931348623157e308,
                                  -1.7976931348623157e308, np.inf, -np.inf, np.nan])])
    y = np.empty_like(x)
    with np.errstate(invalid="ignore", over="ignore"):
        want = np.nextafter(x, np.inf) - x
    lib.vgap(x.ctypes.data, y.ctypes.data, len(x))
    same = (y.view(np.uint64) == want.view(np.uint64)) | (np.isnan(y) & np.isnan(want))
    assert same.all(), (x[~same][:5], y[~same][:5], want[~same][:5])


def test_inv_root10_exponent_split():
    """inv_root10's branch-free k = floor((e - 1) / 10) over every frexp exponent of a double."""
    for e in range(-1075, 1026):
        em1 = e - 1
        assert ((em1 + 1100) // 10) - 110 == em1 // 10, e


def test_inv_root10_unguarded_tail(tmp_path):
    """The RK45 step factor is 0.9 inv_root10(err^2) without a guard (ctr_device.hpp): for a huge,
    infinite or NaN err^2 it must stay below 0.2 or be NaN, so that a rejection's fmax(0.2, .)
    gives 0.2 as rk.py:171 does for an infinite norm."""
    lib = _lib2(tmp_path)
    x = np.array([1e300, 3e300, 1e305, 1.7976931348623157e308, np.inf, np.nan])
    y = np.empty_like(x)
    lib.vir10(x.ctypes.data, y.ctypes.data, len(x))
    f = 0.9 * y
    assert np.all(np.isnan(f) | (f < 0.2)), f
    assert np.all(np.fmax(0.2, f) == 0.2)
