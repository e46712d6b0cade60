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
                   '  for (long i = 0; i < n; ++i) ctr_math::sincos_cw(x[i], s + i, c + i); }\n')
    so = tmp_path / "m.so"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC",
                           "-I", os.path.join(ROOT, "gym-ctr-reach_amd", "csrc"), str(src), "-o", str(so)])
    lib = ctypes.CDLL(str(so))
    lib.vsincos.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_long]
    return lib


def _ulp_err(got, want):
    return np.abs(got - want) / np.spacing(np.maximum(np.abs(want), 1e-300))


def test_sincos_cw_accuracy(tmp_path):
    lib = _lib(tmp_path)
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-np.pi, np.pi, 200000), rng.uniform(-300, 300, 200000),
                        rng.uniform(-1e5, 1e5, 50000), np.array([0.0, -0.0, 1e-300, np.pi / 2, -np.pi, 1e6, 3e7]),
                        np.arange(-40, 41) * (np.pi / 2), np.arange(-40, 41) * (np.pi / 2) + 1e-9])
    s = np.empty_like(x)
    c = np.empty_like(x)
    lib.vsincos(x.ctypes.data, s.ctypes.data, c.ctypes.data, len(x))
    # absolute error bound (values near zero crossings) + ulp bound elsewhere
    es = np.abs(s - np.sin(x))
    ec = np.abs(c - np.cos(x))
    assert es.max() < 4e-16 and ec.max() < 4e-16, (es.max(), ec.max())
    big = np.abs(np.sin(x)) > 1e-3
    assert _ulp_err(s[big], np.sin(x[big])).max() <= 2.0
    big = np.abs(np.cos(x)) > 1e-3
    assert _ulp_err(c[big], np.cos(x[big])).max() <= 2.0
