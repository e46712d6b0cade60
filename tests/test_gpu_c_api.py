"""The C ABI used from plain C (examples/fk_c_api.c, built by __graft_entry__.build()): ctr_fk on
hipMalloc'd buffers, no Python or torch in the process.  Bar: tips within 1e-10 m of the oracle."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "fk_c_api")


@pytest.mark.gpu
def test_c_program_fk_matches_oracle(tmp_path, oracle_mod, cuda):
    assert os.path.exists(EXE), "examples/fk_c_api not built (__graft_entry__.build())"
    out = tmp_path / "tips.bin"
    r = subprocess.run([EXE, str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    tips = np.fromfile(str(out), dtype=np.float64).reshape(4, 3)
    q = np.array([[0, 0, 0, 0, 0, 0], [-0.05, -0.04, -0.03, 0.3, -0.2, 1.0],
                  [-0.2, -0.15, -0.1, 2.0, 1.0, -2.5], [-0.3, -0.2, -0.05, -1.0, 3.0, 0.5]], np.float32)
    ref = oracle_mod.fk(q)["tip"]
    assert np.abs(tips - ref).max() < 1e-10


def test_header_is_plain_c(tmp_path):
    """include/ctr_reach_amd.h and the example compile as C11 with gcc (no C++ or HIP types)."""
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "examples", "fk_c_api.c")])
