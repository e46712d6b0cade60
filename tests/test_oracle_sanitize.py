"""The CPU oracle (host C code) under AddressSanitizer + UndefinedBehaviorSanitizer: a small
driver (oracle/sanitize/sanitize_main.c) runs FK, backbone shape, Jacobian and env steps over
sampled and edge joints; any sanitizer report fails the test."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_clean_under_asan_ubsan(tmp_path):
    exe = tmp_path / "sanitize"
    src = [os.path.join(ROOT, "oracle", "sanitize", "sanitize_main.c"), os.path.join(ROOT, "oracle", "ctr_oracle.c")]
    subprocess.check_call(["gcc", "-O1", "-g", "-std=c11", "-D_GNU_SOURCE", "-ffp-contract=off",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                           *src, "-o", str(exe), "-lm"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
