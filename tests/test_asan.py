"""AddressSanitizer / UBSan runs of the CPU-side code:
the CPU restatement (oracle/dmt_oracle.c, fp64 + fp32) and libdmt's host code
(dmt_runtime.hip, the host instantiation of dmt_filter.h) under -fsanitize=address,undefined,
each driven over the edge sizes of the parity tests (tests/asan/*).  GPU code is not
sanitized (no GPU sanitizer on this pool).  CPU only; the libdmt host build takes ≈2 min."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _build(args, timeout):
    r = subprocess.run(["make", "-s"] + args, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]


def _run(exe):
    r = subprocess.run([exe], cwd=ROOT, capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    return r.stdout


def test_oracle_under_asan_ubsan():
    _build(["-C", "oracle", "asan"], 600)
    assert "OK" in _run(os.path.join(ROOT, "oracle", "_asan", "asan_oracle"))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc absent")
def test_libdmt_host_code_under_asan_ubsan():
    _build(["-C", "diffusionmcmctools.jl_amd/csrc", "asan"], 1200)
    assert "OK" in _run(os.path.join(ROOT, "build_asan", "asan_host"))
