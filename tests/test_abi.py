"""The C-ABI library loads, exports every entry point include/dmt.h declares, and fails loudly
(no CPU fallback) when no GPU is present.  CPU only: no compute call needs a device here."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "diffusionmcmctools.jl_amd", "libdmt.so")
HDR = os.path.join(ROOT, "include", "dmt.h")


def declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:dmt_status|const char\*)\s+(dmt_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = declared()
    for want in ("dmt_create", "dmt_draw_proposal", "dmt_accept_reject", "dmt_fetch_ll",
                 "dmt_loglikhd", "dmt_recompute_path", "dmt_swap", "dmt_comm_init"):
        assert want in names


def test_library_exports_every_declared_symbol(dmt):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if " T " in line)
    missing = [n for n in declared() if n not in exported]
    assert not missing, f"declared in dmt.h but not exported: {missing}"
    from diffusionmcmctools_amd import _lib
    assert sorted(_lib.SYMBOLS) == declared()


def test_library_is_gfx950_code_object():
    # the embedded offload bundle names its target triple
    assert b"amdgcn-amd-amdhsa--gfx950" in open(LIB, "rb").read()


def test_version_and_no_cpu_fallback(dmt):
    assert "gfx950" in dmt.version()
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is present")
    with pytest.raises(dmt.DMTError) as ei:
        dmt.Ensemble(0, 1, 1, [[11]])
    assert ei.value.code == 2 and "no CPU fallback" in str(ei.value)


def test_host_only_entry_points_work_without_gpu(dmt):
    H, F, c = dmt.guiding_linear([[-1.0]], [0.0], [1.0], np.linspace(0, 1, 11), [100.0], [30.0], 0.0)
    assert H.shape == (11, 1) and np.all(np.isfinite(H)) and H[0, 0] < H[-1, 0]
    with pytest.raises(dmt.DMTError):
        dmt.guiding_linear([[-1.0]], [0.0], [1.0], np.array([0.0, 0.0]), [1.0], [1.0], 0.0)
