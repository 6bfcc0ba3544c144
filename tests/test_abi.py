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


def test_recent_kernels_names_launches_without_gpu(dmt):
    """dmt_recent_kernels (no device work): empty before any launch on this thread, and the
    bench's family match reads demangled kernel names (bench.dispatched_kernel)."""
    from diffusionmcmctools_amd import _lib
    from conftest import gpu_available
    if not gpu_available():
        assert _lib.recent_kernels() == []
    import sys
    sys.path.insert(0, ROOT)
    import bench
    names = ["void dmt::k_accept_reduce_lb(dmt::AcceptArgs, double*, double*, unsigned int*)",
             "void dmt::k_block_ps_pk<dmt::Lorenz<float>, float, 4, true>(dmt::BlockArgs<float>)"]
    assert bench.dispatched_kernel(names) == "k_block_ps_pk<"
    assert bench.dispatched_kernel(
        ["void dmt::k_block<dmt::FHN<double>, double, 0, false, 4, false>(dmt::BlockArgs<double>)"]
    ) == "k_block<"
    assert bench.dispatched_kernel(["void dmt::k_mcmc_resident_pc<dmt::OU<double, 2, 2>, double, 1,"
                                    " false, 4>(dmt::BlockArgs<double>)"]) == "k_mcmc_resident_pc"
    assert bench.dispatched_kernel(["?"]) is None
