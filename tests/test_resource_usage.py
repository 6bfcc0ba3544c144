"""Register, spill and LDS use of the shipped persistent kernels, read from
the resource-usage remarks the build keeps beside each kernel object
(``build_obj/dmt_kernels_*.o.ru``: ``-Rpass-analysis=kernel-resource-usage``, csrc/Makefile).

Every instantiation of the persistent kernels — ``k_mcmc_resident_pc`` (the C2 headline and the
MCMC service), ``k_mcmc_resident``, ``k_mcmc_scan`` — must match one row of ``BOUNDS`` and stay
within its stated bounds (DESIGN.md §5 "register budget"): no VGPR spills to scratch memory where
a kernel's iteration loop would reload them, and an SGPR-spill ceiling (SGPR spills go to VGPR
lanes: one ``v_readlane`` per reload, VALU work in VALU-bound kernels).  CPU only: no GPU, the
numbers are the compiler's.
"""
from __future__ import annotations

import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "build_obj")
SRC = os.path.join(ROOT, "diffusionmcmctools.jl_amd", "csrc", "dmt_kernels.hip")

FIELDS = ("TotalSGPRs", "VGPRs", "AGPRs", "ScratchSize", "SGPRs Spill", "VGPRs Spill",
          "LDS Size", "Occupancy")

# (demangled-name regex, bounds): every persistent-kernel instantiation matches exactly one row.
# "VGPRs Spill"/"ScratchSize" 0: no register spilled to memory.  SGPR spill ceilings: the shipped
# counts (round 6) with a small margin — a regression guard, and the record of what the kernels
# spill (to VGPR lanes) today.  k_mcmc_scan<…, TD = true> is the opt-in persistent TD path
# (DMT_MCMC_SCAN_TD=1): its scan body is a call, whose frame is the scratch it reports.
BOUNDS = [
    # the C2 headline: one producer, four blocks per workgroup, two waves per SIMD, no scratch
    (r"k_mcmc_resident_pc<dmt::OU<double, 2, 2>, double, 1, false, 4>",
     {"VGPRs Spill": 0, "ScratchSize": 0, "SGPRs Spill": 160, "Occupancy": (2, 2)}),
    (r"k_mcmc_resident_pc<dmt::OU<double, 2, 1>, double, 1, false, 4>",
     {"VGPRs Spill": 8, "ScratchSize": 32, "SGPRs Spill": 135}),
    # the MCMC service (SVC = true) and the one-block-per-workgroup form (DMT_PC_BPW=1)
    (r"k_mcmc_resident_pc<dmt::OU<double, 2, [12]>, double, 1, (true, 4|false, 1)>",
     {"VGPRs Spill": 4, "ScratchSize": 16, "SGPRs Spill": 180}),
    # two producers (DMT_MCMC_PC=2, measured slower, not the default): three waves per SIMD
    (r"k_mcmc_resident_pc<dmt::OU<double, 2, [12]>, double, 2, (true|false), 4>",
     {"VGPRs Spill": 50, "ScratchSize": 180, "SGPRs Spill": 145}),
    (r"k_mcmc_resident_pc<dmt::OU<double, 1, 1>, double, [12], (true|false), [14]>",
     {"VGPRs Spill": 0, "ScratchSize": 0, "SGPRs Spill": 130}),
    (r"k_mcmc_resident_pc<dmt::OU<float, ",
     {"VGPRs Spill": 8, "ScratchSize": 32, "SGPRs Spill": 110}),
    (r"k_mcmc_resident<dmt::OU<(double|float), [12], [12]>, (double|float)>",
     {"VGPRs Spill": 0, "ScratchSize": 0, "SGPRs Spill": 180}),
    # the general persistent scan: register spills go to AGPRs (no scratch)
    (r"k_mcmc_scan<dmt::OU<(double|float), [123], [123]>, (double|float), false>",
     {"SGPRs Spill": 230, "VGPRs Spill": 70, "ScratchSize": 0}),
    # the opt-in persistent TD scan (DMT_MCMC_SCAN_TD=1): its out-of-line body's call frame
    (r"k_mcmc_scan<dmt::OU<(double|float), [123], [123]>, (double|float), true>",
     {"SGPRs Spill": 50, "VGPRs Spill": 90, "ScratchSize": 2700}),
]
PERSISTENT = re.compile(r"\bdmt::(k_mcmc_resident_pc|k_mcmc_resident|k_mcmc_scan)<")


def _demangle(names):
    cf = shutil.which("c++filt")
    if not cf:
        pytest.skip("no c++filt")
    out = subprocess.run([cf], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.split("\n")
    return dict(zip(names, out))


def load_usage():
    files = sorted(glob.glob(os.path.join(OBJ, "dmt_kernels_*.o.ru")))
    if not files:
        pytest.skip("no resource-usage files: build the library first (make -C "
                    "diffusionmcmctools.jl_amd/csrc, or __graft_entry__.build())")
    if any(os.path.getmtime(f) < os.path.getmtime(SRC) for f in files):
        pytest.skip("resource-usage files older than dmt_kernels.hip: rebuild")
    usage, cur = {}, None
    for f in files:
        for line in open(f, errors="replace"):
            m = re.search(r"remark: Function Name: (\S+)", line)
            if m:
                cur = m.group(1)
                usage[cur] = {}
                continue
            m = re.search(r"remark:\s+(" + "|".join(re.escape(x) for x in FIELDS) +
                          r")(?: \[[^\]]*\])?: (\d+)", line)
            if m and cur:
                usage[cur][m.group(1)] = int(m.group(2))
    dm = _demangle(list(usage))
    return {dm[k]: v for k, v in usage.items()}


def test_every_persistent_kernel_is_within_its_bounds():
    usage = load_usage()
    pers = {k: v for k, v in usage.items() if PERSISTENT.search(k)}
    assert len(pers) >= 20, sorted(pers)
    bad = []
    for name, u in sorted(pers.items()):
        rows = [b for pat, b in BOUNDS if re.search(pat, name)]
        assert len(rows) == 1, f"{name}: {len(rows)} bound rows match"
        for field, lim in rows[0].items():
            v = u.get(field)
            assert v is not None, (name, field)
            lo, hi = lim if isinstance(lim, tuple) else (0, lim)
            if not lo <= v <= hi:
                bad.append(f"{name}: {field} = {v}, bound [{lo}, {hi}]")
    assert not bad, "\n".join(bad)


def test_headline_kernel_has_no_scratch_in_its_loop():
    """The C2 headline instantiation reloads nothing from scratch memory (a VGPR spill would be
    a memory load inside the iteration loop) and keeps two waves per SIMD."""
    usage = load_usage()
    head = [v for k, v in usage.items()
            if "k_mcmc_resident_pc<dmt::OU<double, 2, 2>, double, 1, false, 4>" in k]
    assert len(head) == 1
    assert head[0]["ScratchSize"] == 0 and head[0]["VGPRs Spill"] == 0
    assert head[0]["Occupancy"] == 2
