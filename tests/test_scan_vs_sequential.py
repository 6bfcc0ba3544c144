"""Decision identity of the device's OU recursion with the reference's.

libdmt integrates linear drifts (C1, C2) with a parallel affine scan whose
canonical arithmetic the oracle restates bit for bit (GPU parity tests); the reference runs
GuidedProposals' step-by-step Euler loop.  Here the two recursions run whole MCMC chains on
identical Wiener draws and Exp(1) variables — C1 for 1000 iterations, full-size C2
(1024 × 500) for 100 — and every Metropolis–Hastings decision must agree, with |Δll°| within
SURVEY.md §8(c)'s 1e-10·(1 + Σ|G dt|) (checked against the stricter 1e-10·(1 + |ll°|)).
The sequential chain's decisions are pinned by tests/golden/scan_vs_sequential.json
(tests/golden/make_scan_vs_sequential.py)."""
from __future__ import annotations

import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_scan_vs_sequential as g  # noqa: E402

FIXTURE = json.load(open(os.path.join(HERE, "golden", "scan_vs_sequential.json")))


@pytest.mark.parametrize("case", ["c1", "c2"])
def test_scan_and_sequential_decisions_identical(case):
    mk, kw, n = g.CASES[case]
    got = g.summarize(g.chains(mk(**kw), n, nthreads=min(8, os.cpu_count() or 1)))
    want = FIXTURE[case]
    assert got["decision_flips"] == 0
    assert got["max_rel_dll_prop"] <= FIXTURE["tolerance_rel"]
    assert got["near_ties"] == 0
    assert got["accepted_per_iteration"] == want["accepted_per_iteration"]
    assert got["decisions_sha256"] == want["decisions_sha256"]
