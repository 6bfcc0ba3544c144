"""Generates tests/golden/scan_vs_sequential.json: the canonical parallel affine scan (the
device's OU recursion, oracle/dmt_oracle.c, bit-identical to libdmt by the GPU parity tests)
against the reference's step-by-step Euler recursion (oracle sequential=True: the loop of
GuidedProposals' solve!) on identical Wiener draws and Exp(1)
variables, at C1 (1 block x 200 steps, 1000 MCMC iterations) and full C2 (1024 blocks x 500
steps, 100 iterations).  Records per-iteration accepted counts and a hash of every decision of
the sequential chain, decision flips between the chains, near-ties and max |Δll°|.

  python tests/golden/make_scan_vs_sequential.py      (from the repo root; ~1 min on 8 cores)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as orc  # noqa: E402
from diffusionmcmctools_amd import workloads as W  # noqa: E402

SEED = 0xD1FF
TOL = 1e-10   # |Δll| ≤ 1e-10·(1 + Σ|G dt|); here scaled by (1 + |ll°|) ≤ that
CASES = {"c1": (W.c1_ou1d, {}, 1000), "c2": (W.c2_ou2d, {}, 100)}


def chains(w, n_iter, nthreads=8):
    B, npts = w.nblocks, w.n_points[0][0]
    draw = lambda Xa, Wa, rho, it, seq, Z=None: orc.draw_terminal_blocks(  # noqa: E731
        w.model.kind, w.d, w.m, npts, w.laws, w.t, w.H, w.F, Xa, Wa, rho, Z=Z, seed=SEED,
        it=it, salt=0, prec=w.precision, nthreads=nthreads, t_shared=True,
        H_shared=w.H_shared, sequential=seq)
    # init_paths!: one fresh draw (ρ = 0) with the workload's normals, shared by both chains
    X0, W0, ll0, nf = draw(w.X0, np.zeros((B * npts, w.m)), np.zeros(B), 0, False, Z=w.Z0)
    assert nf == 0
    rho = np.full(B, w.rho)
    out = {}
    for name, seq in (("scan", False), ("sequential", True)):
        Xa, Wa, lla = X0.copy(), W0.copy(), ll0.copy()
        acc_all, llp_all, margin = [], [], []
        for it in range(1, n_iter + 1):
            Xo, Wo, llp, _ = draw(Xa, Wa, rho, it, seq)
            E = orc.exp1_range(SEED, 0, B, it, 0)
            acc = E > -(llp - lla)
            margin.append(np.abs(E + (llp - lla)))
            sel = np.repeat(acc, npts)
            Xa = np.where(sel[:, None], Xo, Xa)
            Wa = np.where(sel[:, None], Wo, Wa)
            lla = np.where(acc, llp, lla)
            acc_all.append(acc)
            llp_all.append(llp)
        out[name] = (np.array(acc_all), np.array(llp_all), np.array(margin))
    return out


def summarize(out):
    a_s, l_s, m_s = out["scan"]
    a_q, l_q, m_q = out["sequential"]
    flips = int((a_s != a_q).sum())
    # |Δll°| while the chains agree (identical decisions ⇒ the same proposals up to rounding)
    rel = np.abs(l_s - l_q) / (1.0 + np.abs(l_q))
    return {"iterations": int(a_q.shape[0]), "blocks": int(a_q.shape[1]),
            "decision_flips": flips, "decisions": int(a_q.size),
            "near_ties": int((m_q < TOL * (1.0 + np.abs(l_q))).sum()),
            "max_rel_dll_prop": float(rel.max()),
            "min_decision_margin": float(m_q.min()),
            "accepted_per_iteration": a_q.sum(axis=1).astype(int).tolist(),
            "decisions_sha256": hashlib.sha256(np.packbits(a_q).tobytes()).hexdigest()}


def main():
    res = {"seed": SEED, "tolerance_rel": TOL}
    for k, (mk, kw, n) in CASES.items():
        res[k] = summarize(chains(mk(**kw), n))
        print(k, {x: y for x, y in res[k].items() if x != "accepted_per_iteration"})
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                           "scan_vs_sequential.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
