"""Generates the committed golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference cannot run here (Julia absent, GuidedProposals/DiffusionDefinition not vendored,
empty reference tests — DESIGN.md §4), so no fixture holds reference output.  What the
fixtures pin instead:
  * philox_kat.npz   — Random123's published Philox4x32-10 known-answer vectors (kat_vectors);
  * ou1d_guiding.npz — the closed-form 1-D OU guiding term (H, F, c) at grid points, computed
                       here from the analytic formulas (independent of every code under test);
  * c1_trace.npz     — C1 (1-D OU bridge) inputs and the canonical-arithmetic outputs of the
                       oracle: one guided solve, 5 parity-mode MCMC iterations;
  * ragged_trace.npz — the ragged 3-recording FHN case with two alternating blockings:
                       inputs (Z, E per iteration) and outputs (decisions, ll, ll°, fetch_ll,
                       final paths).
The last two freeze the canonical arithmetic: any later change to the kernels or
the oracle that alters a bit shows up against them.  Inputs are stored in full, so tests never
regenerate them.  Rounds 5 and 6 changed FHN's canonical order: the ragged
trace's outputs were refreshed from its stored inputs (``--refresh-ragged-outputs``)."""
from __future__ import annotations

import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

OUT = os.path.dirname(os.path.abspath(__file__))

# Random123 kat_vectors, philox4x32_10: (ctr, key) -> out
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


def philox_kat():
    ctr = np.array([k[0] for k in PHILOX_KAT], dtype=np.uint32)
    key = np.array([k[1] for k in PHILOX_KAT], dtype=np.uint32)
    out = np.array([k[2] for k in PHILOX_KAT], dtype=np.uint32)
    np.savez(os.path.join(OUT, "philox_kat.npz"), ctr=ctr, key=key, out=out)


def ou1d_guiding():
    """dX = -θ X dt + σ dW observed at T with V ~ N(X_T, Σ): backward filter closed form
    H(t) = 1/(Σ e^{2θτ}·… ) via the Gaussian transition X_T | X_t ~ N(e^{-θτ}x, s²(τ))."""
    theta, sigma, T, v, Sig = 0.5, 0.5, 1.0, 0.3, 0.01
    t = np.linspace(0.0, T, 11)
    tau = T - t
    mu = np.exp(-theta * tau)
    s2 = sigma ** 2 * (1 - np.exp(-2 * theta * tau)) / (2 * theta)
    V = s2 + Sig
    H = mu * mu / V
    F = mu * v / V
    c = 0.5 * v * v / V + 0.5 * np.log(2 * math.pi * V)
    np.savez(os.path.join(OUT, "ou1d_guiding.npz"), theta=theta, sigma=sigma, T=T, v=v,
             Sigma=Sig, t=t, H=H, F=F, c=c)


def c1_trace():
    import oracle as orc
    from diffusionmcmctools_amd import workloads as W
    from diffusionmcmctools_amd import _lib as L
    w = W.c1_ou1d(N=200)
    iters = 5
    w.meta["hist_len"] = iters
    ora = orc.OracleEnsemble(w.model.kind, w.d, w.m, w.n_points, prec=w.precision, seed=5,
                             grid_shared=w.grid_shared)
    lay = W.fill(ora, w, init_Z=True)
    X0u = ora.download_paths(L.U, 0)
    W0u = ora.download_paths(L.U, 1)
    rng = np.random.default_rng(2024)
    Zs = rng.standard_normal((iters, w.steps_per_iter, w.m))
    Es = rng.exponential(1.0, (iters, w.nblocks))
    ora.loglikhd(lay, L.U, 0, w.nblocks)
    ll0 = ora.block_ll(lay, 0, w.nblocks)[0]
    acc, llp, fetch = [], [], []
    for i in range(1, iters + 1):
        ora.draw_proposal(lay, 0, w.nblocks, Z=Zs[i - 1], iter=i)
        llp.append(ora.block_ll(lay, 0, w.nblocks)[1])
        acc.append(ora.accept_reject(lay, 0, w.nblocks, i, E=Es[i - 1], want_acc=True))
        fetch.append(ora.fetch_ll(lay, 0, w.nblocks, i))
    np.savez(os.path.join(OUT, "c1_trace.npz"), t=w.t, H=w.H, F=w.F, laws=w.laws, X0=w.X0,
             Z0=w.Z0, rho=w.rho, Zs=Zs, Es=Es, X_init=X0u, W_init=W0u, ll0=ll0,
             llp=np.array(llp), acc=np.array(acc), fetch=np.array(fetch, dtype=np.float64),
             X_final=ora.download_paths(L.U, 0), W_final=ora.download_paths(L.U, 1),
             Xp_final=ora.download_paths(L.UPROP, 0))


def ragged_trace():
    import _cases as cs
    import oracle as orc
    from diffusionmcmctools_amd import _lib as L
    case = cs.ragged_case()
    m = case["model"]
    ora = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=case["prec"], seed=11)
    cs.load_ragged(ora, case)
    layA = dict(n_blocks=[2, 3, 2], seg_first=[0, 2, 0, 2, 4, 0, 3], seg_last=[1, 3, 1, 3, 5, 2, 4],
                last=[0, 1, 0, 0, 1, 0, 1], rho=0.7)
    layB = dict(n_blocks=[1, 2, 2], seg_first=[0, 0, 3, 0, 2], seg_last=[3, 2, 5, 1, 4],
                last=[1, 0, 1, 0, 1], rho=0.3)
    iters = 6
    ids = []
    for lay in (layA, layB):
        nb = sum(lay["n_blocks"])
        ids.append((ora.create_layout(lay["n_blocks"], lay["seg_first"], lay["seg_last"],
                                      lay["last"], np.full(nb, lay["rho"]), iters), nb))
    for lid, nb in ids:
        ora.loglikhd(lid, L.U, 0, nb)
    S = ora.S
    rng = np.random.default_rng(99)
    Zs = rng.standard_normal((iters, S, 1))
    Es = rng.exponential(1.0, (iters, 7))
    acc, ll, llp, fetch = [], [], [], []
    for i in range(1, iters + 1):
        lid, nb = ids[(i - 1) % 2]
        ora.draw_proposal(lid, 0, nb, Z=Zs[i - 1], iter=i)
        a = ora.accept_reject(lid, 0, nb, i, E=Es[i - 1, :nb], want_acc=True)
        b_ll, b_llp = ora.block_ll(lid, 0, nb)
        pad = lambda v: np.concatenate([v, np.full(7 - nb, np.nan)])  # noqa: E731
        acc.append(np.concatenate([a, np.zeros(7 - nb, bool)]))
        ll.append(pad(b_ll))
        llp.append(pad(b_llp))
        fetch.append(ora.fetch_ll(lid, 0, nb, i))
    arrays = {k: np.asarray(v) for k, v in case.items() if isinstance(v, np.ndarray)}
    arrays.update(nsegs=np.array(case["nsegs"]),
                  n_points=np.array([n for r in case["n_points"] for n in r]),
                  Zs=Zs, Es=Es, acc=np.array(acc), ll=np.array(ll), llp=np.array(llp),
                  fetch=np.array(fetch, dtype=np.float64),
                  X_final=ora.download_paths(L.U, 0), W_final=ora.download_paths(L.U, 1),
                  Xp_final=ora.download_paths(L.UPROP, 0), Wp_final=ora.download_paths(L.UPROP, 1))
    for k, lay in (("A", layA), ("B", layB)):
        for f in ("n_blocks", "seg_first", "seg_last", "last"):
            arrays[f"lay{k}_{f}"] = np.array(lay[f])
        arrays[f"lay{k}_rho"] = np.array(lay["rho"])
    np.savez_compressed(os.path.join(OUT, "ragged_trace.npz"), **arrays)


def refresh_ragged_outputs():
    """Rounds 5 and 6 (FHN drift reassociated; the FHN step map): keep ragged_trace.npz's stored INPUTS and
    recompute its outputs (decisions, ll, ll°, fetch_ll, final paths) with the current oracle —
    the replay of test_golden.replay_ragged, recording instead of asserting."""
    import oracle as orc
    from diffusionmcmctools_amd import _lib as L
    path = os.path.join(OUT, "ragged_trace.npz")
    g = dict(np.load(path))
    npts, nested, i = g["n_points"], [], 0
    for K in g["nsegs"]:
        nested.append([int(x) for x in npts[i:i + K]])
        i += K
    ens = orc.OracleEnsemble(1, 2, 1, nested, prec=0, seed=11)
    ens.upload_grid(g["t"])
    ens.upload_law(L.U, L.LAW_PP, H=g["H"], F=g["F"], laws=g["laws"])
    ens.upload_law(L.U, L.LAW_PPB, H=g["Hb"], F=g["Fb"], laws=g["lawsb"])
    ens.set_paths(L.U, X=g["X0"])
    ens.draw_unit(L.U, Z=g["Z0"], iter=0, salt=1)
    ens.set_paths(L.UPROP, X=ens.download_paths(L.U, 0), W=ens.download_paths(L.U, 1))
    iters = g["Zs"].shape[0]
    ids = []
    for k in ("A", "B"):
        nb = int(g[f"lay{k}_n_blocks"].sum())
        ids.append((ens.create_layout(g[f"lay{k}_n_blocks"], g[f"lay{k}_seg_first"],
                                      g[f"lay{k}_seg_last"], g[f"lay{k}_last"],
                                      np.full(nb, float(g[f"lay{k}_rho"])), iters), nb))
    for lid, nb in ids:
        ens.loglikhd(lid, L.U, 0, nb)
    acc, ll, llp, fetch = [], [], [], []
    for it in range(1, iters + 1):
        lid, nb = ids[(it - 1) % 2]
        ens.draw_proposal(lid, 0, nb, Z=g["Zs"][it - 1], iter=it)
        a = ens.accept_reject(lid, 0, nb, it, E=g["Es"][it - 1, :nb], want_acc=True)
        pad = lambda v: np.concatenate([v, np.full(7 - nb, np.nan)])  # noqa: E731
        acc.append(np.concatenate([a, np.zeros(7 - nb, bool)]))
        ll.append(pad(ens.get_block_state(lid, L.BLK_LL, 0, nb)))
        llp.append(pad(ens.get_block_state(lid, L.BLK_LLPROP, 0, nb)))
        fetch.append(ens.fetch_ll(lid, 0, nb, it))
    g.update(acc=np.array(acc), ll=np.array(ll), llp=np.array(llp),
             fetch=np.array(fetch, dtype=np.float64),
             X_final=ens.download_paths(L.U, 0), W_final=ens.download_paths(L.U, 1),
             Xp_final=ens.download_paths(L.UPROP, 0), Wp_final=ens.download_paths(L.UPROP, 1))
    np.savez_compressed(path, **g)


if __name__ == "__main__" and "--refresh-ragged-outputs" in sys.argv:
    refresh_ragged_outputs()
    sys.exit(0)

if __name__ == "__main__":
    philox_kat()
    ou1d_guiding()
    c1_trace()
    ragged_trace()
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))
