"""Shared builders for parity tests: the same reference-layout inputs feed libdmt and the
oracle.  Test infrastructure."""
from __future__ import annotations

import math

import numpy as np

import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L
from diffusionmcmctools_amd import workloads as W
from diffusionmcmctools_amd.models import (FHN, OU, Observation, artificial_obs_info, guiding_chain,
                                           packed, standard_guid_prop_time_transf)
import oracle as orc


_FULL = {}


def full_workload(cfg):
    """BASELINE.json's per-GPU workloads at full size, built once per test session (C3 takes
    ~40 s of host set-up): C2 1024 × 500, C3 65 536 × 1000 (shorter burn-in of the block
    starts), C5 32 768 × 2000 fp32.  Callers must not modify the arrays."""
    if cfg not in _FULL:
        _FULL[cfg] = {"c2": W.c2_ou2d, "c3": lambda: W.c3_fhn(T_burn=0.2),
                      "c5": W.c5_lorenz}[cfg]()
    return _FULL[cfg]


def sampled_blocks_reference(w, blocks, seed, it, salt=0):
    """Oracle restatement, for single-segment terminal blocks `blocks` of workload w, of the
    fill (init_paths! with w.Z0, ρ = 0) followed by one pCN draw_proposal_path! keyed
    (seed, it, salt) — each block on its own, with its global segment id's normals.  Returns
    per block (X°[npts][d], cumulative W°[npts][m], ll°) as the device downloads them."""
    npts = w.n_points[0][0]
    d, m, prec = w.d, w.m, w.precision
    out = []
    for b in blocks:
        rows = slice(b * npts, (b + 1) * npts)
        laws = w.laws[b:b + 1]
        H = w.H if w.H_shared else w.H[rows]
        F = w.F[rows]
        Z0 = w.Z0[b * (npts - 1):(b + 1) * (npts - 1)]
        X1, W1, _, nf = orc.draw_terminal_blocks(
            w.model.kind, d, m, npts, laws, w.t, H, F, w.X0[rows], np.zeros((npts, m)),
            np.zeros(1), Z=Z0, prec=prec, t_shared=True, H_shared=w.H_shared)
        assert nf == 0
        Z1 = orc.normals_segment(seed, b, it, salt, npts - 1, m, prec)
        Xo, Wo, llo, _ = orc.draw_terminal_blocks(
            w.model.kind, d, m, npts, laws, w.t, H, F, X1, W1, np.full(1, w.rho), Z=Z1,
            prec=prec, t_shared=True, H_shared=w.H_shared)
        out.append((Xo.astype(np.float64), orc.w_from_increments(Wo, prec).astype(np.float64),
                    float(llo[0])))
    return out


def both(w, seed=11, hist_len=0, init_Z=True, mapping=L.MAP_AUTO):
    """Device ensemble + oracle ensemble holding the same workload; returns (dev, ora, layout)."""
    w.meta["hist_len"] = hist_len
    dev = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=seed,
                       grid_shared=w.grid_shared, mapping=mapping)
    lay_d = W.fill(dev, w, init_Z=init_Z)
    ora = orc.OracleEnsemble(w.model.kind, w.d, w.m, w.n_points, prec=w.precision, seed=seed,
                             grid_shared=w.grid_shared)
    lay_o = W.fill(ora, w, init_Z=init_Z)
    assert lay_d == lay_o
    return dev, ora, lay_d


def assert_paths_equal(dev, ora, exact=True, rtol=0.0, atol=0.0, equal_nan=False):
    for unit in (L.U, L.UPROP):
        for what in (0, 1, 2):
            a = dev.download_paths(unit, what)
            b = ora.download_paths(unit, what)
            if exact:
                assert np.array_equal(a, b, equal_nan=equal_nan), (
                    f"unit {unit} {('XX', 'WW', 'dW')[what]}: max |diff| "
                    f"{np.nanmax(np.abs(a - b))} at {np.unravel_index(np.nanargmax(np.abs(a - b)), a.shape)}")
            else:
                np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def assert_ll_equal(dev, ora, lay, nb, exact=True, rtol=0.0):
    a = dev.get_block_state(lay, L.BLK_LL, 0, nb)
    ap = dev.get_block_state(lay, L.BLK_LLPROP, 0, nb)
    b, bp = ora.block_ll(lay, 0, nb)
    if exact:
        assert np.array_equal(a, b), f"ll max diff {np.nanmax(np.abs(a - b))}"
        assert np.array_equal(ap, bp), f"ll° max diff {np.nanmax(np.abs(ap - bp))}"
    else:
        np.testing.assert_allclose(a, b, rtol=rtol)
        np.testing.assert_allclose(ap, bp, rtol=rtol)


def ragged_case(seed=5, prec=L.F64, model=None):
    """3 recordings of an FHN model with 4, 6 and 5 inter-observation segments of unequal
    lengths and point counts (non-shared grids), per-segment linearised auxiliary laws, PP laws
    chained over the whole recording and PPb laws with an artificial exact end observation
    (guid_prop_for_blocking, src/sampling_unit.jl:61-66)."""
    rng = np.random.default_rng(seed)
    model = FHN(0.1, -0.8, 1.5, 0.0, 0.3) if model is None else model
    nsegs = [4, 6, 5]
    n_points, grids, laws_pp, H_pp, F_pp, H_b, F_b, laws_b, X0 = [], [], [], [], [], [], [], [], []
    Hobs, Fobs, cobs = [], [], []
    for r, K in enumerate(nsegs):
        t0 = 0.0
        obs_t = np.cumsum(rng.uniform(0.05, 0.12, K))
        gr, auxes, infos, binfo = [], [], [], []
        for k in range(K):
            n = int(rng.integers(20, 140))
            gr.append(standard_guid_prop_time_transf(t0, obs_t[k], (obs_t[k] - t0) / n))
            v = rng.uniform(-1.2, 1.2)
            auxes.append(model.aux(v))
            infos.append(Observation(obs_t[k], np.array([v]), np.array([[1.0, 0.0]]), 0.01 * np.eye(1)).info())
            Ha, Fa, ca = artificial_obs_info(rng.standard_normal(2) * 0.5, 1e-11)
            Ho, Fo, co = infos[-1]
            binfo.append((Ha + Ho, Fa + Fo, ca + co))
            t0 = obs_t[k]
        for inf in infos:  # the observation at each segment end (for the device filter)
            Hobs.append(packed(inf[0])); Fobs.append(np.asarray(inf[1], dtype=np.float64))
            cobs.append(float(inf[2]))
        chain = guiding_chain(auxes, gr, infos)
        for k in range(K):
            H, F, c = chain[k]
            (Hb, Fb, cb), = guiding_chain([auxes[k]], [gr[k]], [binfo[k]])
            n_points.append(len(gr[k]))
            grids.append(gr[k])
            H_pp.append(H); F_pp.append(F); laws_pp.append(model.law_record(auxes[k], c[0]))
            H_b.append(Hb); F_b.append(Fb); laws_b.append(model.law_record(auxes[k], cb[0]))
            x = np.zeros((len(gr[k]), 2))
            if k == 0:
                x[0] = rng.standard_normal(2) * 0.5
            X0.append(x)
    npts_nested, i = [], 0
    for K in nsegs:
        npts_nested.append(n_points[i:i + K]); i += K
    case = dict(model=model, n_points=npts_nested, t=np.concatenate(grids),
                H=np.concatenate(H_pp), F=np.concatenate(F_pp), laws=np.stack(laws_pp),
                Hb=np.concatenate(H_b), Fb=np.concatenate(F_b), lawsb=np.stack(laws_b),
                X0=np.concatenate(X0), prec=prec, nsegs=nsegs, Hobs=np.stack(Hobs),
                Fobs=np.stack(Fobs), cobs=np.array(cobs))
    P = case["t"].size
    G = sum(nsegs)
    case["Z0"] = rng.standard_normal((P - G, 1))
    return case


def load_ragged(ens, case):
    ens.upload_grid(case["t"])
    ens.upload_law(L.U, L.LAW_PP, H=case["H"], F=case["F"], laws=case["laws"])
    ens.upload_law(L.U, L.LAW_PPB, H=case["Hb"], F=case["Fb"], laws=case["lawsb"])
    ens.set_paths(L.U, X=case["X0"])
    ens.draw_unit(L.U, Z=case["Z0"], iter=0, salt=1)
    X = ens.download_paths(L.U, 0)
    Wp = ens.download_paths(L.U, 1)
    ens.set_paths(L.UPROP, X=X, W=Wp)


def ou_ragged_model():
    """A 2-D OU model with one noise (d = 2, m = 1) for the ragged case: its auxiliary law is
    an OU law with Θ̃ = diag(0.7, 0.4) whatever the observation (G ≢ 0)."""
    class _OU(OU):
        def aux(self, v=None):
            return OU.aux(self, Theta_t=np.diag([0.7, 0.4]))
    return _OU([[1.0, 0.3], [-0.3, 0.8]], [0.1, -0.2], [[0.2], [0.5]])


def ragged_pair(seed=11, hist_len=8, mapping=L.MAP_AUTO, model=None, prec=L.F64):
    case = ragged_case(model=model, prec=prec)
    m = case["model"]
    dev = dmt.Ensemble(m.kind, m.d, m.m, case["n_points"], precision=case["prec"], seed=seed,
                       mapping=mapping)
    ora = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=case["prec"], seed=seed)
    for e in (dev, ora):
        load_ragged(e, case)
    # two alternating block layouts per recording (biblock/smoothing_with_blocking.md:69)
    layA = dict(n_blocks=[2, 3, 2], seg_first=[0, 2, 0, 2, 4, 0, 3], seg_last=[1, 3, 1, 3, 5, 2, 4],
                last=[0, 1, 0, 0, 1, 0, 1])
    layB = dict(n_blocks=[1, 2, 2], seg_first=[0, 0, 3, 0, 2], seg_last=[3, 2, 5, 1, 4],
                last=[1, 0, 1, 0, 1])
    ids = []
    for lay, rho in ((layA, 0.7), (layB, 0.3)):
        nb = int(sum(lay["n_blocks"]))
        ids_ = [e.create_layout(lay["n_blocks"], lay["seg_first"], lay["seg_last"], lay["last"],
                                np.full(nb, rho), hist_len) for e in (dev, ora)]
        assert ids_[0] == ids_[1]
        ids.append((ids_[0], nb))
    return case, dev, ora, ids
