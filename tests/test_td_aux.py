"""Time-dependent linear auxiliary laws within a segment (include/dmt.h dmt_upload_aux,
DMT_LAW_AUXTD).  The reference takes any linear auxiliary law of
GuidedProposals (aux_laws, /root/reference/src/sampling_unit.jl:55-66), whose B̃(t), β̃(t) may
vary in t; step i of a segment takes the coefficients of its left point t_i, frozen over
[t_i, t_{i+1}], in the Girsanov term G and in the backward filter's exact step transition.

CPU: the oracle's and libdmt's host filters agree bit for bit; a constant table reproduces the
time-homogeneous law bit for bit (filter and oracle ensemble); the frozen-coefficient filter
converges (first order) as the grid is refined — the guiding term of the ODEs of SURVEY.md A.5.
GPU: device == oracle bit for bit on the ragged FHN ensemble with a varying table on part of
the segments, through the blocking loop (set_obs!, recompute_guiding_term!, find_W_for_X!,
loglikhd!, draws with caller and device normals, accept, recompute_path!), lane and wave
mappings, fp64 and fp32; and on the ragged OU ensemble (scan kernels, through the blocking
loop and dmt_mcmc_run).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as orc  # noqa: E402
import _cases as cs  # noqa: E402
import diffusionmcmctools_amd as dmt  # noqa: E402
from diffusionmcmctools_amd import _lib as L  # noqa: E402

MAPPINGS = [L.MAP_LANE, L.MAP_WAVE]


def _law2():
    """A 2-D linear auxiliary law with time-varying coefficients and noise on coordinate 2."""
    B0 = np.array([[-1.0, -0.5], [1.5, -1.0]])
    B1 = np.array([[0.4, 0.0], [-0.3, 0.2]])
    B = lambda t: B0 + np.sin(3.0 * t) * B1  # noqa: E731
    beta = lambda t: np.array([0.3 + 0.5 * t, -0.2 * np.cos(2.0 * t)])  # noqa: E731
    at = np.array([0.0, 0.0, 0.09])  # packed σ̃σ̃ᵀ, σ̃ = (0, 0.3)
    return B, beta, at


def _table(B, beta, t):
    return np.stack([np.concatenate([B(x).ravel(), beta(x)]) for x in t])


def _end_info():
    HT = np.array([[25.0, 0.0], [0.0, 0.0]])
    return orc.packed_sym(HT), np.array([12.5, 0.0]), 3.1


def test_td_filter_host_equals_oracle_and_constant_equals_homogeneous():
    B, beta, at = _law2()
    t = np.sort(np.concatenate([[0.0, 1.0], np.random.default_rng(3).uniform(0, 1, 150)]))
    HT, FT, cT = _end_info()
    aux = _table(B, beta, t)
    h = dmt.guiding_linear_td(aux, at, t, HT, FT, cT)
    o = orc.backward_filter_segment_td(2, aux, at, t, HT, FT, cT)
    for a, b in zip(h, o):
        assert np.array_equal(a, b)
    # a constant table is the time-homogeneous law, bit for bit (host and oracle)
    const = np.tile(np.concatenate([B(0.4).ravel(), beta(0.4)]), (t.size, 1))
    hc = dmt.guiding_linear_td(const, at, t, HT, FT, cT)
    hh = dmt.guiding_linear(B(0.4), beta(0.4), at, t, HT, FT, cT)
    oc = orc.backward_filter_segment_td(2, const, at, t, HT, FT, cT)
    for a, b, c in zip(hc, hh, oc):
        assert np.array_equal(a, b) and np.array_equal(a, c)
    # and the varying table really is used
    assert not np.array_equal(h[0], hh[0])


def test_td_filter_converges_as_the_grid_is_refined():
    """The step transition with the trapezoidal average of the coefficients over each step is a
    second-order scheme for the filter of the time-dependent law (SURVEY.md A.5's ODEs): the
    guiding term at t0 on grids of n, 2n, … steps converges, each halving of the step cutting
    the error against the finest grid by about four (left-point frozen coefficients, the
    previous scheme, halved it)."""
    B, beta, at = _law2()
    HT, FT, cT = _end_info()

    def at_t0(n):
        t = np.linspace(0.0, 1.0, n + 1)
        H, F, c = dmt.guiding_linear_td(_table(B, beta, t), at, t, HT, FT, cT)
        return np.concatenate([H[0], F[0], [c[0]]])

    ref = at_t0(4096)
    errs = [np.max(np.abs(at_t0(n) - ref)) for n in (32, 64, 128, 256)]
    for e0, e1 in zip(errs, errs[1:]):
        assert 3.3 < e0 / e1 < 4.8, errs
    assert errs[-1] < 5e-5 * np.max(np.abs(ref))


def test_td_filter_matches_an_independent_ode_solution():
    """Against an independent solution of SURVEY.md A.5's backward ODEs for the time-dependent
    linear law (scipy solve_ivp, RK45 at tight tolerance, between the observation at t = 1 and
    t0 = 0): dH = -(B̃'H + HB̃ - HãH)dt, dF = -(B̃'F - Hãf + ... ) in information form —
    integrated here for (H, F, c) directly: H' = -B̃ᵀH - HB̃ + HãH, F' = -B̃ᵀF + Hã F + Hβ̃,
    c' = β̃ᵀF + ½ Fᵀ ã F - ½ tr(ã H)."""
    from scipy.integrate import solve_ivp
    B, beta, at = _law2()
    HT, FT, cT = _end_info()
    A = orc.unpacked(at, 2)

    def rhs(t, y):
        H = y[:4].reshape(2, 2)
        F = y[4:6]
        Bt, bt = B(t), beta(t)
        dH = -Bt.T @ H - H @ Bt + H @ A @ H
        dF = -Bt.T @ F + H @ A @ F + H @ bt
        dc = bt @ F + 0.5 * F @ A @ F - 0.5 * np.trace(A @ H)
        return np.concatenate([dH.ravel(), dF, [dc]])

    y1 = np.concatenate([orc.unpacked(HT, 2).ravel(), FT, [cT]])
    sol = solve_ivp(rhs, (1.0, 0.0), y1, rtol=1e-12, atol=1e-12)
    H0, F0 = sol.y[:4, -1].reshape(2, 2), sol.y[4:6, -1]
    t = np.linspace(0.0, 1.0, 1025)
    H, F, c = dmt.guiding_linear_td(_table(B, beta, t), at, t, HT, FT, cT)
    assert np.max(np.abs(orc.unpacked(H[0], 2) - H0)) < 1e-5 * np.max(np.abs(H0))
    assert np.max(np.abs(F[0] - F0)) < 1e-5 * max(1.0, np.max(np.abs(F0)))


def _flag_segments(ens, kinds, segs, value=1.0):
    """Set DMT_LAW_AUXTD (1: B̃, β̃ from the table; 2: ã too) in the law records of `segs`
    (both units, the given kinds)."""
    for unit in (L.U, L.UPROP):
        for kind in kinds:
            laws = ens.download_law(unit, kind)[2].copy()
            laws[segs, L.LAW_AUXTD] = value
            ens.upload_law(unit, kind, laws=laws)


def _tables(case, ens, vary=True, with_a=False):
    """Per-point aux tables of both kinds: each segment's record B̃, β̃ (and with_a: ã = a − (a −
    ã) of the record, packed), plus (vary) a time-varying perturbation — for the PPb laws a
    different one; ã's varies the noise coordinate's variance."""
    t = case["t"]
    out = []
    for kind, laws in ((L.LAW_PP, case["laws"]), (L.LAW_PPB, case["lawsb"])):
        rows = []
        for g, n in enumerate(np.concatenate(case["n_points"])):
            rec = laws[g]
            Bt = rec[L.LAW_BT:L.LAW_BT + 4].reshape(2, 2)
            be = rec[L.LAW_BETA:L.LAW_BETA + 2]
            at = rec[L.LAW_A:L.LAW_A + 3] - rec[L.LAW_DA:L.LAW_DA + 3]
            off = int(np.sum(np.concatenate(case["n_points"])[:g]))
            for tt in t[off:off + n]:
                if vary:
                    s = np.sin(7.0 * tt + g + kind)
                    Bq = Bt + s * np.array([[0.3, -0.1], [0.2, 0.0]])
                    bq = be + np.array([0.4 * np.cos(5.0 * tt), 0.1 * s])
                    aq = at * np.array([1.0, 1.0, 1.0 + 0.3 * np.cos(3.0 * tt + g)])
                else:
                    Bq, bq, aq = Bt, be, at
                rows.append(np.concatenate([Bq.ravel(), bq] + ([aq] if with_a else [])))
        out.append(np.array(rows))
    return out


def _td_pair(mapping, prec, vary=True, segs=None, oracle_only=False, with_a=False, model=None,
             hist_len=6):
    case = cs.ragged_case(prec=prec, model=model)
    m = case["model"]
    ens = []
    if not oracle_only:
        ens.append(dmt.Ensemble(m.kind, m.d, m.m, case["n_points"], precision=prec, seed=11,
                                mapping=mapping))
    ens.append(orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=prec, seed=11))
    G = int(sum(case["nsegs"]))
    segs = np.arange(0, G, 2) if segs is None else segs
    tabs = _tables(case, ens[0], vary, with_a)
    for e in ens:
        cs.load_ragged(e, case)
        e.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
        _flag_segments(e, (L.LAW_PP, L.LAW_PPB), segs, 2.0 if with_a else 1.0)
        e.upload_aux(L.LAW_PP, tabs[0])
        e.upload_aux(L.LAW_PPB, tabs[1])
    layA = dict(n_blocks=[2, 3, 2], seg_first=[0, 2, 0, 2, 4, 0, 3], seg_last=[1, 3, 1, 3, 5, 2, 4],
                last=[0, 1, 0, 0, 1, 0, 1])
    layB = dict(n_blocks=[1, 2, 2], seg_first=[0, 0, 3, 0, 2], seg_last=[3, 2, 5, 1, 4],
                last=[1, 0, 1, 0, 1])
    ids = []
    for lay, rho in ((layA, 0.7), (layB, 0.3)):
        nb = int(sum(lay["n_blocks"]))
        ids_ = [e.create_layout(lay["n_blocks"], lay["seg_first"], lay["seg_last"], lay["last"],
                                np.full(nb, rho), hist_len) for e in ens]
        assert len(set(ids_)) == 1
        ids.append((ids_[0], nb))
    return case, ens, ids


def _blocking_loop(ens, ids, S, iters, rng, device_rng=False):
    out = []
    for i in range(1, iters + 1):
        lid, nb = ids[(i - 1) % 2]
        Z = rng.standard_normal((S, 1))
        E = rng.exponential(1.0, nb)
        for e in ens:
            e.set_obs(lid, 0, nb)
            e.recompute_guiding_term(lid, 0, nb, unit=L.U)
            e.find_W_for_X(lid, 0, nb)
            e.loglikhd(lid, L.U, 0, nb)
            if device_rng:
                e.draw_proposal(lid, 0, nb, iter=i, salt=3)
            else:
                e.draw_proposal(lid, 0, nb, Z=Z, iter=i)
        out.append([e.accept_reject(lid, 0, nb, i, E=E, want_acc=True) for e in ens])
    return out


def _fixed_aux(ens):
    """Auxiliary laws that set_obs! does not re-linearise (DMT_LAW_AUXLIN = 0): a
    time-dependent record takes B̃, β̃ from its table, so only a fixed law compares with it."""
    for unit in (L.U, L.UPROP):
        for kind in (L.LAW_PP, L.LAW_PPB):
            laws = ens.download_law(unit, kind)[2].copy()
            laws[:, L.LAW_AUXLIN] = 0.0
            ens.upload_law(unit, kind, laws=laws)


def test_oracle_constant_table_equals_homogeneous_law():
    """The oracle with every segment flagged time-dependent and a table holding each record's
    own B̃, β̃ runs the blocking loop bit-identically to the plain oracle (fixed laws)."""
    case, (td,), ids = _td_pair(None, L.F64, vary=False, oracle_only=True,
                                segs=np.arange(sum(cs.ragged_case()["nsegs"])))
    m = case["model"]
    plain = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=L.F64, seed=11)
    cs.load_ragged(plain, case)
    plain.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    for e in (td, plain):
        _fixed_aux(e)
    for lay in (dict(n_blocks=[2, 3, 2], seg_first=[0, 2, 0, 2, 4, 0, 3],
                     seg_last=[1, 3, 1, 3, 5, 2, 4], last=[0, 1, 0, 0, 1, 0, 1], rho=0.7),
                dict(n_blocks=[1, 2, 2], seg_first=[0, 0, 3, 0, 2], seg_last=[3, 2, 5, 1, 4],
                     last=[1, 0, 1, 0, 1], rho=0.3)):
        nb = int(sum(lay["n_blocks"]))
        plain.create_layout(lay["n_blocks"], lay["seg_first"], lay["seg_last"], lay["last"],
                            np.full(nb, lay["rho"]), 6)
    S = td.S
    a = _blocking_loop([td], ids, S, 4, np.random.default_rng(2))
    b = _blocking_loop([plain], ids, S, 4, np.random.default_rng(2))
    for x, y in zip(a, b):
        assert np.array_equal(x[0], y[0])
    cs.assert_paths_equal(td, plain)
    for lid, nb in ids:
        cs.assert_ll_equal(td, plain, lid, nb)


# ------------------------------------------------------------------ linear drifts (OU)
# A linear drift's recursion is the target law's affine step map (the scan kernels): the
# auxiliary law enters G and the backward filter only, so a time-dependent one takes step i's
# B̃(t_i), β̃(t_i) (and a − ã(t_i)) in phase 3's G of the scan and in the filter.
def _ou_loop(ens, ids, S, iters, rng, device_rng=False):
    """The OU blocking loop: set_obs!, recompute_guiding_term!, loglikhd!, draws (caller or
    device normals), accept."""
    out = []
    for i in range(1, iters + 1):
        lid, nb = ids[(i - 1) % 2]
        Z = rng.standard_normal((S, 1))
        E = rng.exponential(1.0, nb)
        for e in ens:
            e.set_obs(lid, 0, nb)
            e.recompute_guiding_term(lid, 0, nb, unit=L.U)
            e.loglikhd(lid, L.U, 0, nb)
            if device_rng:
                e.draw_proposal(lid, 0, nb, iter=i, salt=3)
            else:
                e.draw_proposal(lid, 0, nb, Z=Z, iter=i)
        out.append([e.accept_reject(lid, 0, nb, i, E=E, want_acc=True) for e in ens])
    return out


def test_oracle_ou_constant_table_equals_homogeneous_law():
    """OU: every segment flagged time-dependent with a table holding each record's own B̃, β̃
    runs the blocking loop bit-identically to the plain oracle; a varying table changes the
    Girsanov weights and the guiding term."""
    model = cs.ou_ragged_model()
    G = sum(cs.ragged_case()["nsegs"])
    case, (td,), ids = _td_pair(None, L.F64, vary=False, oracle_only=True, segs=np.arange(G),
                                model=model)
    plain = orc.OracleEnsemble(model.kind, model.d, model.m, case["n_points"], prec=L.F64, seed=11)
    cs.load_ragged(plain, case)
    plain.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    for lay in (dict(n_blocks=[2, 3, 2], seg_first=[0, 2, 0, 2, 4, 0, 3],
                     seg_last=[1, 3, 1, 3, 5, 2, 4], last=[0, 1, 0, 0, 1, 0, 1], rho=0.7),
                dict(n_blocks=[1, 2, 2], seg_first=[0, 0, 3, 0, 2], seg_last=[3, 2, 5, 1, 4],
                     last=[1, 0, 1, 0, 1], rho=0.3)):
        nb = int(sum(lay["n_blocks"]))
        plain.create_layout(lay["n_blocks"], lay["seg_first"], lay["seg_last"], lay["last"],
                            np.full(nb, lay["rho"]), 6)
    a = _ou_loop([td], ids, td.S, 4, np.random.default_rng(2))
    b = _ou_loop([plain], ids, td.S, 4, np.random.default_rng(2))
    for x, y in zip(a, b):
        assert np.array_equal(x[0], y[0])
    cs.assert_paths_equal(td, plain)
    for lid, nb in ids:
        cs.assert_ll_equal(td, plain, lid, nb)
    _, (var,), ids = _td_pair(None, L.F64, vary=True, oracle_only=True, segs=np.arange(G),
                              model=model)
    lid, nb = ids[0]
    for e in (var, td):
        e.loglikhd(lid, L.U, 0, nb)
    assert not np.array_equal(var.get_block_state(lid, L.BLK_LL, 0, nb),
                              td.get_block_state(lid, L.BLK_LL, 0, nb))
    for e in (var, td):
        e.recompute_guiding_term(lid, 0, nb, unit=L.U)
    assert not np.array_equal(var.download_law(L.U, L.LAW_PP)[0], td.download_law(L.U, L.LAW_PP)[0])


def _law2a():
    """_law2 with a time-dependent ã(t) = σ̃σ̃ᵀ(t) too (σ̃ = (0, 0.3(1 + 0.4 sin 2t)))."""
    B, beta, _ = _law2()
    at = lambda t: np.array([0.0, 0.0, (0.3 * (1.0 + 0.4 * np.sin(2.0 * t))) ** 2])  # noqa: E731
    return B, beta, at


def _table_a(B, beta, at, t):
    return np.stack([np.concatenate([B(x).ravel(), beta(x), at(x)]) for x in t])


def test_tda_filter_host_equals_oracle_and_constant_equals_td():
    B, beta, at = _law2a()
    t = np.sort(np.concatenate([[0.0, 1.0], np.random.default_rng(5).uniform(0, 1, 150)]))
    HT, FT, cT = _end_info()
    h = dmt.guiding_linear_tda(_table_a(B, beta, at, t), t, HT, FT, cT)
    o = orc.backward_filter_segment_tda(2, _table_a(B, beta, at, t), t, HT, FT, cT)
    for a_, b_ in zip(h, o):
        assert np.array_equal(a_, b_)
    # a constant ã column is the ã of dmt_guiding_linear_td, bit for bit
    a0 = at(0.0)
    hc = dmt.guiding_linear_tda(_table_a(B, beta, lambda x: a0, t), t, HT, FT, cT)
    ht = dmt.guiding_linear_td(_table(B, beta, t), a0, t, HT, FT, cT)
    for a_, b_ in zip(hc, ht):
        assert np.array_equal(a_, b_)
    assert not np.array_equal(h[0], ht[0])


def test_tda_filter_converges_to_the_ode_at_second_order():
    """With ã(t) time-dependent as well, the trapezoidal step transition still converges at
    second order to SURVEY.md A.5's backward ODEs (here integrated independently with
    solve_ivp, ã(t) in the Riccati term)."""
    from scipy.integrate import solve_ivp
    B, beta, at = _law2a()
    HT, FT, cT = _end_info()

    def rhs(t, y):
        H = y[:4].reshape(2, 2)
        F = y[4:6]
        Bt, bt, A = B(t), beta(t), orc.unpacked(at(t), 2)
        dH = -Bt.T @ H - H @ Bt + H @ A @ H
        dF = -Bt.T @ F + H @ A @ F + H @ bt
        dc = bt @ F + 0.5 * F @ A @ F - 0.5 * np.trace(A @ H)
        return np.concatenate([dH.ravel(), dF, [dc]])

    sol = solve_ivp(rhs, (1.0, 0.0), np.concatenate([orc.unpacked(HT, 2).ravel(), FT, [cT]]),
                    rtol=1e-12, atol=1e-12)
    ref = np.concatenate([orc.packed_sym(sol.y[:4, -1].reshape(2, 2)), sol.y[4:6, -1]])

    def at_t0(n):
        t = np.linspace(0.0, 1.0, n + 1)
        H, F, _ = dmt.guiding_linear_tda(_table_a(B, beta, at, t), t, HT, FT, cT)
        return np.concatenate([H[0], F[0]])

    errs = [np.max(np.abs(at_t0(n) - ref)) for n in (32, 64, 128, 256)]
    for e0, e1 in zip(errs, errs[1:]):
        assert 3.3 < e0 / e1 < 4.8, errs


def test_oracle_tda_with_the_records_a_equals_td():
    """An ã column equal to each record's own ã (FHN: ã = a, so a − ã(t_i) = 0 exactly and the
    trace term adds fma(−½, 0, G) = G) runs the blocking loop bit-identically to the B̃, β̃-only
    table (DMT_LAW_AUXTD 2 vs 1) on the oracle."""
    segs = np.arange(sum(cs.ragged_case()["nsegs"]))
    _, (ta,), ids = _td_pair(None, L.F64, vary=False, oracle_only=True, segs=segs, with_a=True)
    _, (t1,), _ = _td_pair(None, L.F64, vary=False, oracle_only=True, segs=segs)
    for e in (ta, t1):
        _fixed_aux(e)
    a = _blocking_loop([ta], ids, ta.S, 4, np.random.default_rng(2))
    b = _blocking_loop([t1], ids, t1.S, 4, np.random.default_rng(2))
    for x, y in zip(a, b):
        assert np.array_equal(x[0], y[0])
    cs.assert_paths_equal(ta, t1)
    for lid, nb in ids:
        cs.assert_ll_equal(ta, t1, lid, nb)


def test_oracle_varying_a_enters_girsanov_and_filter():
    """A varying ã(t) changes both the guiding term and the Girsanov weights (oracle)."""
    segs = np.arange(sum(cs.ragged_case()["nsegs"]))
    _, (ta,), ids = _td_pair(None, L.F64, vary=True, oracle_only=True, segs=segs, with_a=True)
    _, (t1,), _ = _td_pair(None, L.F64, vary=True, oracle_only=True, segs=segs)
    lid, nb = ids[0]
    for e in (ta, t1):
        e.set_obs(lid, 0, nb)
        e.recompute_guiding_term(lid, 0, nb, unit=L.U)
    assert not np.array_equal(ta.download_law(L.U, L.LAW_PP)[0], t1.download_law(L.U, L.LAW_PP)[0])
    for e in (ta, t1):
        e.upload_law(L.U, L.LAW_PP, H=t1.download_law(L.U, L.LAW_PP)[0])
        e.loglikhd(lid, L.U, 0, nb)
    assert not np.array_equal(ta.block_ll(lid, 0, nb)[0], t1.block_ll(lid, 0, nb)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("with_a", [False, True], ids=["Bbeta", "Bbeta_a"])
@pytest.mark.parametrize("prec", [L.F64, L.F32], ids=["f64", "f32"])
@pytest.mark.parametrize("mapping", MAPPINGS, ids=["lane", "wave"])
def test_td_aux_blocking_loop_device_equals_oracle(mapping, prec, with_a):
    case, (dev, ora), ids = _td_pair(mapping, prec, with_a=with_a)
    rng = np.random.default_rng(8)
    res = _blocking_loop([dev, ora], ids, dev.S, 6, rng)
    for i, (ad, ao) in enumerate(res):
        assert np.array_equal(ad, ao), f"iteration {i + 1}"
    for kind in (L.LAW_PP, L.LAW_PPB):
        for unit in (L.U, L.UPROP):
            for a_, b_ in zip(dev.download_law(unit, kind), ora.download_law(unit, kind)):
                assert np.array_equal(a_, b_), (unit, kind)
    cs.assert_paths_equal(dev, ora)
    for lid, nb in ids:
        cs.assert_ll_equal(dev, ora, lid, nb)
    # device normals, then recompute_path! under u°'s law
    res = _blocking_loop([dev, ora], ids, dev.S, 2, rng, device_rng=True)
    for ad, ao in res:
        assert np.array_equal(ad, ao)
    for lid, nb in ids:
        for e in (dev, ora):
            e.recompute_path(lid, 0, nb)
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, lid, nb)
    dev.close()


@pytest.mark.gpu
def test_td_aux_removed_table_is_homogeneous_again():
    """upload_aux(kind, None) drops the table: the flagged segments fall back to the record's
    B̃, β̃ (the time-homogeneous kernels run again), device == oracle."""
    case, (dev, ora), ids = _td_pair(L.MAP_LANE, L.F64)
    for e in (dev, ora):
        e.upload_aux(L.LAW_PP, None)
        e.upload_aux(L.LAW_PPB, None)
    res = _blocking_loop([dev, ora], ids, dev.S, 2, np.random.default_rng(4))
    for ad, ao in res:
        assert np.array_equal(ad, ao)
    cs.assert_paths_equal(dev, ora)
    dev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("with_a", [False, True], ids=["Bbeta", "Bbeta_a"])
@pytest.mark.parametrize("prec", [L.F64, L.F32], ids=["f64", "f32"])
def test_ou_td_aux_blocking_loop_device_equals_oracle(prec, with_a):
    """OU (scan kernels, multi-segment blocks, P_last laws) with time-dependent auxiliary laws
    on half the segments: device == oracle bit for bit through set_obs!, the filter, loglikhd!,
    draws with caller and device normals, accept and recompute_path!."""
    case, (dev, ora), ids = _td_pair(L.MAP_AUTO, prec, with_a=with_a, model=cs.ou_ragged_model())
    rng = np.random.default_rng(8)
    for ad, ao in _ou_loop([dev, ora], ids, dev.S, 4, rng):
        assert np.array_equal(ad, ao)
    for kind in (L.LAW_PP, L.LAW_PPB):
        for a_, b_ in zip(dev.download_law(L.U, kind), ora.download_law(L.U, kind)):
            assert np.array_equal(a_, b_), kind
    cs.assert_paths_equal(dev, ora)
    for ad, ao in _ou_loop([dev, ora], ids, dev.S, 2, rng, device_rng=True):
        assert np.array_equal(ad, ao)
    for lid, nb in ids:
        cs.assert_ll_equal(dev, ora, lid, nb)
        for e in (dev, ora):
            e.recompute_path(lid, 0, nb)
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, lid, nb)
    dev.close()


@pytest.mark.gpu
def test_ou_td_aux_mcmc_run_device_equals_oracle():
    """dmt_mcmc_run on an OU ensemble with time-dependent auxiliary laws (by default the
    per-iteration scan + accept kernels — DESIGN.md §7, the round-4 fault of the persistent TD
    kernel; the register-resident kernels are not eligible while a table is present): fetch_ll
    results, paths, ll and histories equal the oracle's, bit for bit."""
    case, (dev, ora), ids = _td_pair(L.MAP_AUTO, L.F64, model=cs.ou_ragged_model(), hist_len=7)
    lid, nb = ids[0]
    for e in (dev, ora):
        e.loglikhd(lid, L.U, 0, nb)
    assert np.array_equal(dev.mcmc_run(lid, 0, nb, 1, 6, salt=7), ora.mcmc_run(lid, 0, nb, 1, 6, salt=7))
    cs.assert_paths_equal(dev, ora)
    for what in (L.BLK_LL, L.BLK_LLPROP):
        assert np.array_equal(dev.get_block_state(lid, what, 0, nb), ora.get_block_state(lid, what, 0, nb))
    for what in (L.BLK_ACC_HIST, L.BLK_LL_HIST, L.BLK_LLPROP_HIST):
        assert np.array_equal(dev.get_block_state(lid, what, 0, nb, 7),
                              ora.get_block_state(lid, what, 0, nb, 7))
    dev.close()


def test_oracle_varying_table_enters_girsanov_and_filter():
    """The table is what the flagged segments use: with the guiding tables left as uploaded,
    loglikhd! (G only) already differs from the constant table's, and so do the guiding tables
    recompute_guiding_term! builds."""
    case, (var,), ids = _td_pair(None, L.F64, vary=True, oracle_only=True)
    _, (con,), _ = _td_pair(None, L.F64, vary=False, oracle_only=True)
    lid, nb = ids[0]
    for e in (var, con):
        e.loglikhd(lid, L.U, 0, nb)
    assert not np.array_equal(var.get_block_state(lid, L.BLK_LL, 0, nb),
                              con.get_block_state(lid, L.BLK_LL, 0, nb))
    for e in (var, con):
        e.recompute_guiding_term(lid, 0, nb, unit=L.U)
    Hv, Hc = var.download_law(L.U, L.LAW_PP)[0], con.download_law(L.U, L.LAW_PP)[0]
    assert not np.array_equal(Hv, Hc)


# ------------------------------------------------------------------ reference-form constructors
def _tutorial_aux(kind):
    """aux_laws of the reference-form SamplingPair: per segment, the FHN law linearised at the
    segment's observation (FitzHughNagumoAux) — as a fixed LinearAux ("fixed"), as the same
    constant given as functions of t ("const"), or with a time-varying perturbation ("vary")."""
    from diffusionmcmctools_amd import models as M

    class Aux:
        def __new__(cls, P, obs):
            lin = P.aux_for(obs)
            B0, b0 = np.array(lin.Bt, dtype=np.float64), np.array(lin.beta, dtype=np.float64)
            if kind == "fixed":
                return M.LinearAux(B0, b0, lin.sigma_t)
            if kind == "const":
                return M.TimeDependentLinearAux(lambda t: B0, lambda t: b0, lin.sigma_t)
            E = np.array([[0.0, 0.3], [0.2, 0.0]])
            return M.TimeDependentLinearAux(lambda t: B0 + np.sin(40.0 * t) * E,
                                            lambda t: b0 + np.array([0.2 * np.cos(30.0 * t), 0.0]),
                                            lin.sigma_t)
    return Aux


def _tutorial_run(kind, backend, n=6):
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import reference_tutorials as T
    from diffusionmcmctools_amd.api import engine_override

    def fac(model, n_points, prec, seed):
        return orc.OracleEnsemble(model.kind, model.d, model.m, n_points, prec=prec, seed=seed)

    T.Random_seed(100)
    rec = T.preamble_recordings()
    run = lambda: T.simple_inference_biblock(_tutorial_aux(kind), rec, 0.001, {"γ": 1.5},  # noqa: E731
                                             ϵ=0.3, ρ=0.96, num_steps=n)
    if backend == "oracle":
        with engine_override(fac):
            return run()
    return run()


def test_reference_form_td_aux_constant_equals_fixed_law():
    """SamplingPair(aux_laws, recording, tts) with time-dependent laws that are constant in t
    runs the biblock inference tutorial exactly as the same fixed LinearAux laws (oracle)."""
    a = _tutorial_run("const", "oracle")
    b = _tutorial_run("fixed", "oracle")
    np.testing.assert_array_equal([t[0] for t in a[1]], [t[0] for t in b[1]])
    np.testing.assert_array_equal(a[2]["a_h"], b[2]["a_h"])
    assert a[2]["bb"].ll == b[2]["bb"].ll
    c = _tutorial_run("vary", "oracle")
    assert c[2]["bb"].ll != a[2]["bb"].ll


@pytest.mark.gpu
def test_reference_form_td_aux_tutorial_device_equals_oracle():
    """The biblock inference tutorial with time-varying auxiliary laws given to the
    reference-form constructor: device == oracle (γ chain, decisions, ll, accepted paths)."""
    d = _tutorial_run("vary", "device", n=8)
    o = _tutorial_run("vary", "oracle", n=8)
    np.testing.assert_array_equal([t[0] for t in d[1]], [t[0] for t in o[1]])
    np.testing.assert_array_equal(d[2]["a_h"], o[2]["a_h"])
    assert d[2]["bb"].ll == o[2]["bb"].ll
    np.testing.assert_array_equal(np.concatenate(d[2]["sp"].u.XX), np.concatenate(o[2]["sp"].u.XX))
    d[2]["sp"].close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_iter", [6, 25])
def test_ou_td_aux_persistent_equals_per_iteration(n_iter):
    """The round-4 fault's shape (gpurun_out/r04g/pytest.log:31): one multi-iteration
    dmt_mcmc_run launch of k_mcmc_scan<…, TD> (opt-in, DMT_MCMC_SCAN_TD=1) against the default
    per-iteration scan + accept kernels on the same ensemble — every iteration's per-block ll°
    (the first wrong one was the third, profiles/r05a) and decisions, the fetch_ll results and
    the paths, bit for bit."""
    ens = []
    for env in ({"DMT_MCMC_SCAN_TD": "1"}, {"DMT_MCMC_SCAN_TD": "0"}):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            _, (dev,), ids = _td_pair_dev_only(n_iter + 1)
        finally:
            for k, v in saved.items():
                os.environ.pop(k) if v is None else os.environ.__setitem__(k, v)
        ens.append(dev)
    lid, nb = ids[0]
    for e in ens:
        e.loglikhd(lid, L.U, 0, nb)
    r = [e.mcmc_run(lid, 0, nb, 1, n_iter, salt=7) for e in ens]
    assert np.array_equal(r[0], r[1])
    for what in (L.BLK_LLPROP_HIST, L.BLK_ACC_HIST, L.BLK_LL_HIST):
        assert np.array_equal(ens[0].get_block_state(lid, what, 0, nb, n_iter + 1),
                              ens[1].get_block_state(lid, what, 0, nb, n_iter + 1))
    cs.assert_paths_equal(ens[0], ens[1])
    for e in ens:
        e.close()


def _td_pair_dev_only(hist_len):
    """The device ensemble of _td_pair (ragged OU, varying tables on every other segment)."""
    case, (dev, _), ids = _td_pair(L.MAP_AUTO, L.F64, model=cs.ou_ragged_model(),
                                   hist_len=hist_len)
    return case, (dev,), ids



@pytest.mark.gpu
def test_auxtd2_needs_the_a_columns():
    """a law record with DMT_LAW_AUXTD = 2 (ã(t) from the table) and a table given
    with only the B̃, β̃ columns is refused — at the table upload, at the law upload, and at the
    first draw when no table was given at all — instead of running with ã(t) = 0."""
    case = cs.ragged_case(model=cs.ou_ragged_model())
    m = case["model"]
    nb_cols = m.d * m.d + m.d
    G = int(sum(case["nsegs"]))

    def fresh():
        e = dmt.Ensemble(m.kind, m.d, m.m, case["n_points"], precision=L.F64, seed=11)
        cs.load_ragged(e, case)
        e.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
        return e
    e = fresh()
    _flag_segments(e, (L.LAW_PP,), np.arange(0, G, 2), 2.0)
    with pytest.raises(dmt.DMTError):
        e.upload_aux(L.LAW_PP, np.zeros((e.P, nb_cols)))
    e.close()
    e = fresh()
    e.upload_aux(L.LAW_PP, np.zeros((e.P, nb_cols)))
    with pytest.raises(dmt.DMTError):
        _flag_segments(e, (L.LAW_PP,), np.arange(0, G, 2), 2.0)
    e.close()
    e = fresh()
    _flag_segments(e, (L.LAW_PP,), np.arange(0, G, 2), 2.0)
    lay = e.create_layout([2, 3, 2], [0, 2, 0, 2, 4, 0, 3], [1, 3, 1, 3, 5, 2, 4],
                          [0, 1, 0, 0, 1, 0, 1], np.full(7, 0.5), 2)
    with pytest.raises(dmt.DMTError):
        e.draw_proposal(lay, 0, 7, iter=1, salt=3)
    e.close()
