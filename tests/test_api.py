"""The host mirror of the reference interface (diffusionmcmctools.jl_amd/api.py).

CPU tests drive the API's host logic (range bookkeeping, BiBlock/BlockCollection/BlockEnsemble
dispatch, ll_of_accepted / accpt_rate / fetch_ll semantics) over the oracle backend through the
``_engine`` test seam; the GPU test runs the same reference-style MCMC program through libdmt and
through the oracle and requires bit-identical results."""
from __future__ import annotations

import math

import numpy as np
import pytest

import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L
import oracle as orc

from _cases import ragged_case

RANGES_A = [[range(0, 2), range(2, 4)],
            [range(0, 2), range(2, 4), range(4, 6)],
            [range(0, 3), range(3, 5)]]
RANGES_B = [[range(0, 4)], [range(0, 3), range(3, 6)], [range(0, 2), range(2, 5)]]


def _sampling_ensemble(case, backend, seed=11):
    m = case["model"]
    if backend == "oracle":
        eng = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=case["prec"], seed=seed)
        se = dmt.SamplingEnsemble(m, case["n_points"], _engine=eng)
    else:
        se = dmt.SamplingEnsemble(m, case["n_points"], precision=case["prec"], seed=seed)
    se.upload_grid(case["t"])
    se.set_guiding(case["H"], case["F"], case["laws"], Hb=case["Hb"], Fb=case["Fb"],
                   lawsb=case["lawsb"])
    X0 = case["X0"]
    e = se.ens
    x0 = X0[e.pt_off[e.rec_seg0[:-1]]]
    se.init_paths(x0, Z=case["Z0"], iter=0, salt=1)
    return se


def _program(se, niter=6, seed=3):
    """The reference's smoothing-with-blocking loop (docs/src/tutorials/biblock/
    smoothing_with_blocking.md:60-75): alternate two blockings; per iteration draw, MH decide,
    record fetch_ll.  Parity-mode draws (Z, E supplied)."""
    rng = np.random.default_rng(seed)
    e = se.ens
    beA = dmt.BlockEnsemble(se, RANGES_A, rho=0.7, ll_hist_len=niter)
    beB = dmt.BlockEnsemble(se, RANGES_B, rho=[0.3, [0.2, 0.5], 0.4], ll_hist_len=niter)
    out = []
    for be in (beA, beB):
        be.loglikhd()
    for i in range(1, niter + 1):
        be = beA if i % 2 else beB
        Z = rng.standard_normal((e.S, 1))
        E = rng.exponential(1.0, be.num_blocks)
        ok = be.draw_proposal_path(Z=Z)
        acc = be.accept_reject_proposal_path(i, E=E)
        out.append((ok, acc, be.fetch_ll(), be.fetch_ll_prop(),
                    [c.fetch_ll() for c in be.recordings], be.ll.copy(), be.ll_prop.copy()))
        # one BiBlock-level step on the first block of recording 1
        bb = be.recordings[1].blocks[0]
        Zb = rng.standard_normal((e.S, 1))
        bb.draw_proposal_path(Z=Zb, iter=100 + i)
        bb.loglikhd_prop()
        out.append((bb.fetch_ll(), bb.fetch_ll_prop()))
    # parameter steps (docs/src/tutorials/pnames/inference_with_biblock.md:17-25): re-solve
    # u° with u's W (recompute_path!), then the parameter MH decision, once accepted (E = 0
    # accepts unless ll° = −Inf) and once rejected (E = 50)
    for E in (0.0, 50.0):
        beB.recompute_path()
        acc, th = beB.accept_reject_proposal_param(niter, [1.5], [1.7], E=E)
        out.append((acc, th, beB.fetch_ll(), beB.fetch_ll_prop(), beB.ll.copy()))
    beA.set_ll(2, -7.5)
    beA.recordings[1].blocks[2].set_ll(3, 1.25, unit=L.UPROP)
    out.append((beA.ll_history.copy(), beA.ll_prop_history.copy()))
    return beA, beB, out


def test_block_ensemble_structure():
    case = ragged_case()
    se = _sampling_ensemble(case, "oracle")
    be = dmt.BlockEnsemble(se, RANGES_A, rho=0.7, ll_hist_len=4)
    assert be.num_recordings() == 3
    assert [len(c.blocks) for c in be.recordings] == [2, 3, 2]
    assert be.num_blocks == 7
    lasts = [[b.is_last for b in c.blocks] for c in be.recordings]
    assert lasts == [[False, True], [False, False, True], [False, True]]
    assert be.recordings[2].blocks[0].segments == range(0, 3)
    assert all(b.rho == 0.7 for c in be.recordings for b in c.blocks)
    assert be.ll.shape == (7,) and np.all(be.ll == -math.inf)  # src/block.jl:75


@pytest.mark.parametrize("bad", [
    [[range(0, 2), range(3, 4)], [range(0, 6)], [range(0, 5)]],   # gap
    [[range(0, 4)], [range(0, 5)], [range(0, 5)]],                # short
    [[range(0, 4)], [range(0, 6)]],                               # missing recording
])
def test_block_ensemble_rejects_bad_ranges(bad):
    case = ragged_case()
    se = _sampling_ensemble(case, "oracle")
    with pytest.raises(ValueError):
        dmt.BlockEnsemble(se, bad)


def test_mcmc_semantics_on_host():
    """ll_of_accepted / accpt_rate / histories / fetch_ll follow the reference definitions."""
    case = ragged_case()
    se = _sampling_ensemble(case, "oracle")
    beA, beB, out = _program(se, niter=6)
    for be in (beA, beB):
        llh, llph, acch = be.ll_history, be.ll_prop_history, be.accpt_history
        for i in range(1, 7):
            if not acch[i - 1].any() and not (llh[i - 1] != 0).any():
                continue  # this blocking was not used at iteration i
            got = be.ll_of_accepted(i)
            want = np.where(acch[i - 1], llph[i - 1], llh[i - 1])
            np.testing.assert_array_equal(np.concatenate(got), want)
        rate = np.concatenate(be.accpt_rate(range(1, 7)))
        np.testing.assert_array_equal(rate, acch.sum(0) / 6)
    ok, acc, f, fp, per_rec, ll, llp = out[0]
    assert ok.all() and 0 < acc.sum() < acc.size
    # fetch_ll of the ensemble is the pairwise tree over its blocks; per recording likewise
    np.testing.assert_equal(f, orc.pairwise_tree(list(ll)))
    np.testing.assert_equal(per_rec[1], orc.pairwise_tree(list(ll[2:5])))
    assert math.isfinite(f) and math.isfinite(fp)
    # BiBlock fetch_ll is its own ll
    b = beA.recordings[0].blocks[1]
    assert b.fetch_ll() == beA.ll[1]


def test_accept_order_matches_reference():
    """accept_reject_proposal_path!: save_ll! records PRE-swap values (src/biblock.jl:121-127)."""
    case = ragged_case()
    se = _sampling_ensemble(case, "oracle")
    be = dmt.BlockEnsemble(se, RANGES_A, rho=0.5, ll_hist_len=3)
    be.loglikhd()
    rng = np.random.default_rng(0)
    for i in (1, 2):
        be.draw_proposal_path(Z=rng.standard_normal((se.ens.S, 1)))
        ll0, llp0 = be.ll.copy(), be.ll_prop.copy()
        E = rng.exponential(1.0, be.num_blocks)
        acc = be.accept_reject_proposal_path(i, E=E)
        np.testing.assert_array_equal(acc, E > -(llp0 - ll0))
        np.testing.assert_array_equal(be.ll_history[i - 1], ll0)
        np.testing.assert_array_equal(be.ll_prop_history[i - 1], llp0)
        np.testing.assert_array_equal(be.ll, np.where(acc, llp0, ll0))
        np.testing.assert_array_equal(be.ll_prop, np.where(acc, ll0, llp0))


def test_param_step_and_set_ll_on_host():
    """accept_reject_proposal_param follows the tutorial helper (swap_XX!, swap_PP!, save_ll!
    of both blocks, swap_ll! on acceptance; decision E > −(Σll° − Σll)); set_ll! writes one
    history entry of b or b°."""
    case = ragged_case()
    se = _sampling_ensemble(case, "oracle")
    be = dmt.BlockEnsemble(se, RANGES_B, rho=0.5, ll_hist_len=3)
    be.loglikhd()
    be.draw_proposal_path(Z=np.random.default_rng(2).standard_normal((se.ens.S, 1)))
    be.loglikhd_prop()
    ll, llp = be.fetch_ll(), be.fetch_ll_prop()
    X_p = [a.copy() for a in se.recordings[0].u_prop.XX]
    lb, lbp = be.ll.copy(), be.ll_prop.copy()
    E = max(0.0, -(llp - ll)) + 1.0          # forces acceptance
    acc, th = be.accept_reject_proposal_param(1, [1.5], [1.7], E=E)
    assert acc and th.tolist() == [1.7]
    for a, b in zip(se.recordings[0].u.XX, X_p):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(be.ll, lbp)
    np.testing.assert_array_equal(be.ll_history[0], lb)   # save_ll! before swap_ll!
    np.testing.assert_array_equal(be.ll_prop_history[0], lbp)
    acc, th = be.accept_reject_proposal_param(2, [1.5], [1.7], E=-math.inf)
    assert not acc and th.tolist() == [1.5]
    be.set_ll(3, 2.5)
    be.recordings[1].blocks[0].set_ll(3, -1.0, unit=L.UPROP)
    assert np.all(be.ll_history[2] == 2.5)
    assert np.ravel(be.recordings[1].blocks[0].ll_prop_history)[2] == -1.0
    assert np.ravel(be.recordings[1].blocks[1].ll_prop_history)[2] != -1.0


def test_init_paths_retries_failed_recordings():
    """init_paths! repeats forward_guide! until it succeeds (src/sampling_unit.jl:83-87): a
    recording whose draw fails is drawn again with the next normal stream (and a new start
    point from x0_prior), the others are left alone."""
    case = ragged_case()
    m = case["model"]
    eng = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=case["prec"], seed=11)
    calls = []

    class Flaky:  # fails recording 1's first two draws
        def __getattr__(self, k):
            return getattr(eng, k)

        def draw_unit(self, unit, r0=0, r1=None, Z=None, iter=0, salt=0):
            r1 = eng.R if r1 is None else r1
            ll, ok = eng.draw_unit(unit, r0, r1, Z=Z, iter=iter, salt=salt)
            calls.append((r0, r1, iter))
            ok = np.array(ok)
            if r0 <= 1 < r1 and sum(1 for c in calls if c[0] <= 1 < c[1]) <= 2:
                ok[1 - r0] = False
            return ll, ok

    se = dmt.SamplingEnsemble(m, case["n_points"], _engine=Flaky())
    se.upload_grid(case["t"])
    se.set_guiding(case["H"], case["F"], case["laws"], Hb=case["Hb"], Fb=case["Fb"],
                   lawsb=case["lawsb"])
    starts = eng.pt_off[eng.rec_seg0[:-1]]
    x0 = case["X0"][starts]
    new_x0 = np.array([0.25, -0.5])
    ll, ok = se.init_paths(x0, iter=5, x0_prior=lambda k: new_x0)
    assert ok.all()
    assert calls == [(0, 3, 5), (1, 2, 6), (1, 2, 7)]
    X = eng.download_paths(L.U, 0)
    np.testing.assert_array_equal(X[starts[1]], new_x0)
    np.testing.assert_array_equal(X[starts[0]], x0[0])
    np.testing.assert_array_equal(eng.download_paths(L.UPROP, 0), X)
    with pytest.raises(RuntimeError):
        calls.clear()
        se.init_paths(x0, iter=5, max_tries=2)


def test_swaps_and_set_accepted():
    case = ragged_case()
    se = _sampling_ensemble(case, "oracle")
    be = dmt.BlockEnsemble(se, RANGES_B, rho=0.5, ll_hist_len=2)
    be.loglikhd()
    be.draw_proposal_path(Z=np.random.default_rng(1).standard_normal((se.ens.S, 1)))
    X_u = se.recordings[1].u.XX
    X_p = se.recordings[1].u_prop.XX
    coll = be.recordings[1]
    coll.swap_XX()
    for a, b in zip(se.recordings[1].u.XX, X_p):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(se.recordings[1].u_prop.XX, X_u):
        np.testing.assert_array_equal(a, b)
    coll.swap_XX()
    ll, llp = coll.ll.copy(), coll.ll_prop.copy()
    coll.swap_ll()
    np.testing.assert_array_equal(coll.ll, llp)
    np.testing.assert_array_equal(coll.ll_prop, ll)
    coll.blocks[1].set_accepted(2, True)
    assert coll.blocks[1].accpt_history[1] and not coll.blocks[0].accpt_history[1]


@pytest.mark.gpu
def test_api_program_gpu_matches_oracle():
    case = ragged_case()
    se_d = _sampling_ensemble(case, "gpu")
    se_o = _sampling_ensemble(case, "oracle")
    beA_d, beB_d, out_d = _program(se_d)
    beA_o, beB_o, out_o = _program(se_o)
    for a, b in zip(out_d, out_o):
        for x, y in zip(a, b):
            if isinstance(x, list):
                for xx, yy in zip(x, y):
                    np.testing.assert_array_equal(np.asarray(xx), np.asarray(yy))
            else:
                np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    for r in range(3):
        for unit in ("u", "u_prop"):
            for a, b in zip(getattr(se_d.recordings[r], unit).XX,
                            getattr(se_o.recordings[r], unit).XX):
                np.testing.assert_array_equal(a, b)
            for a, b in zip(getattr(se_d.recordings[r], unit).WW,
                            getattr(se_o.recordings[r], unit).WW):
                np.testing.assert_array_equal(a, b)
    for bd, bo in ((beA_d, beA_o), (beB_d, beB_o)):
        np.testing.assert_array_equal(bd.ll_history, bo.ll_history)
        np.testing.assert_array_equal(bd.accpt_history, bo.accpt_history)
    se_d.close()


def test_equalize_obs_params_is_a_no_op_on_shared_observations():
    """GP.equalize_obs_params!(bb) (src/biblock.jl:375-387): the observations live once per
    recording for u and u° (dmt_upload_obs), so the call changes nothing and reports no
    critical change; the blocks' ll and paths are untouched."""
    se = _sampling_ensemble(ragged_case(), "oracle")
    be = dmt.BlockEnsemble(se, RANGES_A, rho=0.5, ll_hist_len=2)
    be.loglikhd()
    ll0 = be.ll.copy() if hasattr(be.ll, "copy") else be.ll
    X0 = se.ens.download_paths(L.U, 0).copy()
    crit = be.equalize_obs_params()
    assert crit.dtype == bool and crit.shape == (be.num_blocks,) and not crit.any()
    assert np.array_equal(se.ens.download_paths(L.U, 0), X0)
    assert np.array_equal(be.ll, ll0)


def test_from_recordings_builds_the_reference_containers():
    """SamplingEnsemble.from_recordings(model, recordings, tts) — the reference's
    SamplingEnsemble(aux_laws, recordings, tts; artificial_noise) (src/sampling_unit.jl:55-74):
    laws linearised at each observation, guiding terms through the recording's segments,
    blocking laws with the artificial end observation, observations uploaded, init_paths! —
    equal to the tables built by hand from the same pieces (models.guiding_chain)."""
    from diffusionmcmctools_amd.models import (FHN, Observation, Recording, guiding_chain,
                                               setup_time_grids)
    model = FHN(0.1, -0.8, 1.5, 0.0, 0.3)
    recs = [Recording(obs=[Observation(0.1 * (k + 1), np.array([y]), np.array([[1.0, 0.0]]),
                                       np.array([[0.01]])) for k, y in enumerate(ys)],
                      t0=0.0, x0=np.array([-0.9, -1.0]))
            for ys in ([-0.5, 0.2, 0.9], [0.1, -0.3])]
    tts = [setup_time_grids(r, 0.01) for r in recs]

    def engine(n_points):
        return orc.OracleEnsemble(model.kind, model.d, model.m, n_points, prec=L.F64, seed=3)
    se = dmt.SamplingEnsemble.from_recordings(model, recs, tts, artificial_noise=1e-11,
                                              _engine=engine)
    assert se.n_points == [[len(g) for g in t] for t in tts]
    H, F, laws = se.ens.download_law(L.U, L.LAW_PP)
    for r, rec in enumerate(recs):
        auxes = [model.aux(ob.v[0]) for ob in rec.obs]
        chain = guiding_chain(auxes, tts[r], [ob.info() for ob in rec.obs])
        g0 = sum(len(x) for x in recs[:r] for x in [x.obs])
        p0 = sum(len(g) for t in tts[:r] for g in t)
        for k, (h, f, c) in enumerate(chain):
            n = len(tts[r][k])
            assert np.array_equal(H[p0:p0 + n], h) and np.array_equal(F[p0:p0 + n], f)
            assert np.array_equal(laws[g0 + k], model.law_record(auxes[k], c[0]))
            p0 += n
    Hb, Fb, lawsb = se.ens.download_law(L.U, L.LAW_PPB)
    assert np.all(np.isfinite(Hb)) and Hb.max() > 1e10   # the 1e-11 artificial observation
    X = se.ens.download_paths(L.U, 0)
    assert np.all(np.isfinite(X))
    be = dmt.BlockEnsemble(se, [[range(0, 3)], [range(0, 2)]], rho=0.5, ll_hist_len=2)
    be.loglikhd()
    assert np.isfinite(be.fetch_ll())
