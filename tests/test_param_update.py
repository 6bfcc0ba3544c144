"""set_proposal_law!(bb, θ°, pnames) on the device (SURVEY.md §8(f) rank 3;
src/biblock.jl:334-364): law-record parameter writes with the auxiliary law re-derived,
recompute_guiding_term!(b°) for critical changes, recompute_path!(b°, b.WW).

CPU: the oracle's derivation reproduces the host set-up's law records bit for bit, and the
oracle's set_proposal_law! reproduces the host set-up (records, guiding tables, c(t0)) of the
same case built with θ°.  GPU: device == oracle bit for bit in a parameter-MH loop over the
ragged blocking layouts, and for a non-critical OU drift update."""
from __future__ import annotations

import numpy as np
import pytest

import _cases as cs
import oracle as orc
from diffusionmcmctools_amd import _lib as L
from diffusionmcmctools_amd import workloads as W
from diffusionmcmctools_amd.models import FHN, Lorenz

THETA0 = (0.1, -0.8, 1.5, 0.0, 0.3)
THETA1 = (0.12, -0.7, 1.4, 0.1, 0.35)


def _fhn_params(th):
    return {L.PAR_FHN[k]: v for k, v in zip(("eps", "s", "gamma", "beta", "sigma"), th)}


@pytest.mark.parametrize("y", [-1.1, 0.0, 0.37, 0.9])
def test_fhn_derivation_matches_host_records(y):
    m0, m1 = FHN(*THETA0), FHN(*THETA1)
    rec = m0.law_record(m0.aux(y), 1.5)
    orc.set_law_params(L.MODEL_FHN, 2, rec, _fhn_params(THETA1))
    ref = m1.law_record(m1.aux(y), 1.5)
    assert np.array_equal(rec.view(np.uint64), ref.view(np.uint64))


def test_fhn_partial_update_keeps_other_parameters():
    m0 = FHN(*THETA0)
    rec = m0.law_record(m0.aux(0.4))
    orc.set_law_params(L.MODEL_FHN, 2, rec, {L.PAR_FHN["gamma"]: 1.7})
    m1 = FHN(0.1, -0.8, 1.7, 0.0, 0.3)
    assert np.array_equal(rec, m1.law_record(m1.aux(0.4)))


def test_lorenz_derivation_matches_host_records():
    v = np.array([1.5, -2.0, 20.0])
    m0, m1 = Lorenz(10.0, 28.0, 8.0 / 3.0), Lorenz(9.5, 27.0, 2.5)
    rec = m0.law_record(m0.aux(v))
    orc.set_law_params(L.MODEL_LORENZ, 3, rec, {0: 9.5, 1: 27.0, 2: 2.5})
    assert np.array_equal(rec, m1.law_record(m1.aux(v)))


def _whole_recording_layout(e, case):
    R = len(case["nsegs"])
    return e.create_layout([1] * R, [0] * R, [k - 1 for k in case["nsegs"]], [1] * R,
                           [0.5] * R, 0), R


def test_oracle_set_proposal_law_reproduces_host_setup():
    """After set_proposal_law!(θ°) on whole-recording blocks, u°'s PP laws and tables equal the
    host set-up of the same recordings built with θ° (models.py records + dmt_guiding_linear
    chain), and u's are untouched."""
    case0 = cs.ragged_case()
    case1 = cs.ragged_case(model=FHN(*THETA1))
    m = case0["model"]
    ora = orc.OracleEnsemble(m.kind, m.d, m.m, case0["n_points"], prec=case0["prec"], seed=1)
    cs.load_ragged(ora, case0)
    ora.upload_obs(case0["Hobs"], case0["Fobs"], case0["cobs"])
    lay, R = _whole_recording_layout(ora, case0)
    ok, crit = ora.set_proposal_law(lay, 0, R, _fhn_params(THETA1))
    assert crit.all() and ok.all()
    H, F, laws = ora.download_law(L.UPROP, L.LAW_PP)
    assert np.array_equal(laws, case1["laws"])
    assert np.array_equal(H, case1["H"]) and np.array_equal(F, case1["F"])
    H0, F0, laws0 = ora.download_law(L.U, L.LAW_PP)
    assert np.array_equal(laws0, case0["laws"]) and np.array_equal(H0, case0["H"])


def test_oracle_unchanged_theta_is_not_critical():
    case = cs.ragged_case()
    m = case["model"]
    ora = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=case["prec"], seed=1)
    cs.load_ragged(ora, case)
    lay, R = _whole_recording_layout(ora, case)
    ok, crit = ora.set_proposal_law(lay, 0, R, _fhn_params(THETA0))
    assert not crit.any() and ok.all()
    # s alone moves β̃ (critical); the OU-style "target only" case is covered on the GPU
    ora.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    ok, crit = ora.set_proposal_law(lay, 0, R, {L.PAR_FHN["s"]: -0.75})
    assert crit.all()


def test_oracle_critical_change_false_keeps_the_guiding_term():
    """critical_change = false (src/biblock.jl:340-342): with u°'s law equal to u's, a θ° that
    moves the auxiliary law still leaves u°'s guiding term (H, F, c(t0)) as it was — only the
    records and the path change; after a swap made u°'s law differ from u's, the equalization
    alone makes the update critical again (:361-362)."""
    case = cs.ragged_case()
    m = case["model"]
    ora = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=case["prec"], seed=1)
    cs.load_ragged(ora, case)
    ora.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    lay, R = _whole_recording_layout(ora, case)
    H0, F0, laws0 = ora.download_law(L.UPROP, L.LAW_PP)
    ok, crit = ora.set_proposal_law(lay, 0, R, _fhn_params(THETA1), critical_change=False)
    assert ok.all() and not crit.any()
    H1, F1, laws1 = ora.download_law(L.UPROP, L.LAW_PP)
    assert np.array_equal(H1, H0) and np.array_equal(F1, F0)
    assert not np.array_equal(laws1, laws0)  # θ° written, the auxiliary law re-derived
    ok, crit = ora.set_proposal_law(lay, 0, R, _fhn_params(THETA1), critical_change=True)
    assert crit.all()
    ora.swap(lay, L.SWAP_PP, 0, R)  # u° now holds THETA0's law, u THETA1's
    ok, crit = ora.set_proposal_law(lay, 0, R, _fhn_params(THETA1), critical_change=False)
    assert crit.all()


def test_oracle_false_then_default_recomputes_the_stale_guiding_term():
    """critical_change = false leaves u°'s guiding term stale where θ° moved the
    auxiliary law; a later call with the default and an unchanged θ° must still treat those
    blocks as critical (DMT_LAW_GSTALE), after which u°'s guiding term is the one a `true` call
    gives — and the bit is clear again."""
    case = cs.ragged_case()
    m = case["model"]
    made = []
    for seq in ((False, None), (True,)):
        ora = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=case["prec"], seed=1)
        cs.load_ragged(ora, case)
        ora.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
        lay, R = _whole_recording_layout(ora, case)
        for k, cc in enumerate(seq):
            ok, crit = ora.set_proposal_law(lay, 0, R, _fhn_params(THETA1), critical_change=cc)
            if seq[0] is False:
                laws = ora.download_law(L.UPROP, L.LAW_PP)[2]
                if k == 0:
                    assert not crit.any() and (laws[:, L.LAW_GSTALE] == 1.0).any()
                else:
                    assert crit.all() and (laws[:, L.LAW_GSTALE] == 0.0).all()
        made.append([ora.download_law(L.UPROP, kind) for kind in (L.LAW_PP, L.LAW_PPB)])
    for a_, b_ in zip(made[0], made[1]):
        for x, y in zip(a_, b_):
            assert np.array_equal(x, y)


def test_updt_obs_is_refused():
    """Observation parameters (updt_obs) are not device state: a ParamNamesBlock that would
    update them raises instead of being silently ignored."""
    from diffusionmcmctools_amd import functions as fn
    unit = {"updt": ((1, "γ"),), "updt_aux": [((1, "γ"),)], "updt_obs": [((2, 1),)]}
    empty = {"updt": (), "updt_aux": [], "updt_obs": []}
    pn = {"PP": unit, "P_last": empty, "P_excl": empty, "Pb_excl": empty}
    with pytest.raises(NotImplementedError):
        fn._pairs(pn)
    pn["PP"] = dict(unit, updt_obs=[()])
    assert list(fn._pairs(pn).values()) == [1]
    assert fn._flags(False, 3) == [False] * 3
    assert fn._flags([[True, False], [True]], 3) == [True, False, True]
    with pytest.raises(ValueError):
        fn._flags([True], 2)


def test_api_set_proposal_law_by_name():
    """BlockEnsemble.set_proposal_law(theta={name: value}) maps DD parameter names and runs the
    device operation (here through the oracle seam)."""
    import diffusionmcmctools_amd as dmt
    from test_api import RANGES_A, _sampling_ensemble
    case = cs.ragged_case()
    se = _sampling_ensemble(case, "oracle")
    se.ens.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    be = dmt.BlockEnsemble(se, RANGES_A, rho=0.5, ll_hist_len=2)
    be.loglikhd()
    ok, crit = be.set_proposal_law(theta={"eps": 0.11, "sigma": 0.31})
    assert ok.all() and crit.all()
    with pytest.raises(KeyError):
        be.set_proposal_law(theta={"theta": 1.0})


# ------------------------------------------------------------------------------------ GPU
MAPPINGS = [pytest.param(L.MAP_LANE, id="lane"), pytest.param(L.MAP_WAVE, id="wave")]


@pytest.mark.gpu
@pytest.mark.parametrize("mapping", MAPPINGS)
def test_parameter_mh_loop_bit_exact(mapping):
    """Parameter Metropolis–Hastings over the ragged blocking layouts
    (accept_reject_proposal_param!, docs/src/tutorials/block_ensemble/inference.md:61-67):
    set_proposal_law!(θ°) → decide on fetch_ll° − fetch_ll → swap_XX! + swap_PP! + swap_ll! on
    acceptance; device == oracle bit for bit (laws, tables, paths, ll, critical flags)."""
    case, dev, ora, ids = cs.ragged_pair(mapping=mapping, hist_len=4)
    for e in (dev, ora):
        e.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    rng = np.random.default_rng(21)
    th = np.array(THETA0)
    for i in range(6):
        lid, nb = ids[i % 2]
        for e in (dev, ora):
            e.set_obs(lid, 0, nb)
            e.recompute_guiding_term(lid, 0, nb, unit=L.U)
            e.loglikhd(lid, L.U, 0, nb)
        prop = th.copy()
        which = [0, 1, 2, 4, 3, 0][i]  # every parameter, ϵ twice
        prop[which] += 0.02 * rng.standard_normal()
        okd, crd = dev.set_proposal_law(lid, 0, nb, _fhn_params(prop))
        oko, cro = ora.set_proposal_law(lid, 0, nb, _fhn_params(prop))
        assert np.array_equal(okd, oko) and np.array_equal(crd, cro), f"iteration {i}"
        assert cro.all()
        for unit in (L.U, L.UPROP):
            for kind in (L.LAW_PP, L.LAW_PPB):
                for a_, b_ in zip(dev.download_law(unit, kind), ora.download_law(unit, kind)):
                    assert np.array_equal(a_, b_), f"iteration {i}, unit {unit}, kind {kind}"
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, lid, nb)
        lld = ora.block_ll(lid, 0, nb)
        dll = lld[1].sum() - lld[0].sum()
        if np.log(rng.uniform()) < dll:  # accept θ° for all blocks
            th = prop
            for e in (dev, ora):
                e.swap(lid, L.SWAP_XX | L.SWAP_PP | L.SWAP_LL, 0, nb)
        cs.assert_paths_equal(dev, ora)


@pytest.mark.gpu
@pytest.mark.parametrize("mapping", MAPPINGS)
def test_critical_change_false_bit_exact(mapping):
    """set_proposal_law!(bb, θ°, pnames, false): device == oracle bit for bit — u°'s guiding
    term kept where only θ° moved the auxiliary law, recomputed where the equalization with u's
    law changed it (after a parameter swap)."""
    case, dev, ora, ids = cs.ragged_pair(mapping=mapping, hist_len=4)
    for e in (dev, ora):
        e.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    lid, nb = ids[0]
    for e in (dev, ora):
        e.recompute_guiding_term(lid, 0, nb, unit=L.U)
        e.loglikhd(lid, L.U, 0, nb)
    # False, then the default with θ° unchanged (the stale-guiding-term bit), True,
    # a parameter swap, False again
    for step, cc in enumerate((False, None, True, "swap", False)):
        if cc == "swap":
            for e in (dev, ora):
                e.swap(lid, L.SWAP_XX | L.SWAP_PP | L.SWAP_LL, 0, nb)
            continue
        th = THETA1 if step < 3 else THETA0
        okd, crd = dev.set_proposal_law(lid, 0, nb, _fhn_params(th), critical_change=cc)
        oko, cro = ora.set_proposal_law(lid, 0, nb, _fhn_params(th), critical_change=cc)
        assert np.array_equal(okd, oko) and np.array_equal(crd, cro), step
        for kind in (L.LAW_PP, L.LAW_PPB):
            for a_, b_ in zip(dev.download_law(L.UPROP, kind), ora.download_law(L.UPROP, kind)):
                assert np.array_equal(a_, b_), (step, kind)
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, lid, nb)


@pytest.mark.gpu
def test_ou_drift_update_is_not_critical():
    """OU: Θ, μ changes leave the (fixed) auxiliary law and the guiding term alone; only the
    path is re-solved — device == oracle bit for bit."""
    w = W.c1_ou1d()
    dev, ora, lay = cs.both(w)
    nb = w.nblocks
    for e in (dev, ora):
        e.loglikhd(lay, L.U, 0, nb)
    okd, crd = dev.set_proposal_law(lay, 0, nb, {0: 1.3, 1: 0.1})
    oko, cro = ora.set_proposal_law(lay, 0, nb, {0: 1.3, 1: 0.1})
    assert not crd.any() and not cro.any()
    assert np.array_equal(okd, oko)
    cs.assert_paths_equal(dev, ora)
    cs.assert_ll_equal(dev, ora, lay, nb)
    for a_, b_ in zip(dev.download_law(L.UPROP, L.LAW_PP), ora.download_law(L.UPROP, L.LAW_PP)):
        assert np.array_equal(a_, b_)
