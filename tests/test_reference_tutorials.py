"""The reference's four tutorial loops, written with the reference's own constructors, field
accesses and call signatures (examples/reference_tutorials.py), run on the drop-in API.

CPU: each loop runs on the oracle backend (api.engine_override, test infrastructure) — the
caller code is the same object-for-object.  GPU: each loop runs on libdmt and on the oracle
from the same data and the same host random stream; the γ chains, the path and parameter
decisions, the log-likelihood histories and the final accepted paths are bit-identical.

  biblock/inference.md:11-101              simple_inference_biblock
  biblock/smoothing_with_blocking.md:11-62 simple_smoothing_with_blocking
  block_collection/inference.md:1-77       simple_inference_collection
  block_ensemble/inference.md:53-133       simple_inference_ensemble
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import reference_tutorials as T  # noqa: E402

import diffusionmcmctools_amd as dmt  # noqa: E402
from diffusionmcmctools_amd.api import engine_override  # noqa: E402
from diffusionmcmctools_amd.models import FHN  # noqa: E402

LAYOUT = [[range(0, 25), range(25, 75), range(75, 100)], [range(0, 50), range(50, 100)]]


def _oracle_factory(model, n_points, prec, seed):
    import oracle as orc
    return orc.OracleEnsemble(model.kind, model.d, model.m, n_points, prec=prec, seed=seed)


@pytest.fixture(autouse=True)
def _restore_var_names():
    saved = FHN.var_parameter_names
    yield
    FHN.var_parameter_names = saved


def _run(fn, backend):
    T.Random_seed(100)
    if backend == "oracle":
        with engine_override(_oracle_factory):
            return fn()
    return fn()


def _biblock(n):
    rec = T.preamble_recordings()
    return lambda: T.simple_inference_biblock(T.FitzHughNagumoAux, rec, 0.001, {"γ": 1.5},
                                              ϵ=0.3, ρ=0.96, num_steps=n)


def _smoothing(n):
    rec = T.preamble_recordings()
    return lambda: T.simple_smoothing_with_blocking(T.FitzHughNagumoAux, rec, 0.001,
                                                    T.FitzHughNagumoAux, LAYOUT, ρ=0.96,
                                                    num_steps=n)


def _collection(n):
    all_obs = T.collection_all_obs(T.preamble_recordings())
    return lambda: T.simple_inference_collection(T.FitzHughNagumoAux, all_obs, 0.001,
                                                 {"REC1_γ": 1.5}, ϵ=0.3, ρ=0.96, num_steps=n)


def _ensemble(n):
    all_obs = T.ensemble_all_obs(T.preamble_recordings(num_recs=2))
    return lambda: T.simple_inference_ensemble(T.FitzHughNagumoAux, all_obs, 0.001,
                                               {"γ_shared": 1.5}, ϵ=0.3, ρ=0.96, num_steps=n)


# ------------------------------------------------------------------ CPU: the loops run
def test_biblock_inference_loop():
    paths, θθ, st = _run(_biblock(6), "oracle")
    bb, sp = st["bb"], st["sp"]
    assert len(θθ) == 7 and paths == []
    np.testing.assert_array_equal(np.diff([t[0] for t in θθ]) != 0, st["a_h"])
    # the reference's field accesses
    assert np.isfinite(bb.b.ll) and np.isfinite(bb.b_prop.ll)
    assert bb.b.ll_history.shape == (6,)
    XX = sp.u.XX
    assert len(XX) == 100 and XX[0].shape == (101, 2)
    np.testing.assert_array_equal(bb.b.XX[5], XX[5])
    assert 0.0 <= dmt.accpt_rate(bb, range(1, 7)) <= 1.0
    assert np.isfinite(dmt.ll_of_accepted(bb, 6))


def test_smoothing_with_blocking_loop():
    paths, st = _run(_smoothing(3), "oracle")
    blocks = st["blocks"]
    assert [len(B) for B in blocks] == [3, 2]
    assert [bb.is_last for bb in blocks[0]] == [False, False, True]
    for B in blocks:
        for bb in B:
            assert np.isfinite(bb.b.ll)
            assert bb.ll_history.shape == (3, 1)
    # blocks of both layouts see one another's accepted paths (views onto one SamplingPair)
    np.testing.assert_array_equal(blocks[0][1].b.XX[0], blocks[1][0].b.XX[25])


def test_block_collection_inference_loop():
    paths, θθ, st = _run(_collection(5), "oracle")
    assert len(θθ) == 6
    np.testing.assert_array_equal(np.diff([t[0] for t in θθ]) != 0, st["a_h"])
    bc = st["bc"]
    assert np.isfinite(dmt.fetch_ll(bc)) and np.isfinite(dmt.fetch_ll_prop(bc))


def test_block_ensemble_inference_loop():
    paths, θθ, st = _run(_ensemble(4), "oracle")
    assert len(θθ) == 5
    be, se = st["be"], st["se"]
    assert se.num_recordings() == 2 and len(be.recordings) == 2
    # γ_shared reaches both recordings' laws: the device law records hold the chain's value
    from diffusionmcmctools_amd import _lib as L
    recs = se.ens.download_law(L.U, L.LAW_PP)[2]
    assert np.all(recs[:, L.LAW_THETA + 2] == θθ[-1][0])


def test_param_names_restatement():
    """ParamNamesBlock / ParamNamesRecording / ParamNamesAllObs as
    src/param_names_collections.jl builds them for the tutorials' set-ups."""
    all_obs = T.collection_all_obs(T.preamble_recordings())
    assert all_obs.param_depend_rev == [[("REC1_γ", "γ")]]
    with engine_override(_oracle_factory):
        rec = all_obs.recordings[0]
        tts = dmt.models.setup_time_grids(rec, 0.001)
        sp = dmt.SamplingPair(T.FitzHughNagumoAux, rec, tts)
        bc = dmt.BlockCollection(sp, [range(0, 40), range(40, 100)], 0.9, 2)
        pn = dmt.ParamNamesRecording(bc, ["REC1_γ"], all_obs.param_depend_rev[0],
                                     all_obs.obs_depend_rev[0])
    b0, b1 = pn.blocks
    # non-terminal block: PP over its first 39 laws, P_last / P_excl over the 40th
    assert len(b0.PP.updt_aux) == 39 and len(b0.P_last.updt_aux) == 1
    assert len(b0.P_excl.updt_obs) == 1 and len(b0.Pb_excl.updt_aux) == 39
    assert b0.PP.updt == ((1, "γ"),) and b0.PP.var == ()
    # terminal block: PP over all 60, no P_last
    assert len(b1.PP.updt_aux) == 60 and len(b1.P_last.updt_aux) == 0
    ens = T.ensemble_all_obs(T.preamble_recordings(num_recs=2))
    assert ens.param_depend_rev == [[("γ_shared", "γ")], [("γ_shared", "γ")]]


def test_block_view_ll_is_assignable():
    with engine_override(_oracle_factory):
        rec = T.preamble_recordings()
        sp = dmt.SamplingPair(T.FitzHughNagumoAux, rec, dmt.models.setup_time_grids(rec, 0.001))
        bb = dmt.BiBlock(sp, range(0, 100), 0.9, True, 3)
        dmt.loglikhd(bb)
        ll = bb.b.ll
        assert np.isfinite(ll) and bb.b_prop.ll == -np.inf
        bb.b_prop.ll = ll - 1.0
        assert bb.b_prop.ll == ll - 1.0
        dmt.save_ll(bb.b, 2)
        assert bb.b.ll_history[1] == ll
        # GP.loglikhd(u::SamplingUnit) of the accepted path = the block's ll (one terminal block)
        assert dmt.GP.loglikhd(sp.u) == ll


# ------------------------------------------------------------------ GPU: device == oracle
def _same(a, b, what):
    np.testing.assert_array_equal(np.asarray(a), np.asarray(b), err_msg=what)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n", [("biblock", 12), ("collection", 10), ("ensemble", 8)])
def test_inference_tutorial_device_equals_oracle(name, n):
    make = {"biblock": _biblock, "collection": _collection, "ensemble": _ensemble}[name]
    out = {}
    for backend in ("device", "oracle"):
        paths, θθ, st = _run(make(n), backend)
        x = st.get("bb") or st.get("bc") or st.get("be")
        sp_or_se = st.get("sp") or st.get("se")
        pairs = [sp_or_se] if name != "ensemble" else sp_or_se.recordings
        out[backend] = dict(theta=np.array([t[0] for t in θθ]), a_h=np.array(st["a_h"]),
                            ll=x.ll, llp=x.ll_prop, hist=x.ll_history, acc=x.accpt_history,
                            XX=[np.concatenate(p.u.XX) for p in pairs],
                            WW=[np.concatenate(p.u.WW) for p in pairs],
                            fetch=(dmt.fetch_ll(x), dmt.fetch_ll_prop(x)))
        if backend == "device":
            sp_or_se.close()
    d, o = out["device"], out["oracle"]
    for k in d:
        if k in ("XX", "WW"):
            for a, b in zip(d[k], o[k]):
                _same(a, b, k)
        else:
            _same(d[k], o[k], k)
    assert 0 < d["a_h"].sum() or n < 5


@pytest.mark.gpu
def test_smoothing_with_blocking_device_equals_oracle():
    out = {}
    for backend in ("device", "oracle"):
        paths, st = _run(_smoothing(6), backend)
        blocks = st["blocks"]
        out[backend] = dict(
            XX=np.concatenate(st["sp"].u.XX), WW=np.concatenate(st["sp"].u.WW),
            ll=[bb.b.ll for B in blocks for bb in B],
            hist=[bb.ll_history for B in blocks for bb in B],
            acc=[bb.accpt_history for B in blocks for bb in B])
        if backend == "device":
            st["sp"].close()
    for k in out["device"]:
        _same(out["device"][k], out["oracle"][k], k)
