"""The drop-in boundary for unchanged reference callers (VERDICT r1 "next" item 3).

* Draws without a key come from the handle's stream counter (DMT_RNG_AUTO), as the reference's
  come from the global RNG (src/biblock.jl:94-99,122): the smoothing loop of
  docs/src/tutorials/biblock/smoothing.md:40-44, written verbatim (no iteration argument), gets
  fresh normals every call, an accept takes the Exp(1) variables of the draw it follows, and
  blockings drawn in one iteration get independent streams.
* ``recompute_guiding_term()`` recomputes b and b° (src/biblock.jl:288-291,
  src/block_collection.jl:208-210); ``Val(:P_only)`` / ``Val(:P°_only)`` are ``only=`` flags
  (src/block_collection.jl:212-221).
* The reference's constructors ``BiBlock(sp, range, ρ, last, ll_hist_len)`` and
  ``BlockCollection(sp, ranges, ρρ, ll_hist_len)`` (src/biblock.jl:48-62,
  src/block_collection.jl:22-30).

CPU tests run the API over the oracle backend (``_engine`` seam); the GPU tests require the
device to produce the oracle's chain bit for bit under the same counter-keyed streams."""
from __future__ import annotations

import numpy as np
import pytest

import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L
from diffusionmcmctools_amd import workloads as W
import oracle as orc

from _cases import ragged_case
from test_api import RANGES_A, RANGES_B, _sampling_ensemble


def _ou_se(backend, B=48, N=120, seed=21):
    """A C2-shaped 2-D OU BlockEnsemble (single-segment terminal blocks, shared H)."""
    w = W.c2_ou2d(B=B, N=N)
    if backend == "oracle":
        eng = orc.OracleEnsemble(w.model.kind, w.d, w.m, w.n_points, prec=w.precision, seed=seed,
                                 grid_shared=w.grid_shared)
        se = dmt.SamplingEnsemble(w.model, w.n_points, _engine=eng)
    else:
        se = dmt.SamplingEnsemble(w.model, w.n_points, precision=w.precision, seed=seed,
                                  grid_shared=w.grid_shared)
    se.upload_grid(w.t)
    se.set_guiding(w.H, w.F, w.laws, H_shared=w.H_shared)
    e = se.ens
    se.init_paths(w.X0[e.pt_off[e.rec_seg0[:-1]]])
    return se, w


def _smoothing_loop(se, n, rho=0.9):
    """docs/src/tutorials/biblock/smoothing.md:34-44 at BlockEnsemble level, verbatim."""
    be = dmt.BlockEnsemble(se, [[range(0, len(r))] for r in se.n_points], rho=rho,
                           ll_hist_len=n)
    be.loglikhd()                                    # loglikhd!(bb)
    W_prop, acc = [], []
    for i in range(1, n + 1):
        be.draw_proposal_path()                      # draw_proposal_path!(bb)
        W_prop.append(se.ens.download_paths(L.UPROP, 1).copy())
        acc.append(be.accept_reject_proposal_path(i))  # accept_reject_proposal_path!(bb, i)
    return be, W_prop, acc


def test_unkeyed_draws_are_fresh_on_host():
    se, w = _ou_se("oracle", B=8, N=40)
    eng = se.ens
    c0 = eng.rng_counter()
    be, W_prop, acc = _smoothing_loop(se, 4, rho=0.0)
    # ρ = 0: every proposal is a fresh draw; unkeyed calls never repeat normals
    for a in range(4):
        for b in range(a + 1, 4):
            assert not np.array_equal(W_prop[a], W_prop[b])
    # one counter value per iteration: the accept takes its draw's key
    assert eng.rng_counter() == c0 + 4


def test_accept_takes_the_key_of_its_draw_on_host():
    se, w = _ou_se("oracle", B=8, N=40)
    eng = se.ens
    be = dmt.BlockEnsemble(se, [[range(0, 1)]] * 8, rho=0.5, ll_hist_len=4)
    be.loglikhd()
    k = eng.rng_counter()
    be.draw_proposal_path()
    llp, ll = be.ll_prop.copy(), be.ll.copy()
    acc = be.accept_reject_proposal_path(1)
    it, salt = orc.auto_key(k)
    E = orc.exp1_range(eng.seed, 0, 8, it, salt)
    np.testing.assert_array_equal(acc, E > -(llp - ll))
    # an accept with no unkeyed draw before it takes a fresh key
    be.accept_reject_proposal_path(2)
    assert eng.rng_counter() == k + 2


def test_two_blockings_get_independent_streams_on_host():
    case = ragged_case()
    se = _sampling_ensemble(case, "oracle")
    beA = dmt.BlockEnsemble(se, RANGES_A, rho=0.0, ll_hist_len=2)
    beB = dmt.BlockEnsemble(se, RANGES_B, rho=0.0, ll_hist_len=2)
    for be in (beA, beB):
        be.loglikhd()
    k = se.ens.rng_counter()
    beA.draw_proposal_path()
    WA = se.ens.download_paths(L.UPROP, 1).copy()
    beA.accept_reject_proposal_path(1)
    beB.draw_proposal_path()
    WB = se.ens.download_paths(L.UPROP, 1).copy()
    beB.accept_reject_proposal_path(1)
    assert se.ens.rng_counter() == k + 2
    # segment 0 of recording 0 starts a block in both blockings: different normals
    assert not np.array_equal(WA[1:40], WB[1:40])


def test_mcmc_run_unkeyed_equals_unkeyed_loop_on_host():
    out = []
    for fused in (False, True):
        se, w = _ou_se("oracle", B=6, N=30)
        be = dmt.BlockEnsemble(se, [[range(0, 1)]] * 6, rho=0.8, ll_hist_len=5)
        be.loglikhd()
        if fused:
            r = be.mcmc_run(1, 5)
        else:
            r = []
            for i in range(1, 6):
                be.draw_proposal_path()
                be.accept_reject_proposal_path(i)
                r.append(be._ens.fetch_ll(be._layout, 0, 6, i))
            r = np.array(r, dtype=np.float64)
        out.append((np.asarray(r), se.ens.download_paths(L.U, 0), se.ens.rng_counter()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2]


def test_explicit_salt_limit():
    se, w = _ou_se("oracle", B=4, N=20)
    be = dmt.BlockEnsemble(se, [[range(0, 1)]] * 4, rho=0.5, ll_hist_len=2)
    with pytest.raises(ValueError):
        be.draw_proposal_path(iter=1, salt=L.SALT_LIMIT)


def _corrupt_and_recompute(se, be, only):
    """Overwrite both units' PP guiding tables with garbage, recompute, return which unit's
    tables came back to the filter's values."""
    e = se.ens
    ref = {u: e.download_law(u, L.LAW_PP) for u in (L.U, L.UPROP)}
    for u in (L.U, L.UPROP):
        H, F, laws = ref[u]
        e.upload_law(u, L.LAW_PP, H=np.full_like(H, 7.0), F=np.full_like(F, -3.0), laws=laws)
    be.recompute_guiding_term() if only is None else be.recompute_guiding_term(only=only)
    got = {u: e.download_law(u, L.LAW_PP) for u in (L.U, L.UPROP)}
    return {u: bool(np.array_equal(got[u][0], ref[u][0]) and np.array_equal(got[u][1], ref[u][1]))
            for u in (L.U, L.UPROP)}


def _filter_ready(backend):
    case = ragged_case()
    se = _sampling_ensemble(case, backend)
    se.set_observations(case["Hobs"], case["Fobs"], case["cobs"])
    # terminal blocks over whole recordings: every segment's guiding term is its PP table
    be = dmt.BlockEnsemble(se, [[range(0, len(r))] for r in se.n_points], rho=0.5,
                           ll_hist_len=2)
    be.recompute_guiding_term()          # tables = the filter's values for both units
    return se, be


@pytest.mark.parametrize("only,want", [(None, (True, True)), ("P_only", (True, False)),
                                       ("P°_only", (False, True))])
def test_recompute_guiding_term_units_on_host(only, want):
    se, be = _filter_ready("oracle")
    fixed = _corrupt_and_recompute(se, be, only)
    assert (fixed[L.U], fixed[L.UPROP]) == want
    with pytest.raises(ValueError):
        be.recompute_guiding_term(only="P_everything")


def test_reference_constructors_on_host():
    case = ragged_case()
    se = _sampling_ensemble(case, "oracle")
    sp = se.recordings[1]
    bb = dmt.BiBlock(sp, range(2, 6), 0.6, True, 3)
    assert bb.is_last and bb.rho == 0.6 and bb.segments == range(2, 6) and bb.num_blocks == 1
    bc = dmt.BlockCollection(sp, [range(0, 2), range(2, 4), range(4, 6)], [0.1, 0.2, 0.3], 4)
    assert [b.is_last for b in bc.blocks] == [False, False, True]
    assert [b.rho for b in bc.blocks] == [0.1, 0.2, 0.3]
    with pytest.raises(ValueError):
        dmt.BiBlock(sp, range(0, 1), 0.5, False, 2)       # non-terminal needs >= 2 segments
    # both run the reference loop on their own layouts, views into the same pair
    for x in (bb, bc):
        x.loglikhd()
        x.draw_proposal_path()
        x.accept_reject_proposal_path(1)
        assert np.all(np.isfinite(x.ll))
    be = dmt.BlockEnsemble(se, RANGES_A, rho=0.5, ll_hist_len=[2, 5, 3])
    assert be.ll_hist_len == 5


@pytest.mark.gpu
def test_smoothing_loop_unkeyed_device_equals_oracle():
    """The smoothing loop written as the reference writes it: identical chains on the device
    and the oracle (paths, decisions, ll histories), fresh normals on every call."""
    n = 8
    res = []
    for backend in ("gpu", "oracle"):
        se, w = _ou_se(backend)
        be, W_prop, acc = _smoothing_loop(se, n)
        res.append((W_prop, acc, be.ll_history.copy(), be.ll_prop_history.copy(),
                    se.ens.download_paths(L.U, 0), se.ens.rng_counter()))
        if backend == "gpu":
            assert not any(np.array_equal(W_prop[0], x) for x in W_prop[1:])
            se.close()
    (Wd, ad, hd, hpd, Xd, cd), (Wo, ao, ho, hpo, Xo, co) = res
    for a, b in zip(Wd, Wo):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(np.array(ad), np.array(ao))
    np.testing.assert_array_equal(hd, ho)
    np.testing.assert_array_equal(hpd, hpo)
    np.testing.assert_array_equal(Xd, Xo)
    assert cd == co


@pytest.mark.gpu
def test_blocking_unkeyed_device_equals_oracle():
    """Two blockings per iteration, unkeyed (smoothing_with_blocking.md): device == oracle."""
    case = ragged_case()
    res = []
    for backend in ("gpu", "oracle"):
        se = _sampling_ensemble(case, backend)
        beA = dmt.BlockEnsemble(se, RANGES_A, rho=0.7, ll_hist_len=4)
        beB = dmt.BlockEnsemble(se, RANGES_B, rho=0.4, ll_hist_len=4)
        accs = []
        for i in range(1, 5):
            for be in (beA, beB):
                be.loglikhd()
                be.draw_proposal_path()
                accs.append(be.accept_reject_proposal_path(i))
        res.append((accs, se.ens.download_paths(L.U, 0), beA.ll_history, beB.ll_history))
    for a, b in zip(res[0][0], res[1][0]):
        np.testing.assert_array_equal(a, b)
    for x, y in zip(res[0][1:], res[1][1:]):
        np.testing.assert_array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["ou", "fhn"])
def test_mcmc_run_unkeyed_device(kind):
    """dmt_mcmc_run with DMT_RNG_AUTO (persistent kernel for OU, per-iteration kernels for FHN)
    == the loop of unkeyed draw + accept calls on the device == the oracle's run."""
    n = 6
    out = []
    for mode in ("run", "loop", "oracle"):
        if kind == "ou":
            se, w = _ou_se("oracle" if mode == "oracle" else "gpu", B=40, N=100)
            ranges = [[range(0, 1)]] * 40
        else:
            se = _sampling_ensemble(ragged_case(), "oracle" if mode == "oracle" else "gpu")
            ranges = RANGES_A
        be = dmt.BlockEnsemble(se, ranges, rho=0.8, ll_hist_len=n)
        be.loglikhd()
        se.ens.set_rng_counter(5)
        if mode == "loop":
            r = []
            for i in range(1, n + 1):
                be.draw_proposal_path()
                be.accept_reject_proposal_path(i)
                r.append(be._ens.fetch_ll(be._layout, 0, be.num_blocks, i))
            r = np.array(r, dtype=np.float64)
        else:
            r = be.mcmc_run(1, n)
        out.append((np.asarray(r), se.ens.download_paths(L.U, 0), se.ens.download_paths(L.U, 1),
                    be.accpt_history, se.ens.rng_counter()))
    for x in out[1:]:
        for a, b in zip(out[0], x):
            np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


@pytest.mark.gpu
@pytest.mark.parametrize("only,want", [(None, (True, True)), ("P_only", (True, False)),
                                       ("P°_only", (False, True))])
def test_recompute_guiding_term_units_device(only, want):
    se, be = _filter_ready("gpu")
    fixed = _corrupt_and_recompute(se, be, only)
    assert (fixed[L.U], fixed[L.UPROP]) == want
    se.close()
