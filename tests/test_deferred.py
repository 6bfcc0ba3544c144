"""Deferred draws (include/dmt.h): the unchanged caller's loop of separate calls —
``draw_proposal_path!(be); accept_reject_proposal_path!(be, i); fetch_ll(be)``
(docs/src/tutorials/biblock/smoothing.md:40-44) — runs as one fused launch per iteration on the
register-resident kernel, with results identical to launching every call at once
(DMT_DEFER=0) and to the oracle, whatever other call comes between the draw and its accept.
Also the checkpoint of the auto stream state between a draw and its accept (dmt_rng_state)."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import diffusionmcmctools_amd as dmt  # noqa: E402
from diffusionmcmctools_amd import _lib as L  # noqa: E402
from diffusionmcmctools_amd import workloads as W  # noqa: E402


def _ensembles(defer_values, B=96, N=300, hist=12, with_oracle=True):
    import oracle as orc
    w = W.c2_ou2d(B=B, N=N)
    w.meta["hist_len"] = hist
    out = []
    for dv in defer_values:
        saved = os.environ.get("DMT_DEFER")
        os.environ["DMT_DEFER"] = dv
        try:
            e = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                             grid_shared=w.grid_shared)
        finally:
            if saved is None:
                os.environ.pop("DMT_DEFER")
            else:
                os.environ["DMT_DEFER"] = saved
        out.append(e)
    if with_oracle:
        out.append(orc.OracleEnsemble(w.model.kind, w.d, w.m, w.n_points, prec=w.precision,
                                      seed=5, grid_shared=w.grid_shared))
    lays = [W.fill(e, w) for e in out]
    assert all(x == lays[0] for x in lays)
    return out, lays[0], B


def _loop(e, lay, nb, iters, interleave):
    """The caller's loop as the Python mirror issues it (every call separate, auto stream keys,
    the draw's flags left unread unless used); ``interleave(i, e, …)`` may call something
    between a draw and its accept."""
    e.loglikhd(lay, L.U, 0, nb)
    res = []
    for i in range(1, iters + 1):
        flags = e.draw_proposal(lay, 0, nb, salt=L.RNG_AUTO, want_success="lazy")
        interleave(i, e, lay, nb, flags)
        e.accept_reject(lay, 0, nb, i, salt=L.RNG_AUTO)
        res.append(e.fetch_ll(lay, 0, nb, i))
        res.append(e.fetch_ll(lay, 0, nb, 0))  # fetch_ll° after fetch_ll: the same tree
    return np.array(res)


def _same_state(a, b, lay, nb, hist):
    for unit in (L.U, L.UPROP):
        for what in (0, 1, 2):
            assert np.array_equal(a.download_paths(unit, what), b.download_paths(unit, what))
    for what in (L.BLK_LL, L.BLK_LLPROP):
        assert np.array_equal(a.get_block_state(lay, what, 0, nb), b.get_block_state(lay, what, 0, nb))
    for what in (L.BLK_ACC_HIST, L.BLK_LL_HIST, L.BLK_LLPROP_HIST):
        assert np.array_equal(a.get_block_state(lay, what, 0, nb, hist),
                              b.get_block_state(lay, what, 0, nb, hist))


def _nothing(i, e, lay, nb, flags):
    pass


def _mixed(i, e, lay, nb, flags):
    """Calls between a draw and its accept on some iterations: each must see the drawn
    proposal (the deferred draw is launched first)."""
    if i == 2:
        e.get_block_state(lay, L.BLK_LLPROP, 0, nb)
    elif i == 3:
        assert np.asarray(flags).all() and len(np.asarray(flags)) == nb
    elif i == 5:
        e.download_paths(L.UPROP, 0)


def test_oracle_rng_state_roundtrip():
    import oracle as orc
    w = W.c2_ou2d(B=8, N=20)
    e = orc.OracleEnsemble(w.model.kind, w.d, w.m, w.n_points, prec=w.precision, seed=1,
                           grid_shared=w.grid_shared)
    lay = W.fill(e, w)
    e.draw_proposal(lay, 0, 8, salt=L.RNG_AUTO)
    st = e.rng_state()
    assert st == (1, 0, True)
    e.set_rng_counter(9)
    assert e.rng_state() == (9, 0, False)
    e.set_rng_state(st)
    assert e.rng_state() == st


@pytest.mark.gpu
@pytest.mark.parametrize("interleave", [_nothing, _mixed], ids=["loop", "calls-between"])
def test_deferred_loop_equals_immediate_and_oracle(interleave):
    (dfr, imm, ora), lay, nb = _ensembles(["1", "0"])
    iters = 8
    r = [_loop(e, lay, nb, iters, interleave) for e in (dfr, imm, ora)]
    assert np.array_equal(r[0], r[1])
    assert np.array_equal(r[0], r[2])
    _same_state(dfr, imm, lay, nb, 12)
    _same_state(dfr, ora, lay, nb, 12)
    assert dfr.rng_counter() == imm.rng_counter() == ora.rng_counter()
    for e in (dfr, imm):
        e.close()


@pytest.mark.gpu
def test_deferred_explicit_keys_and_subranges():
    """Explicit keys (iter = mcmciter, one salt) fuse too; a sub-range accept after a
    whole-range draw, or a different key, takes the separate launches — same results."""
    (dfr, imm, ora), lay, nb = _ensembles(["1", "0"])
    for e in (dfr, imm, ora):
        e.loglikhd(lay, L.U, 0, nb)
    for i in range(1, 6):
        for e in (dfr, imm, ora):
            if i == 3:  # draw all, accept in two halves: no fusion
                e.draw_proposal(lay, 0, nb, iter=i, salt=4)
                e.accept_reject(lay, 0, nb // 2, i, salt=4)
                e.accept_reject(lay, nb // 2, nb, i, salt=4)
            elif i == 4:  # different keys for the draw and the decision
                e.draw_proposal(lay, 0, nb, iter=i, salt=4)
                e.accept_reject(lay, 0, nb, i, salt=6)
            else:
                e.draw_proposal(lay, 0, nb, iter=i, salt=4)
                e.accept_reject(lay, 0, nb, i, salt=4)
        f = [e.fetch_ll(lay, 0, nb, i) for e in (dfr, imm, ora)]
        assert f[0] == f[1] == f[2], (i, f)
    _same_state(dfr, imm, lay, nb, 12)
    _same_state(dfr, ora, lay, nb, 12)


@pytest.mark.gpu
def test_rng_state_checkpoint_between_draw_and_accept():
    """a checkpoint taken between an auto draw and its auto accept resumes bit for
    bit when the whole stream state (dmt_rng_state) is restored."""
    (a, b), lay, nb = _ensembles(["1", "1"], with_oracle=False)
    for e in (a, b):
        e.loglikhd(lay, L.U, 0, nb)
        e.draw_proposal(lay, 0, nb, salt=L.RNG_AUTO)
    st = b.rng_state()
    assert st[2] and st[0] == st[1] + 1
    b.set_rng_counter(12345)          # a counter-only restore loses the pending draw's key ...
    b.set_rng_state(st)               # ... the full state restores it
    acc = [e.accept_reject(lay, 0, nb, 1, salt=L.RNG_AUTO, want_acc=True) for e in (a, b)]
    assert np.array_equal(acc[0], acc[1])
    _same_state(a, b, lay, nb, 12)
