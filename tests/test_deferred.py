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


def _ensembles(defer_values, B=96, N=300, hist=12, with_oracle=True, service=None):
    """One device ensemble per DMT_DEFER value (DMT_SERVICE: `service`, one per ensemble, or
    the library's default), then the oracle's."""
    import oracle as orc
    w = W.c2_ou2d(B=B, N=N)
    w.meta["hist_len"] = hist
    out = []
    for k, dv in enumerate(defer_values):
        env = {"DMT_DEFER": dv}
        if service is not None:
            env["DMT_SERVICE"] = service[k]
        saved = {n: os.environ.get(n) for n in env}
        os.environ.update(env)
        try:
            e = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                             grid_shared=w.grid_shared)
        finally:
            for n, v in saved.items():
                if v is None:
                    os.environ.pop(n)
                else:
                    os.environ[n] = v
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


# ------------------------------------------------------------------ the resident service
@pytest.mark.gpu
def test_service_equals_fused_launches_and_oracle():
    """DMT_SERVICE=1 (iterations posted to one resident launch) vs DMT_SERVICE=0 (one fused
    launch per iteration) vs DMT_DEFER=0 vs the oracle: every fetch_ll value, path, flag and
    history bit-identical, over more iterations than one auto-key Exp(1) row (64)."""
    (svc, fused, imm, ora), lay, nb = _ensembles(["1", "1", "0"], hist=80,
                                                 service=["1", "0", "0"])
    r = [_loop(e, lay, nb, 70, _nothing) for e in (svc, fused, imm, ora)]
    for k in (1, 2, 3):
        assert np.array_equal(r[0], r[k]), k
    for e in (fused, imm, ora):
        _same_state(svc, e, lay, nb, 80)
    for e in (svc, fused, imm):
        e.close()


def _loop_gaps(e, lay, nb, iters, fetch_every, sleep_at=(), sleep_s=0.0):
    import time
    e.loglikhd(lay, L.U, 0, nb)
    res = []
    for i in range(1, iters + 1):
        e.draw_proposal(lay, 0, nb, salt=L.RNG_AUTO, want_success="lazy")
        if i in sleep_at:
            time.sleep(sleep_s)      # longer than the launch's idle window (2 ms)
        e.accept_reject(lay, 0, nb, i, salt=L.RNG_AUTO)
        if i % fetch_every == 0:
            res.append(e.fetch_ll(lay, 0, nb, i))
    res.append(e.fetch_ll(lay, 0, nb, 0))
    return np.array(res)


@pytest.mark.gpu
def test_service_unfetched_iterations_and_idle_relaunch():
    """Iterations posted without their fetch_ll in between (the launch's one row set is reused:
    the host waits for the previous tree before posting) and host pauses longer than the
    launch's idle window (the launch leaves; the waiter launches it again from the first
    iteration it did not run): same results as one launch per call."""
    (svc, imm, ora), lay, nb = _ensembles(["1", "0"], hist=40, service=["1", "0"])
    kw = dict(fetch_every=3, sleep_at=(5, 6, 17), sleep_s=0.05)
    r = [_loop_gaps(e, lay, nb, 30, **kw) for e in (svc, imm, ora)]
    assert np.array_equal(r[0], r[1])
    assert np.array_equal(r[0], r[2])
    _same_state(svc, imm, lay, nb, 40)
    _same_state(svc, ora, lay, nb, 40)
    assert np.array_equal(svc.draw_success(lay, 0, nb), imm.draw_success(lay, 0, nb))
    for e in (svc, imm):
        e.close()


@pytest.mark.gpu
def test_service_explicit_keys_ranges_and_capacity():
    """Explicit keys, a change of range in the middle (the service stops and a new one starts),
    a sub-range, and a run to the end of the history (the launch's capacity): same results."""
    (svc, imm, ora), lay, nb = _ensembles(["1", "0"], hist=24, service=["1", "0"])
    h = nb // 2
    out = []
    for e in (svc, imm, ora):
        e.loglikhd(lay, L.U, 0, nb)
        res = []
        for i in range(1, 25):
            b0, b1 = (0, nb) if i <= 10 or i > 16 else (0, h)
            e.draw_proposal(lay, b0, b1, iter=i, salt=7)
            e.accept_reject(lay, b0, b1, i, salt=7)
            res.append(e.fetch_ll(lay, b0, b1, i))
        out.append(np.array(res))
    assert np.array_equal(out[0], out[1])
    assert np.array_equal(out[0], out[2])
    _same_state(svc, imm, lay, nb, 24)
    _same_state(svc, ora, lay, nb, 24)
    for e in (svc, imm):
        e.close()


@pytest.mark.gpu
def test_two_services_on_one_device_interleaved():
    """Two handles on one device, their caller loops interleaved call by call: each resident
    service waits for the device while the other holds it (its launch leaves idle and is
    launched again), and every result equals the one-launch-per-iteration path's."""
    (a, b, a0, b0), lay, nb = _ensembles(["1", "1", "0", "0"], hist=12, with_oracle=False,
                                         service=["1", "1", "0", "0"])
    for e in (a, b, a0, b0):
        e.loglikhd(lay, L.U, 0, nb)
    res = {id(e): [] for e in (a, b, a0, b0)}
    for i in range(1, 6):
        for e in (a, b, a0, b0):
            e.draw_proposal(lay, 0, nb, salt=L.RNG_AUTO, want_success="lazy")
            e.accept_reject(lay, 0, nb, i, salt=L.RNG_AUTO)
            res[id(e)].append(e.fetch_ll(lay, 0, nb, i))
    assert res[id(a)] == res[id(a0)] and res[id(b)] == res[id(b0)]
    _same_state(a, a0, lay, nb, 12)
    _same_state(b, b0, lay, nb, 12)
    for e in (a, b, a0, b0):
        e.close()


@pytest.mark.gpu
def test_service_switch_from_the_api_and_self_disable():
    """dmt_set_service: off (enable 0, or an idle window of 0) runs one fused launch per
    iteration and starts no service; a window so short that every launch leaves before its
    iteration is posted makes the service turn itself off after 16 posts (more than one relaunch
    per four posts: the fallback for a grid that other work keeps from being co-resident).
    Every result equals the default service's and the oracle's."""
    (svc, off, idle0, short, ora), lay, nb = _ensembles(["1", "1", "1", "1"], hist=40,
                                                        service=["1", "1", "1", "1"])
    off.set_service(False)
    idle0.set_service(True, 0.0)
    short.set_service(True, 0.001)
    r = [_loop_gaps(e, lay, nb, 30, fetch_every=1) for e in (svc, off, idle0, ora)]
    # the host away 0.5 ms before every post: each launch has left (1 µs window) by then
    r.insert(3, _loop_gaps(short, lay, nb, 30, fetch_every=1, sleep_at=range(1, 31),
                           sleep_s=0.0005))
    for k in range(1, 5):
        assert np.array_equal(r[0], r[k]), k
    for e in (off, idle0, short, ora):
        _same_state(svc, e, lay, nb, 40)
    assert svc.service_stats()["starts"] >= 1 and svc.service_stats()["off"] == 0
    assert off.service_stats()["starts"] == 0 and idle0.service_stats()["starts"] == 0
    st = short.service_stats()
    assert st["off"] == 1 and st["posts"] < 30, st
    # re-enabled from the API, the service starts again (the self-disable rule counts from the
    # enable): iterations 31-40 without host pauses, equal to the default service's
    short.set_service(True, 2.0)
    r2 = [_loop_from(e, lay, nb, 31, 10) for e in (svc, short)]
    assert np.array_equal(r2[0], r2[1])
    _same_state(svc, short, lay, nb, 40)
    st2 = short.service_stats()
    assert st2["off"] == 0 and st2["starts"] > st["starts"] and st2["posts"] > st["posts"], (st, st2)
    with pytest.raises(Exception):
        svc.set_service(True, -1.0)
    for e in (svc, off, idle0, short):
        e.close()


def _loop_from(e, lay, nb, i0, iters):
    """_loop_gaps continued: iterations i0 … i0 + iters - 1, each fetched, no pauses."""
    res = []
    for i in range(i0, i0 + iters):
        e.draw_proposal(lay, 0, nb, salt=L.RNG_AUTO, want_success="lazy")
        e.accept_reject(lay, 0, nb, i, salt=L.RNG_AUTO)
        res.append(e.fetch_ll(lay, 0, nb, i))
    return np.array(res)
