"""The reference's "Inference with BiBlocks" tutorial end to end
(docs/src/tutorials/biblock/inference.md:42-75 on the preamble.md:52-66 dataset, driven by
examples/fhn_gamma_inference.py): path imputation and the γ random-walk update through
set_proposal_law! / accept_reject_proposal_param! on one terminal BiBlock over 100 segments.

CPU: the loop runs on the oracle backend.  GPU: the device chain equals the oracle's bit for
bit over the first iterations (paths, γ chain, decisions, ll), and a longer device chain
covers the true γ = 1.5 within its 5–95 % range.  The dataset is a fresh simulation (Julia's
seeded stream is not reproducible), so the chain is not comparable with the reference's
published one (docs/src/assets/tutorials/biblock/inference_chain.png) and is not checked
against it."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples"))

import fhn_gamma_inference as tut  # noqa: E402


@pytest.fixture(scope="module")
def recording():
    rec, X, t = tut.tutorial_data()
    return rec


def test_tutorial_data_shape(recording):
    assert len(recording.obs) == 100
    assert [o.t for o in recording.obs[:2]] == [0.1, 0.2] and recording.obs[-1].t == 10.0
    v = np.array([o.v[0] for o in recording.obs])
    assert np.all(np.abs(v) < 2.5)          # the FHN relaxation oscillation stays within ±2


def test_tutorial_loop_on_oracle(recording):
    se = tut.sampling_pair(recording, 1.5, backend="oracle")
    assert sum(se.n_points[0]) == 100 * 101
    res = tut.simple_inference(se, 1.5, num_steps=20, snapshot_every=0)
    assert res["gamma"].shape == (21,) and np.all(np.isfinite(res["ll"]))
    assert 0 < res["accepted_path"].sum() < 20       # ρ = 0.96: most pCN moves accepted
    assert res["accepted_param"].any()
    moved = np.diff(res["gamma"]) != 0
    np.testing.assert_array_equal(moved, res["accepted_param"])
    bb = res["block"]
    hist = bb.ll_history[:, 0]
    assert hist.shape == (20,) and np.all(np.isfinite(hist))


@pytest.mark.gpu
def test_tutorial_device_equals_oracle(recording):
    """25 iterations of simple_inference on the device and on the oracle from the same state and
    seeds: identical γ chains, decisions, fetch_ll values and accepted paths."""
    n = 25
    out = []
    for backend in ("device", "oracle"):
        se = tut.sampling_pair(recording, 1.5, backend=backend)
        res = tut.simple_inference(se, 1.5, num_steps=n, snapshot_every=0)
        X = se.ens.download_paths(0, 0)
        out.append((res, X))
        if backend == "device":
            se.close()
    (rd, Xd), (ro, Xo) = out
    np.testing.assert_array_equal(rd["gamma"], ro["gamma"])
    np.testing.assert_array_equal(rd["accepted_path"], ro["accepted_path"])
    np.testing.assert_array_equal(rd["accepted_param"], ro["accepted_param"])
    np.testing.assert_array_equal(rd["ll"], ro["ll"])
    np.testing.assert_array_equal(Xd, Xo)


@pytest.mark.gpu
def test_tutorial_gamma_posterior_on_device(recording):
    """3000 iterations (the reference runs 10⁴): after 500 burn-in the γ chain sits around the
    true value, both update kinds mix, and the 400-iteration path snapshots are recorded."""
    se = tut.sampling_pair(recording, 1.5, backend="device")
    res = tut.simple_inference(se, 1.5, num_steps=3000, snapshot_every=400)
    s = tut.summarize(res, 500)
    assert 1.2 < s["gamma_mean"] < 1.9, s
    assert s["gamma_q05"] < 1.5 < s["gamma_q95"] + 0.2, s
    assert 0.2 < s["path_accept_rate"] < 0.95, s
    assert 0.1 < s["param_accept_rate"] < 0.95, s
    snap, it = se.snapshot(6)
    assert it == 2800 and len(snap[0]) == 100 and snap[0][0].shape == (101, 2)
    np.testing.assert_array_equal(snap[0][0][0], tut.Y1)
    se.close()


# ------------------------------------------------------------------ inference with blocking
def test_set_obs_reanchors_blocking_law(recording):
    """set_obs! freezes the accepted end point of a non-terminal block as P_last's exact
    observation; the FHN auxiliary law of P_last (b and b°) is re-linearised at that end point
    (the host record of the same law built at y_T, bit for bit) so that b̃ = b there."""
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import _lib as L
    from diffusionmcmctools_amd.models import FHN
    se = tut.sampling_pair(recording, 1.5, backend="oracle", blocking=True)
    be = dmt.BlockEnsemble(se, [tut.BLOCKINGS[0]], rho=0.96, ll_hist_len=2)
    be.set_obs()
    X = se.ens.download_paths(L.U, 0)
    e = se.ens
    for g in (24, 74):
        y = X[e.pt_off[g] + e.npts[g] - 1]
        np.testing.assert_array_equal(e.obsv[g], y)
        m = FHN(*tut.THETA)
        want = m.law_record(m.aux(y[0]))
        for unit in (L.U, L.UPROP):
            rec = e.download_law(unit, L.LAW_PPB)[2][g]
            sl = np.r_[0:49, 50:64]            # all but c(t0)
            assert np.array_equal(rec[sl], want[sl]), (g, unit)


def test_set_obs_reanchoring_is_local_to_p_last(recording):
    """Localises the unpinned re-anchoring reading of set_obs! (GuidedProposals'
    set_obs! is not vendored): it rewrites only the P_last law records of the non-terminal
    blocks' last segments (b and b°).  Every PP record, H/F table and terminal block is untouched,
    so a reading without the re-anchoring can differ only in those blocks' guiding terms."""
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import _lib as L
    se = tut.sampling_pair(recording, 1.5, backend="oracle", blocking=True)
    be = dmt.BlockEnsemble(se, [tut.BLOCKINGS[0]], rho=0.96, ll_hist_len=2)
    e = se.ens
    kinds = (L.LAW_PP, L.LAW_PPB)
    before = {(u, k): [np.array(a, copy=True) for a in e.download_law(u, k)]
              for u in (L.U, L.UPROP) for k in kinds}
    be.set_obs()
    for (u, k), (H0, F0, R0) in before.items():
        H1, F1, R1 = e.download_law(u, k)
        assert np.array_equal(H1, H0) and np.array_equal(F1, F0), (u, k)
        changed = sorted(set(np.nonzero(np.any(R1 != R0, axis=1))[0].tolist()))
        assert changed == ([] if k == L.LAW_PP else [24, 74]), (u, k, changed)


def test_blocking_tutorial_loop_on_oracle(recording):
    se = tut.sampling_pair(recording, 1.5, backend="oracle", blocking=True)
    res = tut.simple_inference_with_blocking(se, 1.5, num_steps=6)
    assert res["accepted_path"].shape == (6, 5) and np.all(np.isfinite(res["ll"]))
    assert res["accepted_path"].mean() > 0.3      # every block moves (exact end points anchored)


@pytest.mark.gpu
def test_blocking_tutorial_device_equals_oracle(recording):
    """biblock/inference_with_blocking.md's loop (set_obs!, recompute_guiding_term!,
    find_W_for_X!, loglikhd!, draw, accept per blocking; γ update on the last blocking) for 8
    iterations: device == oracle bit for bit."""
    out = []
    for backend in ("device", "oracle"):
        se = tut.sampling_pair(recording, 1.5, backend=backend, blocking=True)
        res = tut.simple_inference_with_blocking(se, 1.5, num_steps=8)
        out.append((res, se.ens.download_paths(0, 0), se.ens.download_paths(0, 1)))
        if backend == "device":
            se.close()
    (rd, Xd, Wd), (ro, Xo, Wo) = out
    for k in ("gamma", "accepted_path", "accepted_param", "ll"):
        np.testing.assert_array_equal(rd[k], ro[k], err_msg=k)
    np.testing.assert_array_equal(Xd, Xo)
    np.testing.assert_array_equal(Wd, Wo)


# ------------------------------------------------------------------ BlockEnsemble (γ shared)
@pytest.fixture(scope="module")
def recordings2():
    recs, _, _ = tut.tutorial_data(num_recs=2)
    return recs


def test_ensemble_tutorial_loop_on_oracle(recordings2):
    """block_ensemble/inference.md: two recordings, one terminal block each, the ensemble-level
    draw / accept / set_proposal_law! / parameter decision on fetch_ll° − fetch_ll."""
    se = tut.sampling_pair(recordings2, 1.5, backend="oracle")
    assert se.num_recordings() == 2 and sum(map(sum, se.n_points)) == 2 * 100 * 101
    res = tut.simple_inference(se, 1.5, num_steps=8, snapshot_every=0)
    assert res["accepted_path"].shape == (8, 2) and np.all(np.isfinite(res["ll"]))
    np.testing.assert_array_equal(np.diff(res["gamma"]) != 0, res["accepted_param"])


@pytest.mark.gpu
def test_ensemble_tutorial_device_equals_oracle(recordings2):
    out = []
    for backend in ("device", "oracle"):
        se = tut.sampling_pair(recordings2, 1.5, backend=backend)
        res = tut.simple_inference(se, 1.5, num_steps=15, snapshot_every=0)
        out.append((res, se.ens.download_paths(0, 0)))
        if backend == "device":
            se.close()
    (rd, Xd), (ro, Xo) = out
    for k in ("gamma", "accepted_path", "accepted_param", "ll"):
        np.testing.assert_array_equal(rd[k], ro[k], err_msg=k)
    np.testing.assert_array_equal(Xd, Xo)
