"""Committed golden fixtures (tests/golden/, generator make_golden.py): the oracle (CPU) and
the HIP path (GPU, both mappings) must reproduce them bit for bit.  What each fixture pins is
stated in make_golden.py; none holds reference output (parity unpinned)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle as orc
from diffusionmcmctools_amd import _lib as L
from diffusionmcmctools_amd.models import OU, Observation, guiding_chain

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAPPINGS = [pytest.param(L.MAP_LANE, id="lane"), pytest.param(L.MAP_WAVE, id="wave")]


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


# ---------------------------------------------------------------- CPU
def test_philox_kat_fixture_oracle():
    g = load("philox_kat.npz")
    for ctr, key, out in zip(g["ctr"], g["key"], g["out"]):
        seed = int(key[0]) | (int(key[1]) << 32)
        np.testing.assert_array_equal(orc.philox_raw(seed, ctr)[0], out)


def test_ou1d_guiding_fixture_host_filter():
    """The exact discrete backward filter (dmt_guiding_linear, host-only) against the
    closed-form OU guiding term."""
    g = load("ou1d_guiding.npz")
    th, sg = float(g["theta"]), float(g["sigma"])
    model = OU([[th]], [0.0], [[sg]])
    aux = model.aux(Theta_t=[[th]])
    info = Observation(float(g["T"]), np.array([float(g["v"])]), np.eye(1),
                       float(g["Sigma"]) * np.eye(1)).info()
    (H, F, c), = guiding_chain([aux], [g["t"]], [info])
    np.testing.assert_allclose(H[:, 0], g["H"], rtol=1e-12)
    np.testing.assert_allclose(F[:, 0], g["F"], rtol=1e-12)
    np.testing.assert_allclose(c, g["c"], rtol=1e-12)


def _c1_ensemble(g, ens):
    ens.upload_grid(g["t"])
    ens.upload_law(L.U, L.LAW_PP, H=g["H"], F=g["F"], laws=g["laws"], H_shared=True)
    ens.set_paths(L.U, X=g["X0"])
    ens.draw_unit(L.U, Z=g["Z0"], iter=0, salt=0xFFFF)
    ens.set_paths(L.UPROP, X=ens.download_paths(L.U, 0), W=ens.download_paths(L.U, 1))
    iters = g["Zs"].shape[0]
    return ens.create_layout([1], [0], [0], [1], [float(g["rho"])], hist_len=iters)


def replay_c1(ens):
    g = load("c1_trace.npz")
    lay = _c1_ensemble(g, ens)
    assert np.array_equal(ens.download_paths(L.U, 0), g["X_init"])
    assert np.array_equal(ens.download_paths(L.U, 1), g["W_init"])
    ens.loglikhd(lay, L.U, 0, 1)
    assert np.array_equal(ens.get_block_state(lay, L.BLK_LL, 0, 1), g["ll0"])
    for i in range(1, g["Zs"].shape[0] + 1):
        ens.draw_proposal(lay, 0, 1, Z=g["Zs"][i - 1], iter=i)
        assert np.array_equal(ens.get_block_state(lay, L.BLK_LLPROP, 0, 1), g["llp"][i - 1])
        acc = ens.accept_reject(lay, 0, 1, i, E=g["Es"][i - 1], want_acc=True)
        assert np.array_equal(acc, g["acc"][i - 1])
        assert np.array_equal(np.array(ens.fetch_ll(lay, 0, 1, i), dtype=np.float64),
                              g["fetch"][i - 1])
    assert np.array_equal(ens.download_paths(L.U, 0), g["X_final"])
    assert np.array_equal(ens.download_paths(L.U, 1), g["W_final"])
    assert np.array_equal(ens.download_paths(L.UPROP, 0), g["Xp_final"])


def replay_ragged(ens):
    g = load("ragged_trace.npz")
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
    for i in range(1, iters + 1):
        lid, nb = ids[(i - 1) % 2]
        ens.draw_proposal(lid, 0, nb, Z=g["Zs"][i - 1], iter=i)
        acc = ens.accept_reject(lid, 0, nb, i, E=g["Es"][i - 1, :nb], want_acc=True)
        assert np.array_equal(acc, g["acc"][i - 1, :nb]), f"iteration {i}"
        assert np.array_equal(ens.get_block_state(lid, L.BLK_LL, 0, nb), g["ll"][i - 1, :nb])
        assert np.array_equal(ens.get_block_state(lid, L.BLK_LLPROP, 0, nb), g["llp"][i - 1, :nb])
        assert np.array_equal(np.array(ens.fetch_ll(lid, 0, nb, i), dtype=np.float64),
                              g["fetch"][i - 1])
    for unit, what, key in ((L.U, 0, "X_final"), (L.U, 1, "W_final"), (L.UPROP, 0, "Xp_final"),
                            (L.UPROP, 1, "Wp_final")):
        assert np.array_equal(ens.download_paths(unit, what), g[key]), key


def _nested(g):
    npts, out, i = g["n_points"], [], 0
    for K in g["nsegs"]:
        out.append([int(x) for x in npts[i:i + K]])
        i += K
    return out


def test_c1_trace_oracle():
    replay_c1(orc.OracleEnsemble(0, 1, 1, [[201]], prec=0, seed=5, grid_shared=True))


def test_ragged_trace_oracle():
    g = load("ragged_trace.npz")
    replay_ragged(orc.OracleEnsemble(1, 2, 1, _nested(g), prec=0, seed=11))


# ---------------------------------------------------------------- GPU (through the C-ABI)
@pytest.mark.gpu
@pytest.mark.parametrize("mapping", MAPPINGS)
def test_c1_trace_gpu(mapping):
    import diffusionmcmctools_amd as dmt
    ens = dmt.Ensemble(0, 1, 1, [[201]], precision=L.F64, seed=5, grid_shared=True,
                       mapping=mapping)
    replay_c1(ens)
    ens.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mapping", MAPPINGS)
def test_ragged_trace_gpu(mapping):
    import diffusionmcmctools_amd as dmt
    g = load("ragged_trace.npz")
    ens = dmt.Ensemble(1, 2, 1, _nested(g), precision=L.F64, seed=11, mapping=mapping)
    replay_ragged(ens)
    ens.close()


@pytest.mark.gpu
def test_philox_kat_fixture_gpu():
    import diffusionmcmctools_amd as dmt
    g = load("philox_kat.npz")
    for ctr, key, out in zip(g["ctr"], g["key"], g["out"]):
        seed = int(key[0]) | (int(key[1]) << 32)
        np.testing.assert_array_equal(dmt.engine.debug_philox(seed, ctr)[0], out)
