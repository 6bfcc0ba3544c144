"""Path buffers of the lane mapping ("path buffers"), through the C-ABI.

A MAP_LANE ensemble holds three physical buffers per path container (XX, WW); each draw picks,
per wave, where the proposals go (path_plan in dmt_kernels.hip): a buffer holding none of the
wave's u paths, the smallest group's buffer with stragglers writing to the majority's, a
consolidation of every u into the majority's buffer (copied during the sweep), or mixed
per-lane destinations.  Which buffer holds what is bookkeeping only: paths, ll, decisions and
fetch_ll must equal the oracle's bit for bit whatever the acceptance pattern, with three
buffers and with two (DMT_PATH_BUFS=2), with consolidation and without it (DMT_REPAIR_DIV
large: mixed), consolidating whole lines (DMT_FULL_COPY=1), in every lane draw kernel.  Forced decisions (E = ±inf per block) drive the
buffer states through every branch: nearly all accepted, half, few accepted.
"""
import numpy as np
import pytest

import _cases as cs
from diffusionmcmctools_amd import _lib as L
from diffusionmcmctools_amd import workloads as W

pytestmark = pytest.mark.gpu


def _set_bufs(monkeypatch, bufs):
    monkeypatch.setenv("DMT_PATH_BUFS", bufs[0])
    monkeypatch.setenv("DMT_REPAIR_DIV", "100000" if bufs.endswith("mixed") else "1")
    monkeypatch.setenv("DMT_FULL_COPY", "1" if bufs.endswith("full") else "0")


def _workload(cfg):
    # ragged last tiles: 200 = 3 x 64 + 8 recordings, 130 = 2 x 64 + 2
    return W.c5_lorenz(B=200, N=120) if cfg == "c5" else W.c3_fhn(B=130, N=150, T_burn=0.1)


@pytest.mark.parametrize("split", ["0", "1"], ids=["k_block", "k_block_ps"])
@pytest.mark.parametrize("p_acc", [0.97, 0.5, 0.15])
@pytest.mark.parametrize("bufs", ["3", "3-mixed", "3-full", "2", "2-mixed"])
@pytest.mark.parametrize("cfg", ["c5", "c3"])
def test_forced_decisions_bit_exact(cfg, bufs, p_acc, split, monkeypatch):
    _set_bufs(monkeypatch, bufs)
    monkeypatch.setenv("DMT_LANE_SPLIT", split)
    monkeypatch.setenv("DMT_LANE_PAIR", "0")
    w = _workload(cfg)
    iters = 10
    dev, ora, lay = cs.both(w, seed=7, hist_len=iters, mapping=L.MAP_LANE)
    nb = w.nblocks
    rng = np.random.default_rng(int(p_acc * 100) + 17)
    for e in (dev, ora):
        e.loglikhd(lay, L.U, 0, nb)
    for i in range(1, iters + 1):
        for e in (dev, ora):
            e.draw_proposal(lay, 0, nb, iter=i, salt=3)
        E = np.where(rng.random(nb) < p_acc, np.inf, -np.inf)
        ad = dev.accept_reject(lay, 0, nb, i, E=E, want_acc=True)
        ao = ora.accept_reject(lay, 0, nb, i, E=E, want_acc=True)
        assert np.array_equal(ad, ao), f"iteration {i}: decisions differ"
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, lay, nb)
    assert dev.fetch_ll(lay, 0, nb, iters) == ora.fetch_ll(lay, 0, nb, iters)


@pytest.mark.parametrize("bufs", ["3", "3-mixed", "2"])
def test_blocking_layouts_and_swaps_bit_exact(bufs, monkeypatch):
    """Multi-segment blocks of two aliasing blocking layouts (P_last laws), explicit swaps of
    the path containers (dmt_swap, the reference's swap_XX!/swap_WW!) between draws, and
    loglikhd° / recompute_path! reading u° wherever the last draw put it."""
    _set_bufs(monkeypatch, bufs)
    _, dev, ora, ((A, nA), (Bl, nB)) = cs.ragged_pair(hist_len=4, mapping=L.MAP_LANE)
    rng = np.random.default_rng(5)
    for rnd in range(2):
        for lay, nb in ((A, nA), (Bl, nB)):
            for e in (dev, ora):
                e.loglikhd(lay, L.U, 0, nb)
            for i in (1, 2):
                for e in (dev, ora):
                    e.draw_proposal(lay, 0, nb, iter=2 * rnd + i, salt=9)
                for e in (dev, ora):
                    e.loglikhd(lay, L.UPROP, 0, nb)
                E = np.where(rng.random(nb) < 0.5, np.inf, -np.inf)
                assert np.array_equal(
                    dev.accept_reject(lay, 0, nb, 2 * rnd + i, E=E, want_acc=True),
                    ora.accept_reject(lay, 0, nb, 2 * rnd + i, E=E, want_acc=True))
                cs.assert_paths_equal(dev, ora)
                cs.assert_ll_equal(dev, ora, lay, nb)
            h = nb // 2
            for e in (dev, ora):
                e.swap(lay, L.SWAP_XX | L.SWAP_WW, 0, h)
            cs.assert_paths_equal(dev, ora)
