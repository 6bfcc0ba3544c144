"""Parity of the HIP hot path (through the C-ABI) with the CPU oracle on identical inputs.

Bar: paths X/W, log-weights ll/ll°, MH decisions, histories and fetch_ll are
BIT-IDENTICAL to the oracle in parity mode (host-supplied normals Z and Exp(1) draws E), in fp64
and in fp32.  Device-RNG (perf) mode is bit-identical too: the Philox stream and the
Box–Muller transcendentals are the build's own canonical kernels, restated in the oracle
(DESIGN.md §3).  Full-size configurations are checked through size-independent properties.
"""
import math

import numpy as np
import pytest

import _cases as cs
import oracle as orc
from diffusionmcmctools_amd import _lib as L
from diffusionmcmctools_amd import workloads as W

pytestmark = pytest.mark.gpu

# every parity test runs under both thread mappings of the recursion
MAPPINGS = [pytest.param(L.MAP_LANE, id="lane"), pytest.param(L.MAP_WAVE, id="wave")]


def run_mcmc_parity(w, iters, seed=3, hist_len=None, exact=True, check_every=True,
                    mapping=L.MAP_AUTO):
    hist_len = iters if hist_len is None else hist_len
    dev, ora, lay = cs.both(w, hist_len=hist_len, mapping=mapping)
    nb = w.nblocks
    rng = np.random.default_rng(seed)
    for e in (dev, ora):
        e.loglikhd(lay, L.U, 0, nb)
    cs.assert_ll_equal(dev, ora, lay, nb)
    for i in range(1, iters + 1):
        Z = rng.standard_normal((w.steps_per_iter, w.m))
        E = rng.exponential(1.0, nb)
        okd = dev.draw_proposal(lay, 0, nb, Z=Z, iter=i, want_success=True)
        oko = ora.draw_proposal(lay, 0, nb, Z=Z, iter=i, want_success=True)
        assert np.array_equal(okd, oko)
        ad = dev.accept_reject(lay, 0, nb, i, E=E, want_acc=True)
        ao = ora.accept_reject(lay, 0, nb, i, E=E, want_acc=True)
        assert np.array_equal(ad, ao), f"iteration {i}: decisions differ"
        if check_every or i == iters:
            cs.assert_paths_equal(dev, ora)
            cs.assert_ll_equal(dev, ora, lay, nb)
    if hist_len:
        llh, llph, acch = ora.histories(lay, 0, nb)
        assert np.array_equal(dev.get_block_state(lay, L.BLK_LL_HIST, 0, nb, hist_len), llh)
        assert np.array_equal(dev.get_block_state(lay, L.BLK_LLPROP_HIST, 0, nb, hist_len), llph)
        assert np.array_equal(dev.get_block_state(lay, L.BLK_ACC_HIST, 0, nb, hist_len).astype(bool), acch)
        for it in (1, iters):
            assert dev.fetch_ll(lay, 0, nb, it) == ora.fetch_ll(lay, 0, nb, it)
    return dev, ora, lay


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_c1_ou1d_mcmc_bit_exact(mapping):
    run_mcmc_parity(W.c1_ou1d(), iters=40, mapping=mapping)


@pytest.mark.parametrize("mapping", MAPPINGS)
@pytest.mark.parametrize("resident", ["1", "0"])
def test_c2_ou2d_ragged_tile_bit_exact(mapping, resident, monkeypatch):
    # 200 blocks: 3 full recording tiles + a partial one; one-shot draws on k_block_resident
    # (single-segment blocks of <= 512 steps) and on the general k_block_scan
    monkeypatch.setenv("DMT_SCAN_RESIDENT", resident)
    run_mcmc_parity(W.c2_ou2d(B=200, N=500), iters=4, mapping=mapping)
    if resident == "1":
        run_mcmc_parity(W.c1_ou1d(), iters=3, mapping=mapping)


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_c3_fhn_reduced_bit_exact(mapping):
    run_mcmc_parity(W.c3_fhn(B=130, N=1000, T_burn=0.05), iters=3, check_every=False, mapping=mapping)


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_c5_lorenz_fp32_reduced_bit_exact(mapping):
    run_mcmc_parity(W.c5_lorenz(B=70, N=2000), iters=3, check_every=False, mapping=mapping)


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_c5_lorenz_mixed_unit_sigma_bit_exact(mapping):
    """The canonical σ = I rule (M = H, c = F, σ·dW = dW for a non-linear drift):
    every third block gets σ = 0.8·I, so lane-mapping waves mix laws with and without the
    rule (the per-lane selects of the generic path) next to all-σ = I waves (the fast path);
    device == oracle bit for bit, draws, decisions and find_W_for_X!."""
    w = W.c5_lorenz(B=200, N=300)
    laws = w.laws.copy()
    for b in range(0, 200, 3):
        for p in range(3):
            laws[b, L.LAW_SIGMA + 3 * p + p] = 0.8
        laws[b, L.LAW_A:L.LAW_A + 6] = [0.64, 0.0, 0.0, 0.64, 0.0, 0.64]
    w.laws = laws
    dev, ora, lay = run_mcmc_parity(w, iters=3, check_every=False, mapping=mapping)
    for e in (dev, ora):
        e.find_W_for_X(lay, 0, w.nblocks)
    cs.assert_paths_equal(dev, ora)


# fp32 on the lane mapping: the lane-packet path planes on multi-segment,
# unaligned recordings (the FAST=false packet paths, set_obs, find_W_for_X)
RAGGED_CASES = [pytest.param(L.MAP_LANE, L.F64, id="lane"), pytest.param(L.MAP_WAVE, L.F64, id="wave"),
                pytest.param(L.MAP_LANE, L.F32, id="lane-f32")]


@pytest.mark.parametrize("mapping,prec", RAGGED_CASES)
def test_ragged_blocking_layouts_bit_exact(mapping, prec):
    """Multi-segment recordings, non-terminal blocks with P_last laws, two alternating block
    layouts aliasing the same SamplingPair (src/block.jl:66-72), swaps, loglikhd of both units,
    a proposal law and recompute_path! (src/biblock.jl:334-344)."""
    case, dev, ora, ((A, nA), (B, nB)) = cs.ragged_pair(mapping=mapping, prec=prec)
    rng = np.random.default_rng(9)
    S = case["t"].size - sum(case["nsegs"])
    for e in (dev, ora):
        e.loglikhd(A, L.U, 0, nA)
        e.loglikhd(B, L.U, 0, nB)
    for i in range(1, 7):
        for lay, nb in ((A, nA), (B, nB)):
            Z = rng.standard_normal((S, 1))
            E = rng.exponential(1.0, nb)
            for e in (dev, ora):
                e.loglikhd(lay, L.U, 0, nb)
                e.draw_proposal(lay, 0, nb, Z=Z, iter=i)
            assert np.array_equal(dev.accept_reject(lay, 0, nb, i, E=E, want_acc=True),
                                  ora.accept_reject(lay, 0, nb, i, E=E, want_acc=True))
            cs.assert_paths_equal(dev, ora)
            cs.assert_ll_equal(dev, ora, lay, nb)
    # sub-ranges (a BiBlock is a 1-block range, a BlockCollection one recording's blocks)
    Z = rng.standard_normal((S, 1))
    for e in (dev, ora):
        e.draw_proposal(A, 2, 5, Z=Z, iter=7)
    cs.assert_ll_equal(dev, ora, A, nA)
    cs.assert_paths_equal(dev, ora)
    # swaps
    for what in (L.SWAP_XX, L.SWAP_WW | L.SWAP_LL, L.SWAP_XX | L.SWAP_WW):
        for e in (dev, ora):
            e.swap(A, what, 1, 4)
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, A, nA)
    # proposal law (θ° with a different γ), recompute_path!, ll of u°, swap_PP!
    lawsp = case["laws"].copy()
    lawsp[:, 2] = 1.7
    for e in (dev, ora):
        e.upload_law(L.UPROP, L.LAW_PP, laws=lawsp)
    okd = dev.recompute_path(A, 0, nA, want_success=True)
    oko = ora.recompute_path(A, 0, nA, want_success=True)
    assert np.array_equal(okd, oko)
    cs.assert_paths_equal(dev, ora)
    cs.assert_ll_equal(dev, ora, A, nA)
    for e in (dev, ora):
        e.loglikhd(A, L.UPROP, 0, nA)
        e.swap(A, L.SWAP_PP | L.SWAP_XX | L.SWAP_LL, 0, 3)
        e.loglikhd(A, L.U, 0, nA)
        e.loglikhd(B, L.UPROP, 0, nB)
    cs.assert_ll_equal(dev, ora, A, nA)
    cs.assert_ll_equal(dev, ora, B, nB)
    assert dev.fetch_ll(A, 0, nA) == ora.fetch_ll(A, 0, nA)


def test_ou_multichunk_bit_exact():
    """Linear drift with segments longer than one 512-step scan chunk (1300 steps: two full
    chunks and a partial one)."""
    run_mcmc_parity(W.c2_ou2d(B=70, N=1300), iters=3, check_every=False)


def test_ragged_ou_blocking_layouts_bit_exact():
    """The ragged multi-segment case with a linear drift (2-D OU, one noise): scan kernels over
    multi-segment blocks, P_last laws, two alternating layouts, sub-ranges."""
    case, dev, ora, ((A, nA), (B, nB)) = cs.ragged_pair(model=cs.ou_ragged_model())
    rng = np.random.default_rng(19)
    S = case["t"].size - sum(case["nsegs"])
    for i in range(1, 5):
        for lay, nb in ((A, nA), (B, nB)):
            Z = rng.standard_normal((S, 1))
            E = rng.exponential(1.0, nb)
            for e in (dev, ora):
                e.loglikhd(lay, L.U, 0, nb)
                e.draw_proposal(lay, 0, nb, Z=Z, iter=i)
            assert np.array_equal(dev.accept_reject(lay, 0, nb, i, E=E, want_acc=True),
                                  ora.accept_reject(lay, 0, nb, i, E=E, want_acc=True))
            cs.assert_paths_equal(dev, ora)
            cs.assert_ll_equal(dev, ora, lay, nb)
    for e in (dev, ora):  # device RNG on a sub-range
        e.draw_proposal(A, 2, 6, iter=5)
    cs.assert_paths_equal(dev, ora)
    cs.assert_ll_equal(dev, ora, A, nA)


def _env_ensembles(build, env):
    """Two identical ensembles, the second created under extra environment settings
    (libdmt reads DMT_MCMC_* at dmt_create)."""
    import os
    out = []
    for k in range(2):
        saved = {v: os.environ.get(v) for v in env}
        if k == 1:
            os.environ.update(env)
        try:
            out.append(build())
        finally:
            for v, val in saved.items():
                if val is None:
                    os.environ.pop(v, None)
                else:
                    os.environ[v] = val
    return out


def _c2_build(B, N, hist):
    import diffusionmcmctools_amd as d

    def build():
        w = W.c2_ou2d(B=B, N=N)
        w.meta["hist_len"] = hist
        e = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=29,
                       grid_shared=w.grid_shared)
        lay = W.fill(e, w)
        e.loglikhd(lay, L.U, 0, B)
        return e, lay, B
    return build


def _c1_build(hist):
    import diffusionmcmctools_amd as d

    def build():
        w = W.c1_ou1d()
        w.meta["hist_len"] = hist
        e = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=31,
                       grid_shared=w.grid_shared)
        lay = W.fill(e, w)
        e.loglikhd(lay, L.U, 0, 1)
        return e, lay, 1
    return build


def _ragged_ou_build(hist):
    def build():
        _, dev, _, ((A, nA), _) = cs.ragged_pair(model=cs.ou_ragged_model(), hist_len=hist)
        dev.loglikhd(A, L.U, 0, nA)
        return dev, A, nA
    return build


@pytest.mark.parametrize("case", [
    pytest.param(("c2", 100, 60, 6), id="c2-60steps-resident"),
    pytest.param(("c2", 300, 500, 70), id="c2-500steps-resident-70iters"),
    pytest.param(("c2", 40, 1300, 4), id="c2-1300steps-persistent-multichunk"),
    # the in-kernel fetch_ll tail: several LDS row batches; 8-node lane runs; the direct
    # (binary-counter) path for many blocks
    pytest.param(("c2", 1024, 500, 100), id="c2-full-100iters-tail-batches"),
    pytest.param(("c2", 2048, 80, 12), id="c2-2048blocks-tail-run8"),
    pytest.param(("c2", 4100, 40, 5), id="c2-4100blocks-tail-direct"),
    pytest.param(("c1", 1, 200, 5), id="c1-resident-d1"),
    pytest.param(("ragged", 0, 0, 5), id="ragged-ou-persistent-multisegment"),
])
def test_mcmc_run_persistent_paths_equal_step_path(case):
    """dmt_mcmc_run through the persistent kernels (register-resident k_mcmc_resident for
    single-segment blocks of ≤ 512 steps, k_mcmc_scan otherwise) == the per-iteration kernels
    (DMT_MCMC_PERSIST=0), bit for bit: fetch_ll results, paths of u and u°, ll, ll°, histories."""
    kind, B, N, n = case
    build = (_c2_build(B, N, n + 1) if kind == "c2" else _c1_build(n + 1) if kind == "c1"
             else _ragged_ou_build(n + 1))
    (e0, lay, nb), (e1, _, _) = _env_ensembles(build, {"DMT_MCMC_PERSIST": "0",
                                                        "DMT_SCAN_RESIDENT": "0"})
    r0 = e0.mcmc_run(lay, 0, nb, 1, n, salt=7)
    r1 = e1.mcmc_run(lay, 0, nb, 1, n, salt=7)
    assert np.array_equal(r0, r1)
    cs.assert_paths_equal(e0, e1)
    for what in (L.BLK_LL, L.BLK_LLPROP):
        assert np.array_equal(e0.get_block_state(lay, what, 0, nb), e1.get_block_state(lay, what, 0, nb))
    for what in (L.BLK_ACC_HIST, L.BLK_LL_HIST, L.BLK_LLPROP_HIST):
        assert np.array_equal(e0.get_block_state(lay, what, 0, nb, n + 1),
                              e1.get_block_state(lay, what, 0, nb, n + 1))
    # a second run continues from the state the first one left (selectors, ll on the device)
    assert np.array_equal(e0.mcmc_run(lay, 0, nb, n + 1, 1, salt=7),
                          e1.mcmc_run(lay, 0, nb, n + 1, 1, salt=7))
    cs.assert_paths_equal(e0, e1)


@pytest.mark.parametrize("mapping", MAPPINGS)
@pytest.mark.parametrize("kind", ["ragged-fhn", "c2-resident", "c2-scan", "c1"])
def test_recompute_path_skip_bit_exact(kind, mapping, monkeypatch):
    """recompute_path!(b°, b.WW; skip) (src/block.jl:159-187): every segment's last `skip`
    Girsanov terms are left out of ll° (the path is solved to the end) — device == oracle bit
    for bit on multi-segment FHN blocks with P_last laws (lane and wave kernels), the one-shot
    resident and general OU scan kernels, and skip larger than a segment."""
    if kind == "c2-scan":
        monkeypatch.setenv("DMT_SCAN_RESIDENT", "0")
    if kind == "ragged-fhn":
        case, dev, ora, ((A, nA), _) = cs.ragged_pair(mapping=mapping)
        lawsp = case["laws"].copy()
        lawsp[:, 2] = 1.7
        for e in (dev, ora):
            e.upload_law(L.UPROP, L.LAW_PP, laws=lawsp)
        lay, nb = A, nA
    else:
        w = W.c2_ou2d(B=70, N=300) if kind.startswith("c2") else W.c1_ou1d()
        dev, ora, lay = cs.both(w, hist_len=2, mapping=mapping)
        nb = w.nblocks
    for e in (dev, ora):
        e.loglikhd(lay, L.U, 0, nb)
    for skip in (1, 7, 64, 100000):
        okd = dev.recompute_path(lay, 0, nb, skip=skip, want_success=True)
        oko = ora.recompute_path(lay, 0, nb, skip=skip, want_success=True)
        assert np.array_equal(okd, oko)
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, lay, nb)


@pytest.mark.parametrize("case", [
    pytest.param(("c2", 100, 60, 6), id="c2-60steps"),
    pytest.param(("c2", 301, 500, 70), id="c2-500steps-ragged-workgroup-70iters"),
    pytest.param(("c2", 1024, 500, 100), id="c2-full-100iters"),
    pytest.param(("c1", 1, 200, 5), id="c1-d1"),
])
def test_mcmc_run_producer_consumer_equals_one_wave(case):
    """k_mcmc_resident_pc (a producer and a consumer wave per block, the default) == the
    one-wave k_mcmc_resident (DMT_MCMC_PC=0), bit for bit, including a partly idle last
    workgroup (301 blocks) and a continuation run."""
    kind, B, N, n = case
    build = _c2_build(B, N, n + 1) if kind == "c2" else _c1_build(n + 1)
    (e0, lay, nb), (e1, _, _) = _env_ensembles(build, {"DMT_MCMC_PC": "0"})
    r0 = e0.mcmc_run(lay, 0, nb, 1, n)
    r1 = e1.mcmc_run(lay, 0, nb, 1, n)
    assert np.array_equal(r0, r1)
    cs.assert_paths_equal(e0, e1)
    for what in (L.BLK_LL, L.BLK_LLPROP):
        assert np.array_equal(e0.get_block_state(lay, what, 0, nb), e1.get_block_state(lay, what, 0, nb))
    for what in (L.BLK_ACC_HIST, L.BLK_LL_HIST, L.BLK_LLPROP_HIST):
        assert np.array_equal(e0.get_block_state(lay, what, 0, nb, n + 1),
                              e1.get_block_state(lay, what, 0, nb, n + 1))
    assert np.array_equal(e0.mcmc_run(lay, 0, nb, n + 1, 1), e1.mcmc_run(lay, 0, nb, n + 1, 1))
    cs.assert_paths_equal(e0, e1)


def test_mcmc_run_with_failing_blocks_equals_step_path():
    """Blocks whose proposals overflow (σ = 1e160, so a = σσᵀ = inf) fail every iteration
    (ll° = −Inf, never accepted) inside dmt_mcmc_run's persistent kernel exactly as on the
    per-iteration path; the other blocks are unaffected."""
    bad = [0, 5, 17, 63, 64, 99]

    def build():
        import diffusionmcmctools_amd as d
        w = W.c2_ou2d(B=100, N=60)
        w.meta["hist_len"] = 8
        laws = w.laws.copy()
        for g in bad:
            laws[g, L.LAW_SIGMA:L.LAW_SIGMA + 4] *= 1e160
            laws[g, L.LAW_A:L.LAW_A + 3] = [np.inf, 0.0, np.inf]
        w.laws = laws
        e = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=37,
                       grid_shared=w.grid_shared)
        lay = W.fill(e, w)
        return e, lay, 100
    (e0, lay, nb), (e1, _, _) = _env_ensembles(build, {"DMT_MCMC_PERSIST": "0"})
    r0 = e0.mcmc_run(lay, 0, nb, 1, 6)
    r1 = e1.mcmc_run(lay, 0, nb, 1, 6)
    assert np.array_equal(r0, r1, equal_nan=True)
    cs.assert_paths_equal(e0, e1, equal_nan=True)
    llp = e0.get_block_state(lay, L.BLK_LLPROP_HIST, 0, nb, 8)[:6]
    assert np.all(llp[:, bad] == -math.inf)
    acc = e0.get_block_state(lay, L.BLK_ACC_HIST, 0, nb, 8)[:6]
    assert not acc[1:, bad].any()          # iteration 1 may auto-accept (ll = −Inf before)
    good = np.setdiff1d(np.arange(nb), bad)
    assert np.all(np.isfinite(llp[:, good])) and acc[:, good].mean() > 0.3
    for what in (L.BLK_ACC_HIST, L.BLK_LL_HIST, L.BLK_LLPROP_HIST):
        assert np.array_equal(e0.get_block_state(lay, what, 0, nb, 8),
                              e1.get_block_state(lay, what, 0, nb, 8), equal_nan=True)


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_fetch_ll_tree_bit_exact(mapping):
    w = W.c2_ou2d(B=64 * 80, N=8)
    dev, ora, lay = cs.both(w, hist_len=2, mapping=mapping)
    rng = np.random.default_rng(0)
    nb = w.nblocks
    vals = rng.standard_normal(nb) * 10.0 ** rng.integers(-3, 6, nb)
    valsp = rng.standard_normal(nb) * 1e3
    dev.set_block_state(lay, L.BLK_LL, 0, nb, vals)
    dev.set_block_state(lay, L.BLK_LLPROP, 0, nb, valsp)
    acc = (rng.random((2, nb)) < 0.4).astype(np.uint8)
    dev.set_block_state(lay, L.BLK_ACC_HIST, 0, nb, acc)
    for b0, b1 in ((0, 1), (0, 63), (0, 64), (3, 68), (0, 1000), (17, nb), (0, nb)):
        a, p, n = dev.fetch_ll(lay, b0, b1, 2)
        assert a == orc.pairwise_tree(vals[b0:b1])
        assert p == orc.pairwise_tree(valsp[b0:b1])
        assert n == int(acc[1, b0:b1].sum())


def test_philox_stream_bit_exact(dmt):
    rng = np.random.default_rng(1)
    ctr = rng.integers(0, 2 ** 32, (4096, 4), dtype=np.uint64).astype(np.uint32)
    seed = 0x1234_5678_9ABC_DEF0
    from diffusionmcmctools_amd.engine import debug_normals, debug_philox
    assert np.array_equal(debug_philox(seed, ctr), orc.philox_raw(seed, ctr))
    # Box–Muller through the canonical log / sincospi kernels: bit-identical on both sides
    zd = debug_normals(seed, ctr)
    zo = np.array([orc.normal_pair(seed, c) for c in ctr])
    assert np.array_equal(zd, zo)


def run_device_rng_parity(w, iters, seed=11, mapping=L.MAP_AUTO, salt=5):
    """Perf mode (device Philox normals and Exp(1) draws, nothing supplied by the host):
    paths, ll, decisions and histories bit-identical to the oracle's restatement of the same
    streams."""
    dev, ora, lay = cs.both(w, seed=seed, hist_len=iters, mapping=mapping)
    nb = w.nblocks
    for e in (dev, ora):
        e.loglikhd(lay, L.U, 0, nb)
    for i in range(1, iters + 1):
        for e in (dev, ora):
            e.draw_proposal(lay, 0, nb, iter=i, salt=salt)
        ad = dev.accept_reject(lay, 0, nb, i, salt=salt, want_acc=True)
        ao = ora.accept_reject(lay, 0, nb, i, salt=salt, want_acc=True)
        assert np.array_equal(ad, ao), f"iteration {i}: decisions differ"
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, lay, nb)
    assert dev.fetch_ll(lay, 0, nb, iters) == ora.fetch_ll(lay, 0, nb, iters)
    return dev, ora, lay


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_device_rng_mode_bit_exact_c2(mapping):
    run_device_rng_parity(W.c2_ou2d(B=100, N=500), iters=3, mapping=mapping)


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_device_rng_mode_bit_exact_c3(mapping):
    run_device_rng_parity(W.c3_fhn(B=70, N=300, T_burn=0.1), iters=3, mapping=mapping)


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_device_rng_mode_bit_exact_c5_fp32(mapping):
    run_device_rng_parity(W.c5_lorenz(B=40, N=300), iters=2, mapping=mapping)


@pytest.mark.parametrize("variant", [
    pytest.param({"DMT_LANE_PAIR": "0", "DMT_LANE_SPLIT": "0"}, id="single-lane"),
    pytest.param({"DMT_LANE_PAIR": "1"}, id="lane-pair"),
    pytest.param({"DMT_LANE_PAIR": "0", "DMT_LANE_SPLIT": "1"}, id="producer-consumer"),
])
@pytest.mark.parametrize("cfg", ["c3", "c5"])
def test_device_rng_lane_kernels_bit_exact(cfg, variant, monkeypatch):
    """The three lane-mapping draw kernels (k_block one lane per recording, k_block_pair two
    lanes per recording sharing the normals, k_block_ps producer/consumer waves — on C5's fp32
    lane packets k_block_pk, k_block_pk_pair, k_block_ps_pk) draw the same
    device streams and give the oracle's paths, ll and decisions bit for bit — on a ragged
    last tile (70 / 40 recordings) and through two MCMC iterations."""
    for k, v in variant.items():
        monkeypatch.setenv(k, v)
    w = (W.c3_fhn(B=70, N=300, T_burn=0.1) if cfg == "c3" else W.c5_lorenz(B=40, N=300))
    run_device_rng_parity(w, iters=2, mapping=L.MAP_LANE, seed=13)


@pytest.mark.parametrize("pair", ["0", "1"])
def test_device_rng_lane_pair_multisegment_bit_exact(pair, monkeypatch):
    """k_block_pair on multi-segment blocks with P_last laws (two blocking layouts)."""
    monkeypatch.setenv("DMT_LANE_PAIR", pair)
    _, dev, ora, ((A, nA), (Bl, nB)) = cs.ragged_pair(hist_len=3, mapping=L.MAP_LANE)
    for lay, nb in ((A, nA), (Bl, nB)):
        for e in (dev, ora):
            e.loglikhd(lay, L.U, 0, nb)
        for i in (1, 2):
            for e in (dev, ora):
                e.draw_proposal(lay, 0, nb, iter=i, salt=3)
            assert np.array_equal(dev.accept_reject(lay, 0, nb, i, salt=3, want_acc=True),
                                  ora.accept_reject(lay, 0, nb, i, salt=3, want_acc=True))
            cs.assert_paths_equal(dev, ora)
            cs.assert_ll_equal(dev, ora, lay, nb)


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_failure_gives_minus_inf_and_rejects(mapping):
    w = W.c1_ou1d()
    dev, ora, lay = cs.both(w, hist_len=2, mapping=mapping)
    Z = np.full((w.steps_per_iter, 1), 1e300)   # overflows the path
    for e in (dev, ora):
        e.loglikhd(lay, L.U, 0, 1)
    okd = dev.draw_proposal(lay, 0, 1, Z=Z, iter=1, want_success=True)
    oko = ora.draw_proposal(lay, 0, 1, Z=Z, iter=1, want_success=True)
    assert not okd[0] and not oko[0]
    assert dev.get_block_state(lay, L.BLK_LLPROP, 0, 1)[0] == -math.inf
    assert not dev.accept_reject(lay, 0, 1, 1, E=np.array([1e-300]), want_acc=True)[0]


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_first_proposal_auto_accepted_without_loglikhd(mapping):
    """ll = -Inf initially (src/block.jl:75) so the first proposal is accepted unless
    loglikhd! ran first (Appendix B.2 of SURVEY.md)."""
    w = W.c2_ou2d(B=64, N=50)
    dev, ora, lay = cs.both(w, hist_len=1, mapping=mapping)
    rng = np.random.default_rng(2)
    Z = rng.standard_normal((w.steps_per_iter, 2))
    E = rng.exponential(1.0, 64)
    for e in (dev, ora):
        e.draw_proposal(lay, 0, 64, Z=Z, iter=1)
    assert np.all(dev.accept_reject(lay, 0, 64, 1, E=E, want_acc=True))
    assert np.all(ora.accept_reject(lay, 0, 64, 1, E=E, want_acc=True))
    cs.assert_paths_equal(dev, ora)


# ---------------------------------------------------------------- full-size properties
@pytest.mark.parametrize("cfg", ["c3", "c5"])
def test_full_size_sampled_blocks_bit_exact(cfg):
    """The full per-GPU shard of C3 (65 536 × 1000, fp64) and C5 (32 768 × 2000, fp32) on the
    device (MAP_AUTO: the lane mapping): after init_paths! and one pCN draw, 48 blocks drawn at
    random equal the oracle's restatement of those blocks bit for bit (paths X°, cumulative W°,
    ll°) — blocks are independent, so the sample pins the whole launch."""
    import diffusionmcmctools_amd as d
    w = cs.full_workload(cfg)
    w.meta["hist_len"] = 0
    seed = 4
    dev = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=seed,
                     grid_shared=w.grid_shared)
    lay = W.fill(dev, w, init_Z=True)
    nb = w.nblocks
    ok = dev.draw_proposal(lay, 0, nb, iter=1, salt=0, want_success=True)
    assert ok.all()
    X, Wc = dev.download_paths(L.UPROP, 0), dev.download_paths(L.UPROP, 1)
    llp = dev.get_block_state(lay, L.BLK_LLPROP, 0, nb)
    dev.close()
    npts = w.n_points[0][0]
    blocks = np.sort(np.random.default_rng(7).choice(nb, 48, replace=False))
    blocks[0], blocks[-1] = 0, nb - 1  # the first and last lane of the first and last tile
    for b, (Xo, Wo, llo) in zip(blocks, cs.sampled_blocks_reference(w, blocks, seed, 1)):
        rows = slice(b * npts, (b + 1) * npts)
        np.testing.assert_array_equal(X[rows], Xo)
        np.testing.assert_array_equal(Wc[rows], Wo)
        assert llp[b] == llo


@pytest.mark.parametrize("mapping", MAPPINGS)
@pytest.mark.parametrize("cfg", ["c2", "c3", "c5"])
def test_full_size_properties(cfg, mapping):
    """At BASELINE.json's full sizes (oracle too slow here): size-independent invariants."""
    w = cs.full_workload(cfg)
    import diffusionmcmctools_amd as d
    dev = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=4,
                     grid_shared=w.grid_shared, mapping=mapping)
    w.meta["hist_len"] = 4
    lay = W.fill(dev, w, init_Z=False)
    nb = w.nblocks
    dev.loglikhd(lay, L.U, 0, nb)
    ll0 = dev.get_block_state(lay, L.BLK_LL, 0, nb)
    assert np.all(np.isfinite(ll0))
    for i in (1, 2, 3):
        ok = dev.draw_proposal(lay, 0, nb, iter=i, want_success=True)
        assert ok.mean() > 0.99
        llp = dev.get_block_state(lay, L.BLK_LLPROP, 0, nb)
        # the weight accumulated during the draw == loglikhd° of the stored proposal, bit for bit
        dev.loglikhd(lay, L.UPROP, 0, nb)
        assert np.array_equal(dev.get_block_state(lay, L.BLK_LLPROP, 0, nb), llp)
        acc = dev.accept_reject(lay, 0, nb, i, want_acc=True)
        assert 0.02 < acc.mean() <= 1.0
        ll = dev.get_block_state(lay, L.BLK_LL, 0, nb)
        dev.loglikhd(lay, L.U, 0, nb)
        assert np.array_equal(dev.get_block_state(lay, L.BLK_LL, 0, nb), ll)
    # ρ = 1: the pCN proposal reproduces the accepted path exactly
    lay1 = dev.create_layout(w.n_blocks, w.seg_first, w.seg_last, w.last, np.ones(nb), 1)
    dev.loglikhd(lay1, L.U, 0, nb)
    dev.draw_proposal(lay1, 0, nb, iter=9)
    assert np.array_equal(dev.download_paths(L.UPROP, 0), dev.download_paths(L.U, 0))
    assert np.array_equal(dev.get_block_state(lay1, L.BLK_LLPROP, 0, nb),
                          dev.get_block_state(lay1, L.BLK_LL, 0, nb))
    dev.close()


@pytest.mark.parametrize("mapping", MAPPINGS)
@pytest.mark.parametrize("B", [100, 2500])
def test_mcmc_step_equals_separate_calls(mapping, B):
    """dmt_mcmc_step == draw_proposal + accept_reject + fetch_ll, bit for bit."""
    import diffusionmcmctools_amd as d
    w = W.c2_ou2d(B=B, N=60)
    w.meta["hist_len"] = 4
    ens = []
    for _ in range(2):
        e = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=21,
                       grid_shared=w.grid_shared, mapping=mapping)
        lay = W.fill(e, w)
        e.loglikhd(lay, L.U, 0, B)
        ens.append(e)
    for i in (1, 2, 3, 4):
        ens[0].draw_proposal(lay, 0, B, iter=i, salt=3)
        ens[0].accept_reject(lay, 0, B, i, salt=3)
        r0 = ens[0].fetch_ll(lay, 0, B, i)
        r1 = ens[1].mcmc_step(lay, 0, B, i, salt=3)
        assert r0 == r1
    cs.assert_paths_equal(ens[0], ens[1])


@pytest.mark.parametrize("B", [100, 2500])
def test_mcmc_run_equals_step_sequence(B):
    """dmt_mcmc_run(iter0, n) == n dmt_mcmc_step calls, bit for bit (results, paths, ll,
    histories)."""
    import diffusionmcmctools_amd as d
    w = W.c2_ou2d(B=B, N=60)
    w.meta["hist_len"] = 6
    ens = []
    for _ in range(2):
        e = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=23,
                       grid_shared=w.grid_shared)
        lay = W.fill(e, w)
        e.loglikhd(lay, L.U, 0, B)
        ens.append(e)
    steps = [ens[0].mcmc_step(lay, 0, B, i, salt=5) for i in range(1, 7)]
    run = ens[1].mcmc_run(lay, 0, B, 1, 6, salt=5)
    assert np.array_equal(np.array(steps, dtype=np.float64), run)
    cs.assert_paths_equal(ens[0], ens[1])
    for what in (L.BLK_LL, L.BLK_LLPROP):
        assert np.array_equal(ens[0].get_block_state(lay, what, 0, B),
                              ens[1].get_block_state(lay, what, 0, B))
    assert np.array_equal(ens[0].get_block_state(lay, L.BLK_ACC_HIST, 0, B, 6),
                          ens[1].get_block_state(lay, L.BLK_ACC_HIST, 0, B, 6))


@pytest.mark.parametrize("mapping", MAPPINGS)
@pytest.mark.parametrize("cfg", ["c1", "c2", "c3", "c5"])
def test_find_W_for_X_bit_exact(cfg, mapping):
    """find_W_for_X! (DD.invsolve!) on the device == the oracle, bit for bit, then one more
    MCMC iteration from the reconstructed W agrees too."""
    w = {"c1": lambda: W.c1_ou1d(),
         "c2": lambda: W.c2_ou2d(B=200, N=300),
         "c3": lambda: W.c3_fhn(B=130, N=300, T_burn=0.1),
         "c5": lambda: W.c5_lorenz(B=70, N=300)}[cfg]()
    dev, ora, lay = cs.both(w, hist_len=1, mapping=mapping)
    nb = w.nblocks
    for e in (dev, ora):
        e.find_W_for_X(lay, 0, nb)
    cs.assert_paths_equal(dev, ora)
    rng = np.random.default_rng(4)
    Z = rng.standard_normal((w.steps_per_iter, w.m))
    E = rng.exponential(1.0, nb)
    for e in (dev, ora):
        e.loglikhd(lay, L.U, 0, nb)
        e.draw_proposal(lay, 0, nb, Z=Z, iter=1)
    assert np.array_equal(dev.accept_reject(lay, 0, nb, 1, E=E, want_acc=True),
                          ora.accept_reject(lay, 0, nb, 1, E=E, want_acc=True))
    cs.assert_paths_equal(dev, ora)
    cs.assert_ll_equal(dev, ora, lay, nb)


@pytest.mark.parametrize("mapping,prec", RAGGED_CASES)
def test_find_W_for_X_blocking_layouts(mapping, prec):
    """Ragged multi-segment FHN with P_last laws: invsolve uses PPb on the last segment of
    non-terminal blocks (src/block.jl:118-124); set_obs! before it (fp32 lane packets too)."""
    case, dev, ora, ids = cs.ragged_pair(mapping=mapping, prec=prec)
    for e in (dev, ora):
        e.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    for lid, nb in ids:
        for e in (dev, ora):
            e.set_obs(lid, 0, nb)
            e.find_W_for_X(lid, 0, nb)
        cs.assert_paths_equal(dev, ora)
        for kind in (L.LAW_PP, L.LAW_PPB):
            for a_, b_ in zip(dev.download_law(L.U, kind), ora.download_law(L.U, kind)):
                assert np.array_equal(a_, b_)


@pytest.mark.parametrize("env", [{"DMT_PATH_PACKETS": "0"}, {"DMT_LANE_PAIR": "1"}],
                         ids=["rows", "lane-pairs"])
def test_fp32_lane_variants_bit_identical(env):
    """fp32 lane ensembles: the row layout (DMT_PATH_PACKETS=0) and the lane-pair packet kernel
    (DMT_LANE_PAIR=1, k_block_pk_pair) against the default packet kernel on the ragged
    multi-segment case — device-RNG draws, accepts, loglikhd and the downloaded paths, bit for
    bit."""
    import diffusionmcmctools_amd as d

    def build():
        case = cs.ragged_case(prec=L.F32)
        m = case["model"]
        e = d.Ensemble(m.kind, m.d, m.m, case["n_points"], precision=L.F32, seed=4,
                       mapping=L.MAP_LANE)
        cs.load_ragged(e, case)
        lay = e.create_layout([2, 3, 2], [0, 2, 0, 2, 4, 0, 3], [1, 3, 1, 3, 5, 2, 4],
                              [0, 1, 0, 0, 1, 0, 1], np.full(7, 0.6), 6)
        return e, lay, 7
    (e0, lay, nb), (e1, _, _) = _env_ensembles(build, env)
    for e in (e0, e1):
        e.loglikhd(lay, L.U, 0, nb)
    for i in range(1, 6):
        acc = []
        for e in (e0, e1):
            e.draw_proposal(lay, 0, nb, iter=i, salt=2)
            acc.append(e.accept_reject(lay, 0, nb, i, salt=2, want_acc=True))
        assert np.array_equal(acc[0], acc[1]), i
        cs.assert_paths_equal(e0, e1)
        for what in (L.BLK_LL, L.BLK_LLPROP):
            assert np.array_equal(e0.get_block_state(lay, what, 0, nb),
                                  e1.get_block_state(lay, what, 0, nb)), (i, what)
    for e in (e0, e1):
        e.close()


def test_fp32_split_packets_single_segment_blocks_bit_identical():
    """The packet layout's producer/consumer kernel (DMT_LANE_SPLIT=1, k_block_ps_pk) against the
    default packet kernel on one-segment blocks of the ragged case (terminal: a non-terminal
    block needs two segments): block index 0 holds every recording's first segment
    (packet-aligned), the later block indices segments that start inside a packet (the kernel's
    fallback to lane_block_pk) —
    device-RNG draws, accepts, loglikhd and the downloaded paths, bit for bit."""
    import diffusionmcmctools_amd as d

    def build():
        case = cs.ragged_case(prec=L.F32)
        m = case["model"]
        e = d.Ensemble(m.kind, m.d, m.m, case["n_points"], precision=L.F32, seed=6,
                       mapping=L.MAP_LANE)
        cs.load_ragged(e, case)
        segs = [0, 1, 2, 3, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4]
        lay = e.create_layout([4, 6, 5], segs, segs, [1] * 15, np.full(15, 0.5), 6)
        return e, lay, 15
    (e0, lay, nb), (e1, _, _) = _env_ensembles(build, {"DMT_LANE_SPLIT": "1"})
    for e in (e0, e1):
        e.loglikhd(lay, L.U, 0, nb)
    for i in range(1, 5):
        acc = []
        for e in (e0, e1):
            e.draw_proposal(lay, 0, nb, iter=i, salt=5)
            acc.append(e.accept_reject(lay, 0, nb, i, salt=5, want_acc=True))
        assert np.array_equal(acc[0], acc[1]), i
        cs.assert_paths_equal(e0, e1)
        for what in (L.BLK_LL, L.BLK_LLPROP):
            assert np.array_equal(e0.get_block_state(lay, what, 0, nb),
                                  e1.get_block_state(lay, what, 0, nb)), (i, what)
    for e in (e0, e1):
        e.close()


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_device_guiding_term_reproduces_uploaded_tables(mapping):
    """recompute_guiding_term! on the device over whole-recording terminal blocks rebuilds the
    uploaded PP tables bit for bit (same chained filter as the host set-up)."""
    import diffusionmcmctools_amd as d
    case = cs.ragged_case()
    m = case["model"]
    dev = d.Ensemble(m.kind, m.d, m.m, case["n_points"], precision=case["prec"], seed=1,
                     mapping=mapping)
    cs.load_ragged(dev, case)
    H0, F0, laws0 = dev.download_law(L.U, L.LAW_PP)
    R = len(case["nsegs"])
    lay = dev.create_layout([1] * R, [0] * R, [k - 1 for k in case["nsegs"]], [1] * R,
                            [0.5] * R, 0)
    dev.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    dev.recompute_guiding_term(lay, 0, R, unit=L.U)
    H1, F1, laws1 = dev.download_law(L.U, L.LAW_PP)
    assert np.array_equal(H1, H0) and np.array_equal(F1, F0)
    assert np.array_equal(laws1[:, L.LAW_C0], laws0[:, L.LAW_C0])


@pytest.mark.parametrize("split", [False, True], ids=["fused", "scan_chain"])
def test_device_filter_many_blocks(split):
    """4 100 single-segment FHN blocks of 130 steps (3 chunks, a partial one): one call over all
    of them runs k_filter_fused (a wave per block), calls over halves run k_filter_scan +
    k_filter_chain; both rebuild the host-made tables (the same chunked filter) bit for bit."""
    import diffusionmcmctools_amd as d
    from diffusionmcmctools_amd.models import Observation, packed
    w = W.c3_fhn(B=4100, N=130, T_burn=0.05)
    dev = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=1,
                     grid_shared=w.grid_shared)
    lay = W.fill(dev, w, init_Z=False)
    H0, F0, laws0 = dev.download_law(L.U, L.LAW_PP)
    infos = [Observation(0.1, np.array([v]), np.array([[1.0, 0.0]]), 0.01 * np.eye(1)).info()
             for v in w.meta["v"]]
    dev.upload_obs(np.stack([packed(i[0]) for i in infos]), np.stack([i[1] for i in infos]),
                   np.array([float(i[2]) for i in infos]))
    dev.upload_law(L.U, L.LAW_PP, H=np.zeros_like(H0), F=np.zeros_like(F0))
    ranges = [(0, 2050), (2050, w.nblocks)] if split else [(0, w.nblocks)]
    for b0, b1 in ranges:
        dev.recompute_guiding_term(lay, b0, b1, unit=L.U)
    H1, F1, laws1 = dev.download_law(L.U, L.LAW_PP)
    assert np.array_equal(H1, H0) and np.array_equal(F1, F0)
    assert np.array_equal(laws1[:, L.LAW_C0], laws0[:, L.LAW_C0])
    dev.close()


@pytest.mark.parametrize("B", [300, 4100], ids=["scan_chain", "fused"])
def test_device_filter_lorenz_fp32(B):
    """The device filter for d = 3 on an fp32 ensemble (C5's Lorenz law, full-state
    observations, grids and tables in float): device == oracle bit for bit, through the
    few-blocks kernels (300 blocks) and the fused kernel (4 100 blocks)."""
    from diffusionmcmctools_amd.models import Observation, packed
    w = W.c5_lorenz(B=B, N=130)
    dev, ora, lay = cs.both(w, hist_len=1, init_Z=False)
    infos = [Observation(0.2, v, np.eye(3), 0.1 * np.eye(3)).info() for v in w.meta["v"]]
    Hobs = np.stack([packed(i[0]) for i in infos])
    Fobs = np.stack([i[1] for i in infos])
    cobs = np.array([float(i[2]) for i in infos])
    for e in (dev, ora):
        e.upload_obs(Hobs, Fobs, cobs)
        e.recompute_guiding_term(lay, 0, w.nblocks, unit=L.U)
    Hd, Fd, ld = dev.download_law(L.U, L.LAW_PP)
    Ho, Fo, lo = ora.download_law(L.U, L.LAW_PP)
    assert np.array_equal(Hd, Ho) and np.array_equal(Fd, Fo)
    assert np.array_equal(ld[:, L.LAW_C0], lo[:, L.LAW_C0])
    dev.close()


@pytest.mark.parametrize("mapping", MAPPINGS)
def test_blocking_loop_bit_exact(mapping):
    """The reference's smoothing-with-blocking iteration (docs/src/tutorials/biblock/
    smoothing_with_blocking.md:34-44): set_obs!, recompute_guiding_term!(bb.b),
    find_W_for_X!, loglikhd!, draw_proposal_path!, accept_reject_proposal_path! — alternating
    two blockings, device == oracle bit for bit (laws, paths, ll, decisions)."""
    case, dev, ora, ids = cs.ragged_pair(mapping=mapping, hist_len=6)
    for e in (dev, ora):
        e.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    rng = np.random.default_rng(8)
    S = dev.S
    for i in range(1, 7):
        lid, nb = ids[(i - 1) % 2]
        Z = rng.standard_normal((S, 1))
        E = rng.exponential(1.0, nb)
        for e in (dev, ora):
            e.set_obs(lid, 0, nb)
            e.recompute_guiding_term(lid, 0, nb, unit=L.U)
            e.find_W_for_X(lid, 0, nb)
            e.loglikhd(lid, L.U, 0, nb)
            e.draw_proposal(lid, 0, nb, Z=Z, iter=i)
        for kind in (L.LAW_PP, L.LAW_PPB):
            for a_, b_ in zip(dev.download_law(L.U, kind), ora.download_law(L.U, kind)):
                assert np.array_equal(a_, b_), f"iteration {i}, law kind {kind}"
        ad = dev.accept_reject(lid, 0, nb, i, E=E, want_acc=True)
        ao = ora.accept_reject(lid, 0, nb, i, E=E, want_acc=True)
        assert np.array_equal(ad, ao), f"iteration {i}"
        cs.assert_paths_equal(dev, ora)
        cs.assert_ll_equal(dev, ora, lid, nb)


@pytest.mark.parametrize("n_iter", [5])
def test_headline_mcmc_run_full_c2_bit_exact(n_iter):
    """The bench's headline kernel itself — dmt_mcmc_run on the full C2 shard (1 024 blocks ×
    500 steps, fp64, device RNG), i.e. k_mcmc_resident_pc: draw, MH decision, histories and
    every iteration's fetch_ll tree in one launch — against the oracle's restatement of the same
    iterations (src/biblock.jl:80-127: pCN draw, E > -(ll° - ll), swaps), ALL blocks, bit for
    bit: every iteration's decisions, fetch_ll, fetch_ll° and accepted count, and the final
    paths X, W and ll of u.  The oracle runs the canonical arithmetic on the
    device's own Philox normal and Exp(1) streams (key (iteration, salt 0))."""
    import diffusionmcmctools_amd as d
    w = cs.full_workload("c2")
    w.meta["hist_len"] = n_iter
    seed = 0xD1FF
    dev = d.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=seed,
                     grid_shared=w.grid_shared)
    lay = W.fill(dev, w, init_Z=False)
    B, npts = w.nblocks, w.n_points[0][0]
    dev.loglikhd(lay, L.U, 0, B)
    X, Wd = dev.download_paths(L.U, 0), dev.download_paths(L.U, 2)
    ll = dev.get_block_state(lay, L.BLK_LL, 0, B)
    out = dev.mcmc_run(lay, 0, B, 1, n_iter)          # one k_mcmc_resident_pc launch
    acc_dev = dev.get_block_state(lay, L.BLK_ACC_HIST, 0, B, hist_len=n_iter).astype(bool)
    Xd, Wdd = dev.download_paths(L.U, 0), dev.download_paths(L.U, 2)
    lld = dev.get_block_state(lay, L.BLK_LL, 0, B)
    dev.close()
    rho = np.full(B, w.rho)
    for it in range(1, n_iter + 1):
        Xo, Wo, llp, nf = orc.draw_terminal_blocks(
            w.model.kind, w.d, w.m, npts, w.laws, w.t, w.H, w.F, X, Wd, rho, Z=None, seed=seed,
            it=it, salt=0, prec=w.precision, nthreads=8, t_shared=True, H_shared=w.H_shared)
        assert nf == 0
        E = orc.exp1_range(seed, 0, B, it, 0)
        acc = E > -(llp - ll)
        np.testing.assert_array_equal(acc_dev[it - 1], acc, err_msg=f"decisions, iteration {it}")
        llprop_after = np.where(acc, ll, llp)         # swap_ll! on acceptance
        ll = np.where(acc, llp, ll)
        sel = np.repeat(acc, npts)[:, None]
        X, Wd = np.where(sel, Xo, X), np.where(sel, Wo, Wd)
        want = (orc.pairwise_tree(ll), orc.pairwise_tree(llprop_after), float(acc.sum()))
        assert tuple(out[it - 1]) == want, (it, tuple(out[it - 1]), want)
    assert 0.3 < acc_dev.mean() < 1.0
    np.testing.assert_array_equal(Xd, X)
    np.testing.assert_array_equal(Wdd, Wd)
    np.testing.assert_array_equal(lld, ll)
