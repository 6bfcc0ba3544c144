"""Known-answer tests that pin the oracle (and libdmt's host set-up) without the reference.

The reference cannot run here and its own tests are empty (/root/reference/test/runtests.jl:4-6),
so these analytic KATs are what pins the arithmetic.  CPU only.
"""
import math

import numpy as np
import pytest

import np_oracle as npo
import oracle as orc


def _packed(M):
    d = M.shape[0]
    return np.array([M[a, b] for a in range(d) for b in range(a, d)])


# ---------------------------------------------------------------- Philox (Random123 KATs)
@pytest.mark.parametrize("ctr,key,want", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox4x32_10_known_answers(ctr, key, want):
    seed = key[0] | (key[1] << 32)
    out = orc.philox_raw(seed, np.array(ctr, dtype=np.uint32))
    assert tuple(int(v) for v in out[0]) == want


def test_normals_moments():
    Z = orc.normals_segment(123, 7, 3, 0, 200000, 1)
    assert abs(Z.mean()) < 0.01 and abs(Z.std() - 1) < 0.01
    E = np.array([orc.exp1(1, b, 5, 0) for b in range(20000)])
    assert abs(E.mean() - 1) < 0.03 and E.min() > 0


def test_bm_tables_match_generator():
    """The fp64 Box–Muller tables compiled into libdmt and into the oracle are the output of
    scripts/gen_bm_tables.py (60-digit decimal values rounded once)."""
    import subprocess
    import sys
    root = __import__("os").path.dirname(__import__("os").path.dirname(__file__))
    r = subprocess.run([sys.executable, "scripts/gen_bm_tables.py", "--check"], cwd=root)
    assert r.returncode == 0


def test_fp64_normals_match_libm_box_muller():
    """The canonical fp64 normal pair (table-driven log and sincospi) equals
    sqrt(-2 log u1)·(cos, sin)(2π u2) of the same 53-bit uniforms through libm, within a few
    ulp, over 20 000 Philox blocks, including u1 → 1 (log → 0⁻, never a NaN)."""
    seed = 0x5EED
    ctr = np.zeros((20000, 4), dtype=np.uint32)
    ctr[:, 0] = np.arange(20000)
    ctr[:, 2] = 9
    words = orc.philox_raw(seed, ctr).astype(np.uint64)
    k1 = ((words[:, 0] >> np.uint64(5)) << np.uint64(26)) | (words[:, 1] >> np.uint64(6))
    k2 = ((words[:, 2] >> np.uint64(5)) << np.uint64(26)) | (words[:, 3] >> np.uint64(6))
    u1 = (k1 + np.uint64(1)).astype(np.float64) * 2.0 ** -53
    u2 = k2.astype(np.float64) * 2.0 ** -53
    rad = np.sqrt(-2.0 * np.log(u1))
    want = np.stack([rad * np.cos(2 * np.pi * u2), rad * np.sin(2 * np.pi * u2)], 1)
    got = np.array([orc.normal_pair(seed, c) for c in ctr])
    assert np.all(np.isfinite(got))
    assert np.max(np.abs(got - want) / (1.0 + np.abs(want))) < 4e-15
    # u1 → 1⁻: the log stays negative and exact near 0
    assert orc.lib.orc_bm_log(1.0) == 0.0
    for k in range(1, 200):
        u = 1.0 - k * 2.0 ** -53
        v = orc.lib.orc_bm_log(u)
        assert v < 0 and abs(v - math.log(u)) <= 2 ** -52 * abs(math.log(u))


# ---------------------------------------------------------------- guiding term
def test_guiding_ou1d_closed_form(dmt):
    theta, mu, sigma, T, v, Sig = 0.5, 0.2, 0.7, 1.0, 0.3, 0.01
    t = np.linspace(0, T, 101) ** 1.3
    t = t / t[-1] * T
    Hc, Fc, cc = npo.ou1d_guiding(theta, mu, sigma, T, t, v, Sig)
    HT, FT = 1 / Sig, v / Sig
    cT = 0.5 * v * v / Sig + 0.5 * math.log(2 * math.pi * Sig)
    H, F, c = dmt.guiding_linear([[-theta]], [theta * mu], [sigma ** 2], t, [HT], [FT], cT)
    np.testing.assert_allclose(H[:, 0], Hc, rtol=1e-12)
    np.testing.assert_allclose(F[:, 0], Fc, rtol=1e-12)
    np.testing.assert_allclose(c, cc, rtol=1e-12)


@pytest.mark.parametrize("case", ["ou2d", "fhn", "fhn_blocking", "lorenz"])
def test_guiding_matches_expm_filter(dmt, case):
    rng = np.random.default_rng(0)
    if case == "ou2d":
        B = -np.diag([0.5, 0.5]); beta = np.zeros(2); at = 0.25 * np.eye(2)
        HT = np.eye(2) / 0.01; FT = np.array([0.3, -0.2]) / 0.01; cT = 1.0; T = 1.0
    elif case in ("fhn", "fhn_blocking"):
        from diffusionmcmctools_amd.models import FHN
        m = FHN(0.1, -0.8, 1.5, 0.0, 0.3)
        aux = m.aux(-0.7)
        B, beta, at = aux.Bt, aux.beta, aux.at
        if case == "fhn":
            HT = np.array([[100.0, 0], [0, 0]]); FT = np.array([-70.0, 0]); cT = 2.0
        else:  # exact full-state artificial observation, noise 1e-11 (src/sampling_unit.jl:57)
            HT = np.eye(2) / 1e-11; FT = np.array([-0.7, -0.4]) / 1e-11; cT = 0.0
        T = 0.1
    else:
        from diffusionmcmctools_amd.models import Lorenz
        m = Lorenz()
        aux = m.aux(np.array([1.0, 2.0, 20.0]))
        B, beta, at = aux.Bt, aux.beta, aux.at
        HT = np.eye(3) / 0.1; FT = np.array([1.0, 2.0, 20.0]) / 0.1; cT = 0.5; T = 0.2
    from diffusionmcmctools_amd.models import standard_guid_prop_time_transf
    t = standard_guid_prop_time_transf(0.0, T, T / 200)
    H, F, c = dmt.guiding_linear(B, beta, _packed(at), t, _packed(HT), FT, cT)
    He, Fe, ce = npo.backward_filter_expm(B, beta, at, t, HT, FT, cT)
    d = len(beta)
    Hp = np.stack([_packed(He[i]) for i in range(len(t))])
    # relative to the scale of each quantity (H spans 1e11 in the blocking case)
    np.testing.assert_allclose(H, Hp, rtol=1e-8, atol=1e-9 * np.abs(Hp).max())
    np.testing.assert_allclose(F, Fe, rtol=1e-8, atol=1e-9 * np.abs(Fe).max())
    np.testing.assert_allclose(c, ce, rtol=1e-8, atol=1e-8 * max(1.0, np.abs(ce).max()))
    assert d in (2, 3)
    # the oracle's C restatement of the filter (used for the device recompute_guiding_term
    # parity) is the same arithmetic as the product's host filter: bit for bit
    Ho, Fo, co = orc.backward_filter_segment(d, np.asarray(B).ravel(), beta, _packed(at), t,
                                             _packed(HT), FT, cT)
    assert np.array_equal(Ho, H) and np.array_equal(Fo, F) and np.array_equal(co, c)


def test_obs_term_is_gaussian_density(dmt):
    """log rho~(t0, x0) == log N(v; L mu_T(x0), L Sigma_T L' + Sigma) for a linear aux law."""
    Th = np.array([[0.5, 0.1], [-0.2, 0.7]]); mu = np.array([0.1, -0.3]); sg = 0.4 * np.eye(2)
    B = -Th; beta = Th @ mu; at = sg @ sg.T
    L = np.array([[1.0, 0.5]]); Sig = np.array([[0.02]]); v = np.array([0.4])
    Si = np.linalg.inv(Sig)
    HT = L.T @ Si @ L; FT = L.T @ Si @ v
    cT = 0.5 * v @ Si @ v + 0.5 * math.log(2 * math.pi) + 0.5 * math.log(np.linalg.det(Sig))
    t = np.linspace(0, 1.0, 51)
    H, F, c = dmt.guiding_linear(B, beta, _packed(at), t, _packed(HT), FT, cT)
    x0 = np.array([0.3, -0.1])
    law = np.zeros(64); law[49] = c[0]
    lo = orc.obs_term(2, law, H[0], F[0], x0)
    Phi, m_, K = npo.transition_expm(B, beta, at, 1.0)
    want = npo.gaussian_logpdf(v, L @ (Phi @ x0 + m_), L @ K @ L.T + Sig)
    assert abs(lo - want) < 1e-11


# ---------------------------------------------------------------- Euler recursion + weight
def _law(model, d, m, theta, sigma, Bt, beta, at_tilde, c0=0.0):
    from diffusionmcmctools_amd import _lib as L
    rec = np.zeros(64)
    rec[:len(theta)] = theta
    sg = np.asarray(sigma).reshape(d, m)
    rec[16:16 + d * m] = sg.ravel()
    a = sg @ sg.T
    rec[25:25 + d * (d + 1) // 2] = _packed(a)
    rec[31:31 + d * d] = np.asarray(Bt).ravel()
    rec[40:40 + d] = beta
    da = a - at_tilde
    rec[43:43 + d * (d + 1) // 2] = _packed(da)
    rec[49] = c0
    rec[50] = 1.0 if np.any(da != 0) else 0.0
    assert L.LAW_STRIDE == 64
    return rec


@pytest.mark.parametrize("model", ["ou", "fhn", "lorenz", "ou_trace"])
def test_c_oracle_matches_naive_numpy(dmt, model):
    rng = np.random.default_rng(3)
    from diffusionmcmctools_amd.models import FHN, OU, Lorenz
    if model in ("ou", "ou_trace"):
        M = OU([[1.0, 0.3], [-0.3, 0.8]], [0.1, 0.0], 0.5 * np.eye(2))
        aux = M.aux(Theta_t=np.diag([0.5, 0.5]), sigma_t=(0.6 * np.eye(2) if model == "ou_trace" else None))
        kind = 0
    elif model == "fhn":
        M = FHN(0.1, -0.8, 1.5, 0.0, 0.3); aux = M.aux(-0.8); kind = 1
    else:
        M = Lorenz(); aux = M.aux(np.array([1.0, 2.0, 20.0])); kind = 2
    d, m = M.d, M.m
    n = 301
    t = np.linspace(0, 0.1, n)
    H = rng.uniform(0.5, 2.0, (n, d * (d + 1) // 2)); H[:, 0] += 3
    F = rng.standard_normal((n, d))
    W = np.vstack([np.zeros(m), np.cumsum(rng.standard_normal((n - 1, m)) * np.sqrt(np.diff(t))[:, None], 0)])
    law = M.law_record(aux)
    y1 = rng.standard_normal(d) * 0.3
    X, ll, ok = orc.solve_segment(kind, d, m, law, t, H, F, orc.w_to_increments(W), y1)
    Xn, lln = npo.solve_segment_naive(kind, d, m, law, t, H, F, W, y1)
    assert ok
    np.testing.assert_allclose(X, Xn, rtol=1e-11, atol=1e-12)
    assert abs(ll - lln) <= 1e-11 * (1 + abs(lln))
    # stored-path weight == weight accumulated during the solve (same order, bit for bit)
    assert orc.path_ll_segment(kind, d, m, law, t, H, F, X) == ll


def test_weight_vanishes_when_target_is_aux():
    """Linear target equal to the auxiliary law: G ≡ 0 up to rounding."""
    d = m = 2
    Th = np.array([[1.0, 0.3], [-0.3, 0.8]]); mu = np.zeros(2); sg = 0.5 * np.eye(2)
    theta = np.zeros(12); theta[:4] = Th.ravel()
    law = _law(0, d, m, theta, sg, -Th, Th @ mu, sg @ sg.T)
    rng = np.random.default_rng(1)
    n = 501; t = np.linspace(0, 1, n)
    H = np.tile([4.0, 0.5, 3.0], (n, 1)); F = rng.standard_normal((n, 2))
    W = np.vstack([np.zeros(2), np.cumsum(rng.standard_normal((n - 1, 2)) * 0.0447, 0)])
    _, ll, ok = orc.solve_segment(0, d, m, law, t, H, F, orc.w_to_increments(W), np.zeros(2))
    assert ok and abs(ll) < 1e-13


def test_pcn_limits():
    """Increment-form pCN: rho = 1 reuses dW exactly, rho = 0 is a fresh draw sqrt(dt) Z,
    and the cumulative path is rho W + sqrt(1-rho^2) W_fresh up to rounding."""
    rng = np.random.default_rng(2)
    n, m = 101, 2
    t = np.linspace(0, 1, n) ** 1.5
    W = np.vstack([np.zeros(m), np.cumsum(rng.standard_normal((n - 1, m)), 0)])
    dW = orc.w_to_increments(W)
    Z = rng.standard_normal((n - 1, m))
    assert np.array_equal(orc.pcn_segment(m, t, dW, Z, 1.0, 0.0), dW)
    fresh = np.vstack([np.zeros(m), Z * np.sqrt(np.diff(t))[:, None]])
    assert np.array_equal(orc.pcn_segment(m, t, dW, Z, 0.0, 1.0), fresh)
    rho = 0.8
    Wo = orc.w_from_increments(orc.pcn_segment(m, t, dW, Z, rho, math.sqrt(1 - rho ** 2)))
    np.testing.assert_allclose(Wo, rho * W + math.sqrt(1 - rho ** 2) * np.cumsum(fresh, 0), atol=1e-12)


def test_bridge_hits_endpoint_small_noise(dmt):
    """Brownian target = aux, exact-ish end observation: the guided path ends at v."""
    d = m = 1
    law = _law(0, 1, 1, np.zeros(12), [[1.0]], [[0.0]], [0.0], np.eye(1))
    n = 2001
    t = np.linspace(0, 1, n)
    v, Sig = 1.7, 1e-9
    H, F, c = dmt.guiding_linear([[0.0]], [0.0], [1.0], t, [1 / Sig], [v / Sig], 0.0)
    rng = np.random.default_rng(4)
    W = np.concatenate([[0], np.cumsum(rng.standard_normal(n - 1) * math.sqrt(1 / (n - 1)))])[:, None]
    X, ll, ok = orc.solve_segment(0, 1, 1, law, t, H, F, orc.w_to_increments(W), np.zeros(1))
    assert ok and abs(X[-1, 0] - v) < 0.05


def test_pairwise_tree_order():
    v = [1e16, 1.0, -1e16, 1.0]
    assert orc.pairwise_tree(v) == (1e16 + 1.0) + (-1e16 + 1.0)
    assert orc.pairwise_tree([]) == 0.0
    assert orc.pairwise_tree([3.0, 4.0, 5.0]) == (3.0 + 4.0) + (5.0 + 0.0)


# ---------------------------------------------------------------- find_W_for_X! (invsolve)
@pytest.mark.parametrize("cfg", ["ou2d", "fhn", "lorenz"])
def test_invsolve_inverts_the_forward_solve(cfg):
    """DD.invsolve! restated: increments recovered from a forward-solved path reproduce the
    drawn increments (up to cancellation rounding) and re-solve to the same path."""
    from diffusionmcmctools_amd import workloads as W
    w = {"ou2d": lambda: W.c2_ou2d(B=1, N=300),
         "fhn": lambda: W.c3_fhn(B=1, N=300, T_burn=0.1),
         "lorenz": lambda: W.c5_lorenz(B=1, N=300)}[cfg]()
    prec = w.precision
    npts = w.n_points[0][0]
    rng = np.random.default_rng(3)
    dW = np.zeros((npts, w.m))
    dW[1:] = rng.standard_normal((npts - 1, w.m)) * np.sqrt(np.diff(w.t))[:, None]
    H = w.H if not w.H_shared else w.H
    X, ll, ok = orc.solve_segment(w.model.kind, w.d, w.m, w.laws[0], w.t, H, w.F, dW, w.X0[0], prec)
    assert ok
    W2 = orc.invsolve_segment(w.model.kind, w.d, w.m, w.laws[0], w.t, H, w.F, X, prec)
    tol = 1e-9 if prec == 0 else 2e-3
    np.testing.assert_allclose(W2[1:], dW[1:], rtol=tol, atol=tol * 1e-2)
    assert np.all(W2[0] == 0)
    X2, _, ok2 = orc.solve_segment(w.model.kind, w.d, w.m, w.laws[0], w.t, H, w.F, W2, w.X0[0], prec)
    assert ok2
    np.testing.assert_allclose(X2, X, rtol=tol, atol=tol)


def test_oracle_recompute_guiding_term_reproduces_uploaded_tables():
    """recompute_guiding_term! restated on whole-recording terminal blocks, from the per-segment
    observation information, rebuilds exactly the PP tables the set-up uploaded (both are the
    same chained backward filter)."""
    import _cases as cs
    case = cs.ragged_case()
    m = case["model"]
    ora = orc.OracleEnsemble(m.kind, m.d, m.m, case["n_points"], prec=case["prec"], seed=1)
    cs.load_ragged(ora, case)
    H0, F0, laws0 = ora.download_law(0, 0)
    R = len(case["nsegs"])
    lay = ora.create_layout([1] * R, [0] * R, [k - 1 for k in case["nsegs"]], [1] * R,
                            [0.5] * R, 0)
    ora.upload_obs(case["Hobs"], case["Fobs"], case["cobs"])
    ora.recompute_guiding_term(lay, 0, R, unit=0)
    H1, F1, laws1 = ora.download_law(0, 0)
    assert np.array_equal(H1, H0) and np.array_equal(F1, F0)
    assert np.array_equal(laws1[:, 49], laws0[:, 49])


@pytest.mark.parametrize("npts", [1, 2, 64, 65, 66, 129, 300])
def test_chunked_filter_lengths(dmt, npts):
    """The chunked filter (64-step chunks from the segment end, DESIGN.md §3, guiding term) at chunk-edge
    lengths: host == oracle bit for bit, and both agree with the matrix-exponential filter."""
    from diffusionmcmctools_amd.models import FHN, standard_guid_prop_time_transf
    aux = FHN(0.1, -0.8, 1.5, 0.0, 0.3).aux(0.4)
    B, beta, at = aux.Bt, aux.beta, aux.at
    HT = np.array([[100.0, 0], [0, 0]]); FT = np.array([40.0, 0]); cT = 1.0
    t = standard_guid_prop_time_transf(0.0, 0.2, 0.2 / max(npts - 1, 1))[:npts] if npts > 1 \
        else np.array([0.0])
    H, F, c = dmt.guiding_linear(B, beta, _packed(at), t, _packed(HT), FT, cT)
    Ho, Fo, co = orc.backward_filter_segment(2, np.asarray(B).ravel(), beta, _packed(at), t,
                                             _packed(HT), FT, cT)
    assert np.array_equal(Ho, H) and np.array_equal(Fo, F) and np.array_equal(co, c)
    He, Fe, ce = npo.backward_filter_expm(B, beta, at, t, HT, FT, cT)
    Hp = np.stack([_packed(He[i]) for i in range(len(t))])
    np.testing.assert_allclose(H, Hp, rtol=1e-9, atol=1e-10 * np.abs(Hp).max())
    np.testing.assert_allclose(F, Fe, rtol=1e-9, atol=1e-10 * np.abs(Fe).max())
    np.testing.assert_allclose(c, ce, rtol=1e-9, atol=1e-9)


def test_recompute_path_skip_semantics():
    """recompute_path!(b°, b.WW; skip) in the oracle (GP.solve_and_ll!(…; skip), GuidedProposals
    v0.1.0, not vendored — DESIGN.md §7): the path is solved to the end whatever `skip`; the
    last `skip` Girsanov terms leave ll°; skip ≥ the segment's steps leaves loglikhd_obs only."""
    from diffusionmcmctools_amd import _lib as L
    from diffusionmcmctools_amd import workloads as W
    w = W.c1_ou1d()
    w.meta["hist_len"] = 1
    ora = orc.OracleEnsemble(w.model.kind, w.d, w.m, w.n_points, prec=w.precision, seed=4,
                             grid_shared=w.grid_shared)
    lay = W.fill(ora, w)
    res = {}
    for skip in (0, 1, 5, 10 ** 6):
        ora.recompute_path(lay, 0, 1, skip=skip)
        res[skip] = (ora.download_paths(L.UPROP, 0).copy(),
                     float(ora.get_block_state(lay, L.BLK_LLPROP, 0, 1)[0]))
    for skip in (1, 5, 10 ** 6):
        assert np.array_equal(res[skip][0], res[0][0])
    ll = [res[k][1] for k in (0, 1, 5, 10 ** 6)]
    assert all(np.isfinite(ll)) and len(set(ll)) == 4
    # skip beyond the segment: only the observation term of the block start remains
    X = res[0][0].reshape(-1, w.d)
    lw = ora.up.PP[0]
    obs = orc.obs_term(w.d, lw.rec, lw.H[0], lw.F[0], X[0], w.precision)
    assert ll[3] == float(obs)
