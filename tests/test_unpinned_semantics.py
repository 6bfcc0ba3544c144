"""Where the inferred (unpinned) semantics of DESIGN.md §7 can and cannot move a result.

GuidedProposals.jl and DiffusionDefinition.jl are not vendored, so three conventions of the
path are our reading, not the reference's code: the observation term loglikhd_obs inside a
block's ll, pCN in increment form, and W(t0) = 0 from find_W_for_X!.  Each test below states
the alternative reading and checks, on the oracle, what switching to it would change:
  * loglikhd_obs (src/block.jl:176-178 starts a recomputed block's ll with it; GP.loglikhd,
    src/block.jl:140-144, is upstream): for a path update, u and u° start at the same point under
    the same law, so the term cancels in ll° − ll.  Leaving it out changes no path MH decision
    (src/biblock.jl:121-127) beyond rounding-level ties.  For a parameter update (the tutorials'
    accept_reject_proposal_param!, docs/src/tutorials/biblock/inference.md:43) the term differs
    between θ and θ°, and the reference includes it through recompute_path!.
  * pCN increments vs the cumulative form W° = ρW + √(1−ρ²)W_fresh (src/biblock.jl:94-99):
    equal in exact arithmetic.  Paths and ll agree to rounding, and no decision flips.
  * W(t0) (find_W_for_X! → DD.invsolve!, src/block.jl:120-131): row 0 of the W planes
    enters no solve.  Paths and ll are bit-identical whatever W(t0) holds.
CPU only (oracle)."""
import math

import numpy as np
import pytest

import oracle as orc


def _setup(model, seed):
    from diffusionmcmctools_amd.models import FHN, OU, Lorenz
    rng = np.random.default_rng(seed)
    if model == "ou":
        M = OU([[1.0, 0.3], [-0.3, 0.8]], [0.1, 0.0], 0.5 * np.eye(2))
        aux, kind = M.aux(Theta_t=np.diag([0.5, 0.5])), 0
    elif model == "fhn":
        M = FHN(0.1, -0.8, 1.5, 0.0, 0.3)
        aux, kind = M.aux(-0.8), 1
    else:
        M = Lorenz()
        aux, kind = M.aux(np.array([1.0, 2.0, 20.0])), 2
    d, m, n = M.d, M.m, 201
    t = np.linspace(0, 0.1, n)
    H = rng.uniform(0.5, 2.0, (n, d * (d + 1) // 2))
    H[:, 0] += 3
    F = rng.standard_normal((n, d))
    return dict(kind=kind, d=d, m=m, t=t, H=H, F=F, law=M.law_record(aux), rng=rng)


def _draw_W(s):
    dt = np.diff(s["t"])
    dW = np.zeros((s["t"].size, s["m"]))
    dW[1:] = s["rng"].standard_normal((dt.size, s["m"])) * np.sqrt(dt)[:, None]
    return dW


def _solve(s, dW, x0):
    X, sl, ok = orc.solve_segment(s["kind"], s["d"], s["m"], s["law"], s["t"], s["H"], s["F"],
                                  dW, x0)
    assert ok
    return X, float(sl)


@pytest.mark.parametrize("model", ["ou", "fhn", "lorenz"])
def test_obs_term_cancels_in_path_update(model):
    s = _setup(model, 11)
    flips = 0
    for r in range(64):
        x0 = s["rng"].standard_normal(s["d"]) * 0.3
        obs = float(orc.obs_term(s["d"], s["law"], s["H"][0], s["F"][0], x0))
        dW = _draw_W(s)
        Z = s["rng"].standard_normal((s["t"].size - 1, s["m"]))
        dWo = orc.pcn_segment(s["m"], s["t"], dW, Z, 0.9, math.sqrt(1 - 0.81))
        _, sl = _solve(s, dW, x0)
        _, slo = _solve(s, dWo, x0)
        E = s["rng"].exponential()
        with_obs = (obs + slo) - (obs + sl)
        without = slo - sl
        assert abs(with_obs - without) <= 1e-12 * (1 + abs(obs) + abs(sl) + abs(slo))
        flips += (with_obs > -E) != (without > -E)
    assert flips == 0


@pytest.mark.parametrize("model", ["ou", "fhn", "lorenz"])
def test_pcn_increment_form_vs_cumulative_form(model):
    s = _setup(model, 12)
    rho = 0.8
    srho = math.sqrt(1 - rho ** 2)
    flips = 0
    for r in range(64):
        x0 = s["rng"].standard_normal(s["d"]) * 0.3
        dW = _draw_W(s)
        Z = s["rng"].standard_normal((s["t"].size - 1, s["m"]))
        # increment form (the kernels and the oracle): dW°_i = fma(ρ, dW_i, √(1−ρ²)·√dt_i·Z_i)
        dWi = orc.pcn_segment(s["m"], s["t"], dW, Z, rho, srho)
        # cumulative form: W° = ρW + √(1−ρ²)·W_fresh, then differenced
        W = orc.w_from_increments(dW)
        Wf = np.vstack([np.zeros(s["m"]), np.cumsum(Z * np.sqrt(np.diff(s["t"]))[:, None], 0)])
        dWc = orc.w_to_increments(rho * W + srho * Wf)
        dWc[0] = dWi[0]
        Xi, sli = _solve(s, dWi, x0)
        Xc, slc = _solve(s, dWc, x0)
        _, sl = _solve(s, dW, x0)
        np.testing.assert_allclose(Xi, Xc, rtol=1e-10, atol=1e-12)
        assert abs(sli - slc) <= 1e-9 * (1 + abs(sli))
        E = s["rng"].exponential()
        flips += (sli - sl > -E) != (slc - sl > -E)
    assert flips == 0


@pytest.mark.parametrize("model", ["ou", "fhn", "lorenz"])
def test_w_at_t0_enters_no_solve(model):
    s = _setup(model, 13)
    x0 = s["rng"].standard_normal(s["d"]) * 0.3
    dW = _draw_W(s)
    X0, sl0 = _solve(s, dW, x0)
    for w0 in (3.7, -1e3):
        dW2 = dW.copy()
        dW2[0] = w0
        X2, sl2 = _solve(s, dW2, x0)
        assert np.array_equal(X2, X0) and sl2 == sl0
    # and find_W_for_X! of that path recovers the increments whatever W(t0) was
    W2 = orc.invsolve_segment(s["kind"], s["d"], s["m"], s["law"], s["t"], s["H"], s["F"], X0)
    assert np.all(W2[0] == 0)
    np.testing.assert_allclose(W2[1:], dW[1:], rtol=1e-8, atol=1e-10)
