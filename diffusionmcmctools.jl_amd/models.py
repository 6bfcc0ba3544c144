"""Models, auxiliary laws, observations, time grids and guiding-term set-up (host side).

These replace the set-up the reference delegates to its upstream packages
(DiffusionDefinition `@load_diffusion`, ObservationSchemes recordings/time grids,
GuidedProposals `build_guid_prop`; call sites /root/reference/src/sampling_unit.jl:55-74).
They only build the *inputs* of the device hot path: law records (include/dmt.h) and the
guiding-term tables H, F, c.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .engine import guiding_linear, guiding_linear_td


def packed(M):
    """Row-major upper-triangular packing of a symmetric d×d matrix (00,01,..,11,..)."""
    M = np.asarray(M, dtype=np.float64)
    d = M.shape[0]
    return np.array([M[a, b] for a in range(d) for b in range(a, d)])


def unpacked(p, d):
    M = np.zeros((d, d))
    k = 0
    for a in range(d):
        for b in range(a, d):
            M[a, b] = M[b, a] = p[k]
            k += 1
    return M


# ------------------------------------------------------------------ models
@dataclass
class LinearAux:
    """Auxiliary law dX = (Bt X + beta) dt + sigma_t dW (GuidedProposals' linear P̃)."""
    Bt: np.ndarray
    beta: np.ndarray
    sigma_t: np.ndarray  # d×m
    # the point the model was linearised at (FHN's FitzHughNagumoAux, Lorenz): the device
    # re-derives Bt, beta from θ and this point in set_proposal_law!; None = a fixed law
    anchor: np.ndarray | None = None

    @property
    def at(self):
        s = np.asarray(self.sigma_t, dtype=np.float64)
        return s @ s.T


@dataclass
class TimeDependentLinearAux:
    """Auxiliary law dX = (B̃(t) X + β̃(t)) dt + σ̃ dW whose drift varies within a segment (any
    linear law of GuidedProposals, the reference's aux_laws, src/sampling_unit.jl:55-66).
    ``Bt(t)``, ``beta(t)``: callables; on the device, step i takes its left point's values
    (include/dmt.h dmt_upload_aux).  Non-linear drifts only."""
    Bt: object
    beta: object
    sigma_t: np.ndarray  # d×m
    anchor = None  # never re-linearised: the law is given as functions of t

    @property
    def at(self):
        s = np.asarray(self.sigma_t, dtype=np.float64)
        return s @ s.T

    def table(self, t):
        """Per-point rows B̃(t_i) (row-major), β̃(t_i) on grid ``t``."""
        return np.stack([np.concatenate([np.asarray(self.Bt(x), dtype=np.float64).ravel(),
                                         np.asarray(self.beta(x), dtype=np.float64).ravel()])
                         for x in np.asarray(t, dtype=np.float64)])


def is_time_dependent(aux):
    return isinstance(aux, TimeDependentLinearAux)


# parameter-name aliases: DiffusionDefinition's symbols (:ϵ, :γ, …) and ASCII spellings
_ALIASES = {"eps": "ϵ", "epsilon": "ϵ", "ε": "ϵ", "gamma": "γ", "beta": "β", "sigma": "σ"}


def canonical_name(name):
    name = str(name).lstrip(":")
    return _ALIASES.get(name, name)


class Model:
    kind: int
    d: int
    m: int
    # DiffusionDefinition's parameter names in θ order (set_parameters!, set_proposal_law!)
    param_names: tuple = ()
    # DD.var_parameter_names(P) (src/param_names_collections.jl:141-164): the parameters an MCMC
    # update may change; the tutorials restrict it per type, e.g.
    # ``FHN.var_parameter_names = ("γ",)`` for ``DD.var_parameter_names(::FitzHughNagumo) = (:γ,)``
    var_parameter_names: tuple = None

    def variable_names(self):
        v = type(self).var_parameter_names
        return tuple(self.param_names if v is None else (canonical_name(n) for n in v))

    def _attr(self, name):
        raise KeyError(name)

    def get_param(self, name):
        return getattr(self, self._attr(canonical_name(name)))

    def set_param(self, name, value):
        """``DD.set_parameters!``-style update of one named parameter in place."""
        setattr(self, self._attr(canonical_name(name)), float(value))

    def theta_vec(self) -> np.ndarray:
        raise NotImplementedError

    def sigma(self) -> np.ndarray:
        raise NotImplementedError

    def drift(self, x):
        raise NotImplementedError

    def aux_for(self, obs):
        """The auxiliary law of a segment ending in observation ``obs`` (the reference's
        ``AuxLaw(…, obs)`` of build_guid_prop): linearised at the observed value."""
        raise NotImplementedError

    def law_record(self, aux: LinearAux, c0: float = 0.0) -> np.ndarray:
        rec = np.zeros(L.LAW_STRIDE)
        th = self.theta_vec()
        rec[L.LAW_THETA:L.LAW_THETA + len(th)] = th
        sg = np.asarray(self.sigma(), dtype=np.float64).reshape(self.d, self.m)
        rec[L.LAW_SIGMA:L.LAW_SIGMA + self.d * self.m] = sg.ravel()
        a = sg @ sg.T
        hp = self.d * (self.d + 1) // 2
        rec[L.LAW_A:L.LAW_A + hp] = packed(a)
        if is_time_dependent(aux):  # B̃, β̃ come from the per-point table (dmt_upload_aux)
            rec[L.LAW_AUXTD] = 1.0
        else:
            rec[L.LAW_BT:L.LAW_BT + self.d * self.d] = np.asarray(aux.Bt, dtype=np.float64).ravel()
            rec[L.LAW_BETA:L.LAW_BETA + self.d] = np.asarray(aux.beta, dtype=np.float64)
        da = a - aux.at
        rec[L.LAW_DA:L.LAW_DA + hp] = packed(da)
        rec[L.LAW_C0] = c0
        rec[L.LAW_TRACE] = 1.0 if np.any(da != 0.0) else 0.0
        if self.d == self.m:  # σ⁻¹ for find_W_for_X! (invsolve)
            rec[L.LAW_SIGINV:L.LAW_SIGINV + self.d * self.d] = np.linalg.inv(sg).ravel()
        if aux.anchor is not None:
            an = np.atleast_1d(np.asarray(aux.anchor, dtype=np.float64))
            rec[L.LAW_ANCHOR:L.LAW_ANCHOR + an.size] = an
            rec[L.LAW_AUXLIN] = 1.0
        return rec

    def simulate(self, t, x0, rng, substeps=1):
        """Plain Euler–Maruyama forward simulation on grid t (data generation)."""
        t = np.asarray(t, dtype=np.float64)
        x = np.array(x0, dtype=np.float64)
        out = np.empty((t.size, self.d))
        out[0] = x
        sg = self.sigma()
        for i in range(t.size - 1):
            h = (t[i + 1] - t[i]) / substeps
            for _ in range(substeps):
                x = x + self.drift(x) * h + sg @ rng.standard_normal(self.m) * math.sqrt(h)
            out[i + 1] = x
        return out


class OU(Model):
    """dX = -Theta (X - mu) dt + sigma dW (DiffusionDefinition OU-type model)."""

    kind = L.MODEL_OU

    def __init__(self, Theta, mu, sigma):
        self.Theta = np.atleast_2d(np.asarray(Theta, dtype=np.float64))
        self.mu = np.atleast_1d(np.asarray(mu, dtype=np.float64))
        self.sg = np.atleast_2d(np.asarray(sigma, dtype=np.float64))
        self.d = self.Theta.shape[0]
        self.m = self.sg.shape[1]

    def theta_vec(self):
        v = np.zeros(12)
        v[: self.d * self.d] = self.Theta.ravel()
        v[9:9 + self.d] = self.mu
        return v

    def sigma(self):
        return self.sg

    def drift(self, x):
        return -self.Theta @ (np.asarray(x) - self.mu)

    def aux_for(self, obs):
        return self.aux()

    def aux(self, Theta_t=None, mu_t=None, sigma_t=None):
        """OU auxiliary law (Theta_t, mu_t): Bt = -Theta_t, beta = Theta_t mu_t."""
        Th = self.Theta if Theta_t is None else np.atleast_2d(np.asarray(Theta_t, dtype=np.float64))
        mu = self.mu if mu_t is None else np.atleast_1d(np.asarray(mu_t, dtype=np.float64))
        sg = self.sg if sigma_t is None else np.atleast_2d(np.asarray(sigma_t, dtype=np.float64))
        return LinearAux(-Th, Th @ mu, sg)


class FHN(Model):
    """FitzHugh–Nagumo in DiffusionDefinition's parametrisation, θ = (ϵ, s, γ, β, σ)
    (/root/reference/docs/src/tutorials/preamble.md:77):
    dY = (Y - Y^3 - X + s)/ϵ dt,  dX = (γY - X + β) dt + σ dW."""

    kind = L.MODEL_FHN
    d, m = 2, 1
    param_names = ("ϵ", "s", "γ", "β", "σ")
    _ATTRS = {"ϵ": "eps", "s": "s", "γ": "gamma", "β": "beta", "σ": "sg"}

    def _attr(self, name):
        return self._ATTRS[name]

    def __init__(self, eps, s, gamma, beta, sigma):
        self.eps, self.s, self.gamma, self.beta, self.sg = map(float, (eps, s, gamma, beta, sigma))

    def theta_vec(self):
        # the kernels read 1/ϵ, s, γ, β; the raw ϵ and σ follow for set_proposal_law!
        return np.array([1.0 / self.eps, self.s, self.gamma, self.beta, self.eps, self.sg])

    def sigma(self):
        return np.array([[0.0], [self.sg]])

    def drift(self, x):
        y, v = x
        return np.array([(y - y ** 3 - v + self.s) / self.eps, self.gamma * y - v + self.beta])

    def aux_for(self, obs):
        return self.aux(np.atleast_1d(obs.v)[0])  # FitzHughNagumoAux at the observed y

    def aux(self, yT):
        """FitzHughNagumoAux: linearisation at the observed end value yT (the arithmetic
        order of the device's set_proposal_law! re-derivation)."""
        e, y = self.eps, float(yT)
        Bt = np.array([[(1.0 - 3.0 * (y * y)) / e, -1.0 / e], [self.gamma, -1.0]])
        beta = np.array([(self.s + 2.0 * (y * y * y)) / e, self.beta])
        return LinearAux(Bt, beta, self.sigma(), anchor=np.array([y]))


class Lorenz(Model):
    """Lorenz-63 with diagonal noise: b = (s(y-x), x(r-z)-y, xy-βz)."""

    kind = L.MODEL_LORENZ
    d, m = 3, 3
    param_names = ("s", "r", "β")
    _ATTRS = {"s": "s_", "r": "r", "β": "b"}

    def _attr(self, name):
        return self._ATTRS[name]

    def __init__(self, s=10.0, r=28.0, beta=8.0 / 3.0, sigma=(1.0, 1.0, 1.0)):
        self.s_, self.r, self.b = float(s), float(r), float(beta)
        self.sg = np.diag(np.asarray(sigma, dtype=np.float64))

    def theta_vec(self):
        return np.array([self.s_, self.r, self.b])

    def sigma(self):
        return self.sg

    def drift(self, x):
        x0, x1, x2 = x
        return np.array([self.s_ * (x1 - x0), x0 * (self.r - x2) - x1, x0 * x1 - self.b * x2])

    def aux_for(self, obs):
        return self.aux(obs.v)  # full-state observation

    def aux(self, v):
        """Linearisation of the drift at the point v."""
        x0, x1, x2 = (float(u) for u in v)
        J = np.array([[-self.s_, self.s_, 0.0], [self.r - x2, -1.0, -x0], [x1, x0, -self.b]])
        f = self.drift((x0, x1, x2))
        beta = np.array([f[i] - ((J[i, 0] * x0 + J[i, 1] * x1) + J[i, 2] * x2) for i in range(3)])
        return LinearAux(J, beta, self.sg, anchor=np.array([x0, x1, x2]))


# ------------------------------------------------------------------ observations, grids
@dataclass
class Observation:
    """v ~ N(L x(t), Sigma) (ObservationSchemes LinearGsnObs)."""
    t: float
    v: np.ndarray
    L: np.ndarray
    Sigma: np.ndarray

    def info(self):
        """Terminal information (H, F, c) contributed by this observation."""
        Lm = np.atleast_2d(np.asarray(self.L, dtype=np.float64))
        S = np.atleast_2d(np.asarray(self.Sigma, dtype=np.float64))
        v = np.atleast_1d(np.asarray(self.v, dtype=np.float64))
        Si = np.linalg.inv(S)
        k = v.size
        H = Lm.T @ Si @ Lm
        F = Lm.T @ Si @ v
        c = 0.5 * v @ Si @ v + 0.5 * k * math.log(2 * math.pi) + 0.5 * math.log(np.linalg.det(S))
        return H, F, c


@dataclass
class Recording:
    """(P, obs, t0, x0) of ObservationSchemes (docs/src/get_started/overview.md:18-20);
    KnownStartingPt x0.  ``P`` is the recording's target law (a :class:`Model`), which the
    reference-form constructors ``SamplingPair(AuxLaw, recording, tts)`` read."""
    obs: list
    t0: float
    x0: np.ndarray
    extra: dict = field(default_factory=dict)
    P: Model | None = None

    @property
    def x0_prior(self):
        return self.x0


def build_recording(P, data, t0, x0):
    """``build_recording(P, data, t0, KnownStartingPt(y1))`` (docs/src/tutorials/preamble.md:87):
    a recording of the observations ``data`` (a list of :class:`Observation`) of a path of the
    target law ``P`` started at the known point ``x0``.  ``P`` is copied: ``set_parameters``
    changes the recording's own law."""
    import copy
    return Recording(list(data), float(t0), np.asarray(x0, dtype=np.float64), P=copy.deepcopy(P))


def set_parameters(target, theta):
    """``OBS.set_parameters!(recording, θ)`` / ``OBS.set_parameters!(all_obs, θ)``
    (docs/src/tutorials/biblock/inference.md:58): the named parameters of the target law(s).
    ``theta``: a mapping name → value; a name is a law parameter (``"γ"``), a per-recording name
    ``"REC<k>_<p>"`` or a shared name declared with ``AllObservations.add_dependency``."""
    from .param_names import AllObservations
    if isinstance(target, AllObservations):
        target.set_parameters(theta)
        return
    for name, v in dict(theta).items():
        nm = canonical_name(name)
        if nm.startswith("REC") and "_" in nm:
            nm = canonical_name(nm.split("_", 1)[1])
        target.P.set_param(nm, v)


class FitzHughNagumoAux:
    """``FitzHughNagumoAux`` (DiffusionDefinition, docs/src/tutorials/preamble.md:28) as the
    ``aux_laws`` of the reference-form constructors: for the segment ending in observation
    ``obs``, the target law ``P`` linearised at the observed ``y`` (``FHN.aux``)."""

    def __new__(cls, P, obs):
        return P.aux_for(obs)


class LorenzAux:
    """The Lorenz-63 auxiliary law of config C5: the drift linearised at the observed state."""

    def __new__(cls, P, obs):
        return P.aux_for(obs)


def standard_guid_prop_time_transf(t0, T, dt):
    """Uniform grid t0:dt:T mapped by τ(t) = t0 + (t-t0)(2 - (t-t0)/(T-t0))
    (GuidedProposals' standard time change, named at biblock/smoothing.md:27)."""
    n = max(int(round((T - t0) / dt)), 1)
    u = np.linspace(t0, T, n + 1)
    s = u - t0
    tau = t0 + s * (2.0 - s / (T - t0))
    tau[0], tau[-1] = t0, T
    return tau


def setup_time_grids(recording, dt: float, transf=standard_guid_prop_time_transf):
    """One grid per inter-observation interval (OBS.setup_time_grids); of an
    ``AllObservations``, one such list per recording."""
    if hasattr(recording, "recordings"):
        return [setup_time_grids(rec, dt, transf) for rec in recording.recordings]
    grids, t0 = [], recording.t0
    for ob in recording.obs:
        grids.append(transf(t0, ob.t, dt))
        t0 = ob.t
    return grids


def uniform_grid(t0, T, n):
    return np.linspace(t0, T, n + 1)


# ------------------------------------------------------------------ guiding terms
def guiding_chain(auxes, grids, infos, H_in=None):
    """Backward filter over the consecutive segments of one recording.

    auxes[k]: LinearAux on segment k; grids[k]: its grid; infos[k]: (H, F, c) of the
    observation(s) at the end of segment k.  Segment k's terminal condition is its own
    observation information plus the guiding term of segment k+1 at its start
    (GP.build_guid_prop / recompute_guiding_term!).  Returns per segment (H packed, F, c).
    """
    K = len(grids)
    out = [None] * K
    nxt = None
    for k in range(K - 1, -1, -1):
        d = np.asarray(auxes[k].sigma_t).shape[0]
        HT, FT, cT = infos[k]
        HT = np.array(HT, dtype=np.float64).reshape(d, d)
        FT = np.array(FT, dtype=np.float64).reshape(d)
        if nxt is not None:
            Hn, Fn, cn = nxt
            HT = HT + unpacked(Hn, d)
            FT = FT + Fn
            cT = cT + cn
        if is_time_dependent(auxes[k]):
            H, F, c = guiding_linear_td(auxes[k].table(grids[k]), packed(auxes[k].at), grids[k],
                                        packed(HT), FT, cT)
        else:
            H, F, c = guiding_linear(auxes[k].Bt, auxes[k].beta, packed(auxes[k].at), grids[k],
                                     packed(HT), FT, cT)
        out[k] = (H, F, c)
        nxt = (H[0], F[0], c[0])
    return out


def artificial_obs_info(v, noise):
    """Exact full-state artificial observation used by blocking laws
    (guid_prop_for_blocking(…, artificial_noise = 1e-11), src/sampling_unit.jl:57,61-66)."""
    v = np.asarray(v, dtype=np.float64)
    d = v.size
    return Observation(0.0, v, np.eye(d), noise * np.eye(d)).info()
