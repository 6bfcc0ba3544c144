"""Host-side mirror of the reference's composite-unit interface, backed by libdmt.

Same objects and method names as DiffusionMCMCTools.jl (``!`` dropped, ``°`` spelled
``_prop``), same argument meaning (``mcmciter`` is the 1-based MCMC iteration), same
results: every method is one C-ABI call over the block range the object covers.

  reference (src/…)                              here
  SamplingUnit            sampling_unit.jl:48     SamplingUnit     (u or u° of one recording)
  SamplingPair            sampling_pair.jl:33     SamplingPair     (u, u° of one recording)
  SamplingEnsemble        sampling_ensemble.jl:13 SamplingEnsemble (owns the device handle)
  BiBlock{L}              biblock.jl:42           BiBlock          (one block, L = is_last)
  BlockCollection         block_collection.jl:19  BlockCollection  (the blocks of a recording)
  BlockEnsemble           block_ensemble.jl:17    BlockEnsemble    (all recordings' blocks)

Ranges are 0-based half-open Python ``range``s over a recording's inter-observation segments
(the reference's ``ranges[i]`` are 1-based ``UnitRange``s of the same segments).  Path
containers live on the GPU; ``XX``/``WW`` download them in the reference layout.
Draws: by default each call takes fresh variables from the handle's device stream counter
(``DMT_RNG_AUTO``), as the reference's calls take them from the global RNG
(src/biblock.jl:94-99,122): a loop of ``draw_proposal_path()`` / ``accept_reject_proposal_path(i)``
never reuses normals or Exp(1) variables, and blockings drawn in one iteration are independent.
An explicit ``iter``/``salt`` selects a reproducible keyed stream instead; ``Z``/``E`` supply the
normals / Exp(1) variables (parity mode).
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .engine import Ensemble

def _key(iter, salt):
    """(iter, salt) of a draw: no key given → the handle's stream counter (RNG_AUTO)."""
    if iter is None and salt is None:
        return 0, L.RNG_AUTO
    return (0 if iter is None else int(iter)), (0 if salt is None else int(salt))


__all__ = ["SamplingEnsemble", "SamplingPair", "SamplingUnit", "BlockEnsemble",
           "BlockCollection", "BiBlock", "Block"]


# Test seam: an engine factory (model, n_points, precision, seed) -> engine that the
# reference-form constructors use instead of the HIP library (tests run the same caller code
# on the CPU oracle with it).  None (always, outside tests): the HIP library.
_ENGINE_FACTORY = None


class engine_override:
    """``with engine_override(factory): …`` — test infrastructure only (see _ENGINE_FACTORY)."""

    def __init__(self, factory):
        self.factory = factory

    def __enter__(self):
        global _ENGINE_FACTORY
        self.prev, _ENGINE_FACTORY = _ENGINE_FACTORY, self.factory
        return self

    def __exit__(self, *exc):
        global _ENGINE_FACTORY
        _ENGINE_FACTORY = self.prev
        return False


def _is_model(x):
    from .models import Model
    return isinstance(x, Model)


def _aux_callable(AuxLaw):
    """The reference's ``aux_laws`` argument (src/sampling_unit.jl:55-60) as the
    ``aux_laws(model, r, k, obs)`` of :meth:`SamplingEnsemble.from_recordings`: an auxiliary-law
    constructor ``AuxLaw(P, obs)`` (e.g. ``models.FitzHughNagumoAux``: the target linearised at
    the segment's observation), a fixed ``LinearAux`` or ``TimeDependentLinearAux`` (B̃(t), β̃(t))
    for every segment, or one such per segment (a list)."""
    from .models import LinearAux, TimeDependentLinearAux
    if AuxLaw is None:  # the target's own auxiliary law at the observation (Model.aux_for)
        return lambda mdl, r, k, ob: mdl.aux_for(ob)
    if isinstance(AuxLaw, (LinearAux, TimeDependentLinearAux)):
        return lambda mdl, r, k, ob: AuxLaw
    if isinstance(AuxLaw, (list, tuple)):
        return lambda mdl, r, k, ob: (AuxLaw[k](mdl, ob) if callable(AuxLaw[k]) else AuxLaw[k])
    return lambda mdl, r, k, ob: AuxLaw(mdl, ob)


# ============================================================================ sampling units
class SamplingEnsemble:
    """``SamplingEnsemble(aux_laws, recordings, tts, …)`` (src/sampling_ensemble.jl:13-41):
    the u/u° containers of every recording, resident on one GPU.

    ``model`` is a :class:`diffusionmcmctools_amd.models.Model`; ``n_points[r][k]`` the grid
    size of segment k of recording r.  Guiding terms, laws and the grid are uploaded with
    :meth:`set_guiding` / :meth:`upload_grid` (host filter: ``models.guiding_chain``)."""

    def __new__(cls, *args, **kw):
        if args and not _is_model(args[0]):
            # the reference's SamplingEnsemble(aux_laws, recordings, tts; aux_laws_blocking,
            # artificial_noise) (src/sampling_ensemble.jl:20-40): each recording's target law
            # is its ``P`` (models.build_recording)
            return cls._from_reference_args(*args, **kw)
        return super().__new__(cls)

    @classmethod
    def _from_reference_args(cls, aux_laws, recordings, tts, args=(), aux_laws_blocking=None,
                             artificial_noise=1e-11, solver_choice_blocking=None, _pair=False,
                             **kw):
        """The reference's ``SamplingEnsemble(aux_laws, recordings, tts, args=tuple();
        aux_laws_blocking=aux_laws, artificial_noise=1e-11, solver_choice_blocking=args)``
        (src/sampling_ensemble.jl:20-40; ``_pair``: ``SamplingPair(…)`` of one recording,
        src/sampling_pair.jl:40-50).  As there (``_vec_me``), a list ``aux_laws`` /
        ``aux_laws_blocking`` / ``artificial_noise`` of the ensemble form holds one entry per
        recording; each entry (and the pair form's argument) may itself be a list per segment
        (``_aux_callable``).  ``args`` / ``solver_choice_blocking`` choose GuidedProposals' ODE
        solver of the guiding term: the device's guiding term is the exact discrete filter
        (DESIGN.md §7), so they are accepted and have no effect."""
        recordings = list(recordings)
        models = [getattr(rec, "P", None) for rec in recordings]
        if any(m is None for m in models):
            raise ValueError("SamplingEnsemble(aux_laws, recordings, tts): every recording needs "
                             "its target law P (models.build_recording(P, data, t0, x0))")
        if any(type(m) is not type(models[0]) for m in models):
            raise ValueError("all recordings of one ensemble must share the model family")
        R = len(recordings)

        def per_rec(v):  # _vec_me (src/sampling_ensemble.jl:44)
            if not _pair and isinstance(v, (list, tuple)):
                if len(v) != R:
                    raise ValueError(f"a per-recording argument needs {R} entries, got {len(v)}")
                return list(v)
            return [v] * R
        noise = per_rec(artificial_noise)
        if any(x != noise[0] for x in noise):
            raise ValueError("one artificial_noise per device ensemble (the device stores one)")
        artificial_noise = float(noise[0])
        # per-recording target parameters enter the law records (recording r's P)
        aux = [_aux_callable(a) for a in per_rec(aux_laws)]
        auxb = ([_aux_callable(a) for a in per_rec(aux_laws_blocking)]
                if aux_laws_blocking is not None else aux)
        se = cls.from_recordings(models[0], recordings, tts,
                                 aux_laws=lambda mdl, r, k, ob: aux[r](models[r], r, k, ob),
                                 aux_laws_blocking=lambda mdl, r, k, ob: auxb[r](models[r], r, k, ob),
                                 artificial_noise=artificial_noise,
                                 record_models=models, **kw)
        se._ref_built = True
        return se

    def __init__(self, model, n_points=None, precision=L.F64, seed=0, device=0,
                 grid_shared=False, mapping=L.MAP_AUTO, _engine=None, **_):
        if getattr(self, "_ref_built", False):
            return  # built by the reference-form __new__ (Python re-enters __init__)
        self.model = model
        self.n_points = [list(r) for r in n_points]
        # _engine: test seam for driving the host logic on another backend; the product
        # path is always the HIP library (no CPU fallback).
        self.ens = _engine if _engine is not None else Ensemble(
            model.kind, model.d, model.m, n_points, precision=precision, seed=seed,
            device=device, grid_shared=grid_shared, mapping=mapping)
        self.recordings = [SamplingPair(self, r) for r in range(len(self.n_points))]

    @classmethod
    def from_recordings(cls, model, recordings, tts, aux_laws=None, aux_laws_blocking=None,
                        artificial_noise=1e-11, blocking=True, precision=L.F64, seed=0,
                        device=0, mapping=L.MAP_AUTO, init=True, _engine=None,
                        record_models=None):
        """``SamplingEnsemble(aux_laws, recordings, tts; aux_laws_blocking, artificial_noise)``
        (src/sampling_ensemble.jl:13-41 → ``SamplingPair`` → ``SamplingUnit``,
        src/sampling_unit.jl:55-74): the containers built from the recordings and their laws,
        not from hand-packed tables.

        * ``build_guid_prop`` (:60): per segment k of recording r the auxiliary law
          ``aux_laws(model, r, k, obs)`` (default ``model.aux_for(obs)``: the law linearised at
          the observation, as FitzHughNagumoAux / the Lorenz aux of the configs); guiding terms
          by the exact backward filter over the recording's segments (``models.guiding_chain``,
          libdmt's host ``dmt_guiding_linear``), law records ``model.law_record(aux, c(t0))``;
        * ``guid_prop_for_blocking`` (:61-66, ``blocking``): per segment the same law with an
          extra exact full-state artificial observation of noise ``artificial_noise`` at the
          segment end — a placeholder (the observed coordinates, zeros elsewhere) until
          ``set_obs!`` freezes the accepted end point; ``aux_laws_blocking``
          defaults to ``aux_laws``;
        * the observations for the device's re-derivations (``set_observations``) and
          ``init_paths!`` from each recording's ``x0`` (``init``).
        ``tts[r][k]``: the grid of segment k of recording r (``setup_time_grids``);
        ``record_models[r]``: recording r's own target law (its parameters go into its law
        records; default ``model`` for all)."""
        from .models import artificial_obs_info, guiding_chain, is_time_dependent, packed
        aux_laws = aux_laws or (lambda mdl, r, k, ob: mdl.aux_for(ob))
        aux_laws_blocking = aux_laws_blocking or aux_laws
        d = model.d
        t_all, H_all, F_all, laws, n_points, infos_all = [], [], [], [], [], []
        Hb_all, Fb_all, lawsb = [], [], []
        # time-dependent auxiliary laws (models.TimeDependentLinearAux): per-point tables of
        # both kinds, zero rows for time-homogeneous segments (unused there)
        tab_pp, tab_b, any_td = [], [], False
        C_ = d * d + d
        for r, rec in enumerate(recordings):
            grids = [np.asarray(g, dtype=np.float64) for g in tts[r]]
            if len(grids) != len(rec.obs):
                raise ValueError(f"recording {r}: {len(rec.obs)} observations, {len(grids)} grids")
            auxes = [aux_laws(model, r, k, ob) for k, ob in enumerate(rec.obs)]
            for a_, g_ in zip(auxes, grids):
                td = is_time_dependent(a_)
                any_td |= td
                tab_pp.append(a_.table(g_) if td else np.zeros((len(g_), C_)))
            infos = [ob.info() for ob in rec.obs]
            chain = guiding_chain(auxes, grids, infos)
            t_all += grids
            H_all += [c[0] for c in chain]
            F_all += [c[1] for c in chain]
            mdl_r = record_models[r] if record_models is not None else model
            laws += [mdl_r.law_record(a_, c[2][0]) for a_, c in zip(auxes, chain)]
            n_points.append([len(g) for g in grids])
            infos_all += infos
            if blocking:
                for k, ob in enumerate(rec.obs):
                    a_ = aux_laws_blocking(model, r, k, ob)
                    td = is_time_dependent(a_)
                    any_td |= td
                    tab_b.append(a_.table(grids[k]) if td else np.zeros((len(grids[k]), C_)))
                    v = np.zeros(d)
                    vo = np.atleast_1d(np.asarray(ob.v, dtype=np.float64))
                    v[:min(d, vo.size)] = vo[:d]
                    Ha, Fa, ca = artificial_obs_info(v, artificial_noise)
                    Ho, Fo, co = infos[k]
                    (h, f, c), = guiding_chain([a_], [grids[k]], [(Ha + Ho, Fa + Fo, ca + co)])
                    Hb_all.append(h)
                    Fb_all.append(f)
                    lawsb.append(mdl_r.law_record(a_, c[0]))
        if _engine is None and _ENGINE_FACTORY is not None:
            fac = _ENGINE_FACTORY
            _engine = lambda n_points: fac(model, n_points, precision, seed)  # noqa: E731
        if callable(_engine):  # test seam: an engine factory of the structure
            _engine = _engine(n_points)
        se = object.__new__(cls)
        se.__init__(model, n_points, precision=precision, seed=seed, device=device,
                    mapping=mapping, _engine=_engine)
        se._record_models = list(record_models) if record_models is not None else None
        se.upload_grid(np.concatenate(t_all))
        blaws = {}
        if blocking:
            blaws = dict(Hb=np.concatenate(Hb_all), Fb=np.concatenate(Fb_all),
                         lawsb=np.stack(lawsb))
        se.set_guiding(np.concatenate(H_all), np.concatenate(F_all), np.stack(laws), **blaws)
        if any_td:
            se.ens.upload_aux(L.LAW_PP, np.concatenate(tab_pp))
            if blocking:
                se.ens.upload_aux(L.LAW_PPB, np.concatenate(tab_b))
        se.set_observations(np.stack([packed(i[0]) for i in infos_all]),
                            np.stack([np.asarray(i[1], dtype=np.float64) for i in infos_all]),
                            np.array([float(i[2]) for i in infos_all]),
                            artificial_noise=artificial_noise)
        if init:
            _, ok = se.init_paths([rec.x0 for rec in recordings])
            if not ok.all():
                raise RuntimeError("init_paths failed")
        return se

    def num_recordings(self):
        return len(self.recordings)

    def record_model(self, r):
        """Recording r's target law (its own parameters when built from recordings)."""
        rm = getattr(self, "_record_models", None)
        return rm[r] if rm is not None else self.model

    def upload_grid(self, t):
        self.ens.upload_grid(t)

    def set_guiding(self, H, F, laws, Hb=None, Fb=None, lawsb=None, H_shared=False,
                    unit=L.U):
        """Upload the guiding terms of ``PP`` (and ``PPb``, the blocking laws with an
        artificial end observation, src/sampling_unit.jl:61-66) of ``unit``; the first
        upload also seeds the other unit (u° = deepcopy(u), src/sampling_pair.jl:51)."""
        self.ens.upload_law(unit, L.LAW_PP, H=H, F=F, laws=laws, H_shared=H_shared)
        if Hb is not None or Fb is not None or lawsb is not None:
            self.ens.upload_law(unit, L.LAW_PPB, H=Hb, F=Fb, laws=lawsb, H_shared=H_shared)

    def set_observations(self, Hobs, Fobs, cobs, artificial_noise=1e-11):
        """Information of the observation at every segment end (packed H, F, c) and the
        artificial noise of the blocking laws (src/sampling_unit.jl:57): enables
        ``set_obs`` / ``recompute_guiding_term`` on the device."""
        self.ens.upload_obs(Hobs, Fobs, cobs, artificial_noise)

    def init_paths(self, x0, Z=None, iter=None, salt=None, x0_prior=None, max_tries=1000):
        """``init_paths!`` (src/sampling_unit.jl:83-87) for every recording, then
        u° ← u (src/sampling_pair.jl:51).  ``x0``: per-recording start points (R × d).

        Like the reference, which repeats ``forward_guide!`` with a fresh ``x0 ~ x0_prior``
        until it succeeds, a recording whose draw fails is drawn again — with the next device
        normal stream (``iter + k``) and, when ``x0_prior`` (``k -> start point``) is given, a new
        start point — up to ``max_tries`` draws (the reference loops without a bound).
        Parity-mode normals ``Z`` are fixed inputs: no retry.  Without ``iter``/``salt`` every
        draw takes the next variables of the device stream counter.  Returns (ll, success)."""
        d = self.model.d
        x0 = np.asarray(x0, dtype=np.float64).reshape(-1, d)
        starts = self.ens.pt_off[self.ens.rec_seg0[:-1]]
        X = np.zeros((self.ens.P, d))
        X[starts] = x0
        self.ens.set_paths(L.U, X=X)
        auto = iter is None and salt is None
        it0, salt = _key(iter, 0xFFFF if salt is None and not auto else salt)
        ll, ok = self.ens.draw_unit(L.U, Z=Z, iter=it0, salt=salt)
        ll, ok = np.array(ll), np.array(ok)
        tries = 1
        while Z is None and not ok.all():
            if tries >= max_tries:
                raise RuntimeError(f"init_paths: {int((~ok).sum())} recording(s) still failing "
                                   f"after {max_tries} draws")
            if x0_prior is not None:
                X = self.ens.download_paths(L.U, 0)
                for r in np.nonzero(~ok)[0]:
                    X[starts[r]] = np.asarray(x0_prior(tries), dtype=np.float64).reshape(d)
                self.ens.set_paths(L.U, X=X)
            for r in np.nonzero(~ok)[0]:
                llr, okr = self.ens.draw_unit(L.U, int(r), int(r) + 1,
                                              iter=0 if auto else it0 + tries, salt=salt)
                ll[r], ok[r] = llr[0], okr[0]
            tries += 1
        self.ens.set_paths(L.UPROP, X=self.ens.download_paths(L.U, 0),
                           W=self.ens.download_paths(L.U, 1))
        return ll, ok

    # ---- path snapshots: the tutorials' `append!(paths, [deepcopy(rec.u.XX) for rec in
    # se.recordings])` (docs/src/tutorials/block_ensemble/inference.md:124), kept in HBM
    def reserve_snapshots(self, n_slots, XX=True, WW=False):
        self.ens.snapshot_reserve(n_slots, (1 if XX else 0) | (2 if WW else 0))

    def snapshot_paths(self, slot, mcmciter=0, unit=L.U):
        """deepcopy of every recording's ``unit.XX`` (and ``WW`` if reserved) into ``slot``."""
        self.ens.snapshot_take(slot, mcmciter, unit)

    def snapshot(self, slot, what=0):
        """Slot contents as the reference holds them: per recording, the list of per-segment
        paths (``Vector{Trajectory}`` x arrays), and the slot's MCMC iteration."""
        A, it = self.ens.snapshot_download(slot, what)
        out, p = [], 0
        for r in self.n_points:
            segs = []
            for n in r:
                segs.append(A[p:p + n])
                p += n
            out.append(segs)
        return out, it

    def snapshot_every(self, every, slot0=0):
        """Snapshots inside later :meth:`BlockEnsemble.mcmc_run` calls: u's paths after every
        iteration k with k % every == 0 go to slots slot0, slot0 + 1, … (a ring over the
        reserved slots), with no host round trip — the smoothing loop's `deepcopy(sp.u.XX)`
        every few iterations (docs/src/tutorials/biblock/smoothing.md:40-44).  0 turns it off."""
        self.ens.set_run_snapshots(every, slot0)

    def write_snapshots(self, path, s0=0, s1=None):
        """Stream slots [s0, s1) to ``path`` (DMTPATH1 format, include/dmt.h); read back with
        :func:`diffusionmcmctools_amd.read_snapshots`."""
        self.ens.snapshot_write(path, s0, self.ens_slots() if s1 is None else s1)

    def ens_slots(self):
        return getattr(self.ens, "_snap_slots", 0)

    def close(self):
        self.ens.close()


class SamplingPair:
    """``SamplingPair`` (src/sampling_pair.jl:33-57): ``u`` (accepted) and ``u°`` (``u_prop``)
    of one recording.

    Reference constructor: ``SamplingPair(aux_laws, recording, tts; aux_laws_blocking,
    artificial_noise)`` (src/sampling_pair.jl:40-54) — the containers of ONE recording (its own
    one-recording ensemble on the GPU, ``sp.se``), u° = deepcopy(u).  ``recording`` carries its
    target law ``P`` (``models.build_recording``); ``aux_laws`` is an auxiliary-law constructor
    ``AuxLaw(P, obs)`` such as ``models.FitzHughNagumoAux``.  The ensemble form
    ``SamplingPair(se, r)`` is the r-th recording of a :class:`SamplingEnsemble`."""

    def __init__(self, *args, **kw):
        if args and isinstance(args[0], SamplingEnsemble):
            self._init_view(*args)
            return
        se = SamplingEnsemble._from_reference_args(args[0], [args[1]], [args[2]], *args[3:],
                                                   _pair=True, **kw)
        self._init_view(se, 0)
        se.recordings[0] = self

    def _init_view(self, se, r):
        self.se, self.r = se, r
        self.u = SamplingUnit(se, r, L.U)
        self.u_prop = SamplingUnit(se, r, L.UPROP)

    def close(self):
        self.se.close()


class SamplingUnit:
    """``SamplingUnit`` (src/sampling_unit.jl:48-81) view: PP, PPb, WW, XX of one recording."""

    def __init__(self, se: SamplingEnsemble, r: int, unit: int):
        self.se, self.r, self.unit = se, r, unit

    def _rows(self):
        e = self.se.ens
        g0, g1 = e.rec_seg0[self.r], e.rec_seg0[self.r + 1]
        p0 = e.pt_off[g0]
        p1 = e.pt_off[g1 - 1] + e.npts[g1 - 1]
        return p0, p1, g0, g1

    def _split(self, A):
        p0, _, g0, g1 = self._rows()
        e = self.se.ens
        return [A[e.pt_off[g]:e.pt_off[g] + e.npts[g]] for g in range(g0, g1)]

    @property
    def XX(self):
        """Sampled trajectories, one (npts × d) array per segment."""
        return self._split(self.se.ens.download_paths(self.unit, 0))

    @property
    def WW(self):
        """Wiener trajectories (cumulative, as the reference holds them), per segment."""
        return self._split(self.se.ens.download_paths(self.unit, 1))

    def draw_proposal_path(self, Z=None, iter=None, salt=None):
        """``draw_proposal_path!(u::SamplingUnit)`` (src/sampling_unit.jl:118-120): fresh
        Wiener draw and guided solve of the whole recording.  Returns (success, ll)."""
        it, salt = _key(iter, salt)
        ll, ok = self.se.ens.draw_unit(self.unit, self.r, self.r + 1, Z=Z, iter=it, salt=salt)
        return bool(ok[0]), float(ll[0])

    # The unit's methods run on the handle's internal layout 0 (one terminal block per
    # recording over all its segments, ρ = 0 — the unit seen as one block).
    def recompute_guiding_term(self):
        """``GP.recompute_guiding_term!(u::SamplingUnit)`` (src/sampling_unit.jl:100-102): the
        guiding terms of ``u.PP`` over the whole recording, backward from its last
        observation (device filter)."""
        self.se.ens.recompute_guiding_term(0, self.r, self.r + 1, unit=self.unit)

    def loglikhd(self):
        """``GP.loglikhd(u::SamplingUnit)`` (src/sampling_unit.jl:109): the log-likelihood
        ``loglikhd(u.PP, u.XX)`` of the stored path (``loglikhd_obs`` at the start plus every
        segment's Girsanov sum) — a value; the unit is not modified."""
        e = self.se.ens
        e.loglikhd(0, self.unit, self.r, self.r + 1)
        what = L.BLK_LL if self.unit == L.U else L.BLK_LLPROP
        return float(e.get_block_state(0, what, self.r, self.r + 1)[0])


# ============================================================================ blocks
class _BlockRange:
    """Shared implementation: blocks [b0, b1) of a layout (a BlockEnsemble, one of its
    BlockCollections, or one BiBlock)."""

    def __init__(self, ens, layout, b0, b1, hist_len):
        self._ens, self._layout, self._b0, self._b1 = ens, layout, b0, b1
        self.ll_hist_len = hist_len

    @property
    def num_blocks(self):
        return self._b1 - self._b0

    def _call(self, name, *a, **k):
        return getattr(self._ens, name)(self._layout, self._b0, self._b1, *a, **k)

    def _call_what(self, name, what, **k):
        # engine methods whose selector precedes the block range: (layout, what, b0, b1)
        return getattr(self._ens, name)(self._layout, what, self._b0, self._b1, **k)

    # ---- imputation (biblock.jl:78-106, block_collection.jl:46, block_ensemble.jl:50)
    def draw_proposal_path(self, Z=None, iter=None, salt=None):
        """pCN proposal under the accepted law into u°, ll° along the way.  Returns the
        per-block success flags.  Normals: the next ones of the device stream counter, or the
        stream keyed by an explicit ``iter``/``salt``, or ``Z`` (steps × m, whole ensemble)."""
        it, salt = _key(iter, salt)
        # the flags are read only if used: the draw may wait for (and fuse with) the
        # accept_reject that follows (include/dmt.h, deferred draws)
        return self._call("draw_proposal", Z=Z, iter=it, salt=salt, want_success="lazy")

    # ---- accept / reject (biblock.jl:121-127)
    def accept_reject_proposal_path(self, mcmciter, E=None, salt=None):
        """MH decision per block: E > −(ll° − ll), E ~ Exp(1) (the device stream counter —
        the key of the draw this decision follows —, the stream keyed by (``mcmciter``,
        ``salt``) when ``salt`` is given, or ``E``); swap_paths!, set_accepted!, save_ll!,
        swap_ll! in the reference order.  Returns the per-block decisions."""
        return self._call("accept_reject", mcmciter, E=E,
                          salt=L.RNG_AUTO if salt is None else int(salt), want_acc=True)

    def set_accepted(self, i, v):
        self._call("set_accepted", i, v)

    # ---- swaps (biblock.jl:148-208)
    def swap_paths(self):
        self._call_what("swap", L.SWAP_XX | L.SWAP_WW)

    def swap_XX(self):
        self._call_what("swap", L.SWAP_XX)

    def swap_WW(self):
        self._call_what("swap", L.SWAP_WW)

    def swap_PP(self):
        """PP (and, for non-terminal blocks, the P_last law) of the block's segments."""
        self._call_what("swap", L.SWAP_PP)

    def swap_ll(self):
        self._call_what("swap", L.SWAP_LL)

    # ---- log-likelihoods (block.jl:138-152, biblock.jl:233-249, block_collection.jl:166-197)
    def loglikhd(self):
        self._call_what("loglikhd", L.U)

    def loglikhd_prop(self):
        self._call_what("loglikhd", L.UPROP)

    def recompute_path(self, skip=0):
        """``recompute_path!(bb.b°, bb.b.WW; skip)`` (src/block.jl:155-187): u° re-solved
        under u°'s laws with u's Wiener path; ll° stored.  Returns per-block success."""
        return self._call("recompute_path", skip=skip, want_success=True)

    def set_obs(self):
        """``GP.set_obs!`` (src/biblock.jl:273-280): freeze the accepted end point of every
        non-terminal block as the artificial observation of its P_last law."""
        self._call("set_obs")

    def recompute_guiding_term(self, only=None):
        """``GP.recompute_guiding_term!`` (device backward filter of the blocks' laws,
        src/block.jl:102-110): with no flag the guiding terms of both the accepted and the
        proposal laws, b then b° (src/biblock.jl:288-291, src/block_collection.jl:208-210,
        src/block_ensemble.jl:199-200); ``only="P_only"`` the accepted laws only
        (``Val(:P_only)``, i.e. ``recompute_guiding_term!(bb.b)``), ``only="P°_only"`` the
        proposal laws only (``Val(:P°_only)``, ``recompute_guiding_term!(bb.b°)``;
        src/block_collection.jl:212-221)."""
        units = _RGT_ONLY.get(only)
        if units is None:
            raise ValueError(f"only must be one of {sorted(k for k in _RGT_ONLY if k)} or None")
        for unit in units:
            self._call("recompute_guiding_term", unit=unit)

    def equalize_obs_params(self):
        """``GP.equalize_obs_params!(bb)`` (src/biblock.jl:375-387): make u°'s observation
        parameters those of u.  On the device a recording's observations (``dmt_upload_obs``:
        the observed values, their noise, the artificial P_last observation) are stored ONCE
        and read by the laws of both u and u°, so they cannot differ and there is nothing to
        copy; returns the per-block critical-change flags the reference's call would yield
        here (all False)."""
        return np.zeros(self.num_blocks, dtype=bool)

    def find_W_for_X(self):
        """``find_W_for_X!`` (src/block.jl:118-131): u.WW ← the Wiener increments that reproduce
        u.XX under the accepted laws u.PP (+ P_last) — DD.invsolve!, parallel in time."""
        self._call("find_W_for_X")

    def save_ll(self, i):
        self._call("save_ll", i)

    def set_ll(self, i, v, unit=L.U):
        """``set_ll!(b, i, v)`` (src/block.jl:82-86) on ``bb.b`` (``unit=U``) or ``bb.b°``:
        ll_history[i] = v (a scalar or one value per block)."""
        self._ens.set_ll(self._layout, unit, self._b0, self._b1, i, v)

    def accept_reject_proposal_param(self, mcmciter, theta, theta_prop, E=None, rng=None):
        """The tutorials' parameter Metropolis–Hastings step
        (docs/src/tutorials/pnames/inference_with_biblock.md:17-25): accept θ° when
        E > −(ll° − ll) with the range's total log-likelihoods (``fetch_ll``/``fetch_ll°``),
        E ~ Exp(1) (``E`` given, or drawn from ``rng``); on acceptance swap_XX!, swap_PP!;
        save_ll! of both units; swap_ll! on acceptance.  Returns (accepted, θ or θ°)."""
        llp, ll = self.fetch_ll_prop(), self.fetch_ll()
        if E is None:
            E = (rng if rng is not None else np.random.default_rng()).exponential(1.0)
        accepted = bool(E > -(llp - ll))
        if accepted:
            self._call_what("swap", L.SWAP_XX | L.SWAP_PP)
        self.save_ll(mcmciter)
        if accepted:
            self.swap_ll()
        return accepted, (np.array(theta_prop, copy=True) if accepted else np.array(theta, copy=True))

    # BiBlock / BlockCollection sums are this rank's (src/block_collection.jl:144,156);
    # BlockEnsemble overrides _global: with a communicator its fetch_ll is over every rank
    _global = False

    def fetch_ll(self):
        """Σ ll over the blocks (deterministic pairwise tree)."""
        return self._call("fetch_ll", local=not self._global)[0]

    def fetch_ll_prop(self):
        return self._call("fetch_ll", local=not self._global)[1]

    # ---- state
    @property
    def ll(self):
        return self._call_what("get_block_state", L.BLK_LL)

    @property
    def ll_prop(self):
        return self._call_what("get_block_state", L.BLK_LLPROP)

    def _hist(self, what):
        return self._call_what("get_block_state", what, hist_len=self.ll_hist_len)

    @property
    def ll_history(self):
        return self._hist(L.BLK_LL_HIST)

    @property
    def ll_prop_history(self):
        return self._hist(L.BLK_LLPROP_HIST)

    @property
    def accpt_history(self):
        return self._hist(L.BLK_ACC_HIST).astype(bool)

    def ll_of_accepted(self, i):
        """Per block: ll° history if iteration i was accepted, else ll history
        (src/biblock.jl:221-223)."""
        acc = self.accpt_history[i - 1]
        return np.where(acc, self.ll_prop_history[i - 1], self.ll_history[i - 1])

    def accpt_rate(self, rng):
        """Per block: mean of accpt_history over the 1-based iterations in ``rng``
        (src/biblock.jl:230)."""
        idx = np.asarray(list(rng), dtype=np.int64) - 1
        return self.accpt_history[idx].sum(axis=0) / len(idx)

    # ---- parameter updates (biblock.jl:334-375, block_collection.jl:306-334)
    def set_proposal_law(self, theta=None, H=None, F=None, laws=None, Hb=None, Fb=None,
                         lawsb=None, H_shared=False, skip=0, critical_change=None):
        """``set_proposal_law!(bb, θ°, pnames, critical_change; skip)``.

        With ``theta`` ({parameter name or DMT_PAR_* index: value}; names as in
        ``_lib.PAR_FHN`` / ``PAR_LORENZ``, OU indices Θ[i][j] = i·d + j, μ[i] = d² + i) it runs
        on the device: u°'s laws ← u's with θ° set and the auxiliary law re-derived,
        ``recompute_guiding_term!(b°)`` where that changed, then ``recompute_path!(b°, b.WW)``;
        returns (success, critical) per block.  Without ``theta`` it installs host-made tables
        in u° (ensemble-wide upload) and re-solves; returns the success flags.
        ``critical_change=False`` keeps u°'s guiding term unless equalizing u°'s law with u's
        changed its auxiliary law (src/biblock.jl:340-342)."""
        if theta is not None:
            return self._call("set_proposal_law", _param_indices(self._ens, theta), skip=skip,
                              critical_change=critical_change)
        if H is not None or F is not None or laws is not None:
            self._ens.upload_law(L.UPROP, L.LAW_PP, H=H, F=F, laws=laws, H_shared=H_shared)
        if Hb is not None or Fb is not None or lawsb is not None:
            self._ens.upload_law(L.UPROP, L.LAW_PPB, H=Hb, F=Fb, laws=lawsb, H_shared=H_shared)
        return self.recompute_path(skip=skip)

    def mcmc_step(self, mcmciter, salt=None):
        """``draw_proposal_path!`` + ``accept_reject_proposal_path!(·, mcmciter)`` +
        ``fetch_ll`` fused into one call (device RNG: the stream counter, or the stream keyed
        by (``mcmciter``, ``salt``)).  Returns (ll, ll°, n_accepted)."""
        return self._call("mcmc_step", mcmciter, salt=L.RNG_AUTO if salt is None else int(salt),
                          local=not self._global)

    def mcmc_run(self, iter0, n_iter, salt=None):
        """``n_iter`` consecutive :meth:`mcmc_step` iterations starting at ``iter0``, queued on
        the device without host round trips; returns an (n_iter, 3) array of (fetch_ll,
        fetch_ll°, accepted count) — the sampling loop of
        docs/src/tutorials/biblock/smoothing.md:40-44.  Without ``salt`` it draws exactly what
        the loop of counter-keyed :meth:`draw_proposal_path` / :meth:`accept_reject_proposal_path`
        calls would."""
        return self._call("mcmc_run", iter0, n_iter,
                          salt=L.RNG_AUTO if salt is None else int(salt), local=not self._global)


# recompute_guiding_term! flags (src/block_collection.jl:208-221) → units, in call order
_RGT_ONLY = {None: (L.U, L.UPROP), "P_only": (L.U,), "P°_only": (L.UPROP,),
             "Pprop_only": (L.UPROP,)}


def _param_indices(ens, theta):
    """Map parameter names to DMT_PAR_* indices for the ensemble's model."""
    names = {L.MODEL_FHN: L.PAR_FHN, L.MODEL_LORENZ: L.PAR_LORENZ}.get(int(ens.model), {})
    out = {}
    for k, v in theta.items():
        if isinstance(k, str):
            if k not in names:
                raise KeyError(f"unknown parameter {k!r} for model {ens.model}")
            k = names[k]
        out[int(k)] = float(v)
    return out


def _pair_layout(sp, ranges, rhos, ll_hist_len):
    """A layout holding only recording ``sp.r``'s blocks ``ranges`` (the last one terminal):
    the storage of the reference's stand-alone ``BiBlock(sp, …)`` / ``BlockCollection(sp, …)``,
    whose blocks are views into that pair's containers (src/block.jl:66-72)."""
    se = sp.se
    nseg = len(se.n_points[sp.r])
    rr = [_as_range(x) for x in ranges]
    for x in rr:
        if not (0 <= x.start < x.stop <= nseg):
            raise ValueError(f"block range {x} outside recording {sp.r}'s {nseg} segments")
    n_blocks = [0] * se.num_recordings()
    n_blocks[sp.r] = len(rr)
    last = [1 if i == len(rr) - 1 else 0 for i in range(len(rr))]
    layout = se.ens.create_layout(n_blocks, [x.start for x in rr], [x.stop - 1 for x in rr],
                                  last, [float(v) for v in rhos], hist_len=int(ll_hist_len))
    return layout, rr, last


def _as_range(x):
    return range(x.start, x.stop) if isinstance(x, range) else range(x[0], x[1] + 1)


class Block:
    """``Block{L}`` (src/block.jl:49-79): the view ``bb.b`` (unit u, the accepted path and
    laws) or ``bb.b°`` (``bb.b_prop``, unit u°) of a :class:`BiBlock` onto the segments of its
    recording.  ``ll`` reads and assigns the block's log-likelihood (``bb.b°.ll - bb.b.ll`` in
    the reference's parameter step, docs/src/tutorials/biblock/inference.md:44), ``ll_history``
    its history, ``XX`` / ``WW`` download the block's segments (reference layout, resolving
    swaps; src/block.jl:71-72), ``is_last`` is the type parameter L."""

    def __init__(self, bb, unit):
        self.bb, self.unit = bb, unit

    @property
    def is_last(self):
        return self.bb.is_last

    def _state(self, hist=False):
        u = self.unit == L.U
        return (L.BLK_LL_HIST if u else L.BLK_LLPROP_HIST) if hist else (L.BLK_LL if u else L.BLK_LLPROP)

    @property
    def ll(self):
        bb = self.bb
        return float(bb._ens.get_block_state(bb._layout, self._state(), bb._b0, bb._b1)[0])

    @ll.setter
    def ll(self, v):
        bb = self.bb
        bb._ens.set_block_state(bb._layout, self._state(), bb._b0, bb._b1,
                                np.array([float(v)]))

    @property
    def ll_history(self):
        bb = self.bb
        return bb._ens.get_block_state(bb._layout, self._state(True), bb._b0, bb._b1,
                                       hist_len=bb.ll_hist_len)[:, 0]

    def _segments(self, what):
        bb, e = self.bb, self.bb._ens
        A = e.download_paths(self.unit, what)
        g0 = int(e.rec_seg0[bb.rec])
        return [A[e.pt_off[g]:e.pt_off[g] + e.npts[g]]
                for g in range(g0 + bb.segments.start, g0 + bb.segments.stop)]

    @property
    def XX(self):
        return self._segments(0)

    @property
    def WW(self):
        return self._segments(1)


class BiBlock(_BlockRange):
    """``BiBlock{L}`` (src/biblock.jl:42-63): one block b / b° with pCN memory ρ.

    Reference constructor: ``BiBlock(sp, range, rho=0.0, last_block=False, ll_hist_len=0)``
    (src/biblock.jl:48-62) — a block over segments ``range`` (0-based, half-open) of the
    recording of SamplingPair ``sp``.  The BlockEnsemble / BlockCollection constructors make
    their blocks with the internal form ``BiBlock(engine, layout, b, …)``."""

    def __init__(self, *args, **kw):
        if args and isinstance(args[0], SamplingPair):
            self._init_ref(*args, **kw)
        else:
            self._init_view(*args, **kw)

    def _init_ref(self, sp, range_, rho=0.0, last_block=False, ll_hist_len=0):
        if not last_block and len(_as_range(range_)) < 2:
            raise ValueError("a non-terminal BiBlock needs >= 2 segments (src/block.jl:66,178)")
        se = sp.se
        n_blocks = [0] * se.num_recordings()
        n_blocks[sp.r] = 1
        x = _as_range(range_)
        layout = se.ens.create_layout(n_blocks, [x.start], [x.stop - 1], [1 if last_block else 0],
                                      [float(rho)], hist_len=int(ll_hist_len))
        self._init_view(se.ens, layout, 0, int(ll_hist_len), last_block, rho, x, sp.r,
                        se.record_model(sp.r))

    def _init_view(self, ens, layout, b, hist_len, is_last, rho, segments, rec=0, model=None):
        super().__init__(ens, layout, b, b + 1, hist_len)
        self.is_last, self.rho, self.segments = bool(is_last), float(rho), segments
        self.rec, self.model = int(rec), model
        # bb.b / bb.b° (src/biblock.jl:43-46): the accepted and the proposal Block views
        self.b = Block(self, L.U)
        self.b_prop = Block(self, L.UPROP)

    def fetch_ll(self):
        return float(self.ll[0])

    def fetch_ll_prop(self):
        return float(self.ll_prop[0])

    def ll_of_accepted(self, i):
        return float(super().ll_of_accepted(i)[0])

    def accpt_rate(self, rng):
        return float(super().accpt_rate(rng)[0])


class BlockCollection(_BlockRange):
    """``BlockCollection`` (src/block_collection.jl:19-38): the blocks of one recording; the
    last one is terminal (``BiBlock{true}``).

    Reference constructor: ``BlockCollection(sp, ranges, rho=0.0, ll_hist_len=0)``
    (src/block_collection.jl:22-30): blocks over ``ranges`` (0-based, half-open) of SamplingPair
    ``sp``'s recording, ``rho`` a scalar or one per block.  ``BlockEnsemble`` makes its
    collections with the internal form ``BlockCollection(engine, layout, b0, blocks, …)``."""

    def __init__(self, *args, **kw):
        if args and isinstance(args[0], SamplingPair):
            self._init_ref(*args, **kw)
        else:
            self._init_view(*args, **kw)

    def _init_ref(self, sp, ranges, rho=0.0, ll_hist_len=0):
        n = len(ranges)
        rhos = list(rho) if isinstance(rho, (list, tuple, np.ndarray)) else [rho] * n
        layout, rr, last = _pair_layout(sp, ranges, rhos, ll_hist_len)
        ens = sp.se.ens
        blocks = [BiBlock(ens, layout, b, int(ll_hist_len), last[b], rhos[b], rr[b], sp.r,
                          sp.se.record_model(sp.r)) for b in range(n)]
        self._init_view(ens, layout, 0, blocks, int(ll_hist_len))

    def _init_view(self, ens, layout, b0, blocks, hist_len):
        super().__init__(ens, layout, b0, b0 + len(blocks), hist_len)
        self.blocks = blocks


class BlockEnsemble(_BlockRange):
    """``BlockEnsemble(se, ranges, ρρ=0.0, ll_hist_len=0)`` (src/block_ensemble.jl:17-38).

    ``ranges[r]`` lists recording r's blocks as contiguous ranges of its segments covering
    it in order; ``rho`` a scalar, or per recording (scalar or per block)."""

    def __init__(self, se: SamplingEnsemble, ranges, rho=0.0, ll_hist_len=0):
        R = se.num_recordings()
        # ll_hist_len: a scalar or one per recording (_vec_me, src/block_ensemble.jl:27-28);
        # the device layout keeps one history length, the longest
        if isinstance(ll_hist_len, (list, tuple, np.ndarray)):
            ll_hist_len = int(max(ll_hist_len)) if len(ll_hist_len) else 0
        if len(ranges) != R:
            raise ValueError(f"ranges needs one entry per recording ({R})")
        rho_r = rho if isinstance(rho, (list, tuple, np.ndarray)) else [rho] * R
        n_blocks, sf, sl, last, rhos = [], [], [], [], []
        for r, rr in enumerate(ranges):
            rr = [range(x.start, x.stop) if isinstance(x, range) else range(x[0], x[1] + 1)
                  for x in rr]
            nseg = len(se.n_points[r])
            pos = 0
            for x in rr:
                if x.start != pos or x.stop <= x.start:
                    raise ValueError(f"recording {r}: ranges must tile its {nseg} segments")
                pos = x.stop
            if pos != nseg:
                raise ValueError(f"recording {r}: ranges must tile its {nseg} segments")
            rb = rho_r[r]
            rb = list(rb) if isinstance(rb, (list, tuple, np.ndarray)) else [rb] * len(rr)
            n_blocks.append(len(rr))
            for i, x in enumerate(rr):
                sf.append(x.start)
                sl.append(x.stop - 1)
                last.append(1 if i == len(rr) - 1 else 0)
                rhos.append(float(rb[i]))
        ens = se.ens
        layout = ens.create_layout(n_blocks, sf, sl, last, rhos, hist_len=ll_hist_len)
        nb = len(sf)
        super().__init__(ens, layout, 0, nb, ll_hist_len)
        self._global = True
        self.se = se
        self.recordings = []
        b = 0
        for r in range(R):
            blocks = []
            for _ in range(n_blocks[r]):
                blocks.append(BiBlock(ens, layout, b, ll_hist_len, last[b], rhos[b],
                                      range(sf[b], sl[b] + 1), r, se.record_model(r)))
                b += 1
            self.recordings.append(BlockCollection(ens, layout, b - len(blocks), blocks,
                                                   ll_hist_len))

    def num_recordings(self):
        return len(self.recordings)

    def ll_of_accepted(self, i):
        flat = super().ll_of_accepted(i)
        return [flat[c._b0:c._b1] for c in self.recordings]

    def accpt_rate(self, rng):
        flat = super().accpt_rate(rng)
        return [flat[c._b0:c._b1] for c in self.recordings]
