"""Parameter-name bookkeeping of ``set_proposal_law!`` (host side, no device work).

Restates /root/reference/src/param_names_collections.jl: which entries of the MCMC parameter
vector θ° go to which named parameter of the target laws (``updt``), of the auxiliary laws
(``updt_aux``) and of the observations (``updt_obs``) of every law collection of a block
(``PP``, ``P_last``, ``P_excl``, ``Pb_excl``), per block of a recording and per recording.
Pairs ``idx => name`` are Python tuples ``(idx, name)`` with the reference's 1-based ``idx``
into θ°.  ``set_proposal_law`` (functions.py) reads them to call the device.

``AllObservations`` is a minimal stand-in for the part of ObservationSchemes'
``AllObservations`` the tutorials use (docs/src/tutorials/block_ensemble/inference.md:33-45:
``add_recordings!``, ``add_dependency!``, ``initialize``, ``param_depend_rev``,
``obs_depend_rev``); ObservationSchemes itself is upstream and not vendored.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from .models import canonical_name


def _var_names(model):
    return model.variable_names() if model is not None else ()


@dataclass
class ParamNamesUnit:
    """``ParamNamesUnit`` (src/param_names_collections.jl:49-73) of a collection of ``n_laws``
    laws of one target model (the auxiliary laws share the target's variable names, as
    ``DD.var_parameter_names(::FitzHughNagumoAux) = (:γ,)`` in the tutorials' preamble)."""
    var: tuple
    var_aux: list
    updt: tuple
    updt_aux: list
    updt_obs: list

    @classmethod
    def build(cls, model, n_laws, θnames, pdep, odeps):
        θnames = [canonical_name(n) for n in θnames]
        # find_θ_names_for_MCMC_update (:86-100)
        updt = tuple((θnames.index(canonical_name(g)) + 1, canonical_name(p))
                     for g, p in pdep if canonical_name(g) in θnames)
        aux_names = _var_names(model)
        # find_θ_aux_names_for_MCMC_update (:108-113)
        updt_aux = [tuple(p for p in updt if p[1] in aux_names) for _ in range(n_laws)]
        # find_θ_obs_idx_for_MCMC_update (:125-142)
        updt_obs = [tuple((θnames.index(canonical_name(g)) + 1, i)
                          for g, i in odep if canonical_name(g) in θnames) for odep in odeps]
        in_updt = [p[1] for p in updt]
        # find_var_names_not_in_MCMC_update (:150-154)
        var = tuple(p for p in _var_names(model) if p not in in_updt) if n_laws > 0 else ()
        # find_var_aux_names_not_in_MCMC_update (:163-171)
        var_aux = [tuple(p for p in aux_names if p not in [q[1] for q in ua]) for ua in updt_aux]
        return cls(var, var_aux, updt, updt_aux, updt_obs)


@dataclass
class ParamNamesBlock:
    """``ParamNamesBlock`` (src/param_names_collections.jl:204-230) of a block view ``b``
    (``bb.b``): ``PP`` over the block's regular laws, ``P_last`` its artificial last law,
    ``P_excl`` the regular law replaced by it, ``Pb_excl`` the other blocking laws."""
    PP: ParamNamesUnit
    P_last: ParamNamesUnit
    P_excl: ParamNamesUnit
    Pb_excl: ParamNamesUnit

    def __init__(self, b, θnames, pdep, odeps):
        bb = b.bb
        seg = bb.segments
        # _idx_split (:222-230): i1 = PP's segments, i2 = the last one of a non-terminal block
        i1 = list(seg) if bb.is_last else list(seg)[:-1]
        i2 = [] if bb.is_last else [seg[-1]]
        model = bb.model
        odeps = list(odeps)
        self.PP = ParamNamesUnit.build(model, len(i1), θnames, pdep, [odeps[i] for i in i1])
        self.P_last = ParamNamesUnit.build(model, len(i2), θnames, pdep, [() for _ in i2])
        self.P_excl = ParamNamesUnit.build(model, len(i2), θnames, pdep, [odeps[i] for i in i2])
        self.Pb_excl = ParamNamesUnit.build(model, len(i1), θnames, pdep, [() for _ in i1])


class ParamNamesRecording:
    """``ParamNamesRecording(bc, θnames, pdep, odeps)`` (src/param_names_collections.jl:249-257):
    one :class:`ParamNamesBlock` per block of a BlockCollection."""

    def __init__(self, bc, θnames, pdep, odeps):
        self.blocks = [ParamNamesBlock(bb.b, θnames, pdep, odeps) for bb in bc.blocks]


class ParamNamesAllObs:
    """``ParamNamesAllObs(be, θnames, all_obs)`` (src/param_names_collections.jl:274-288)."""

    def __init__(self, be, θnames, all_obs):
        self.recordings = [ParamNamesRecording(be.recordings[i], θnames,
                                               all_obs.param_depend_rev[i],
                                               all_obs.obs_depend_rev[i])
                           for i in range(len(be.recordings))]


@dataclass
class AllObservations:
    """What the tutorials use of ObservationSchemes' ``AllObservations``: recordings, shared
    parameters (``add_dependency``) and, after ``initialize``, per recording the list of
    ``(MCMC name, law parameter name)`` pairs (``param_depend_rev``) and per observation the
    observation-parameter pairs (``obs_depend_rev``; the tutorials' observations have none).
    Unshared variable parameter p of recording k is named ``REC<k>_<p>`` (1-based k), as
    ``:REC1_γ`` in docs/src/tutorials/block_collection/inference.md:80."""
    recordings: list = field(default_factory=list)
    dependencies: dict = field(default_factory=dict)
    param_depend_rev: list = field(default_factory=list)
    obs_depend_rev: list = field(default_factory=list)

    def num_recordings(self):
        return len(self.recordings)

    def add_recording(self, rec):
        self.recordings.append(rec)

    def add_recordings(self, recs):
        self.recordings.extend(recs)

    def add_dependency(self, dep):
        """``dep``: {shared name: [(recording k (1-based), law parameter name), …]}."""
        for g, pairs in dict(dep).items():
            self.dependencies[canonical_name(g)] = [(int(k), canonical_name(p)) for k, p in pairs]

    def initialize(self):
        shared = {(k, p): g for g, pairs in self.dependencies.items() for k, p in pairs}
        self.param_depend_rev = []
        for k, rec in enumerate(self.recordings, start=1):
            names = [(shared.get((k, p), f"REC{k}_{p}"), p) for p in _var_names(rec.P)]
            self.param_depend_rev.append(names)
        self.obs_depend_rev = [[() for _ in rec.obs] for rec in self.recordings]
        return self, None

    def set_parameters(self, theta):
        for name, v in dict(theta).items():
            name = canonical_name(name)
            for rec, deps in zip(self.recordings, self.param_depend_rev):
                for g, p in deps:
                    if g == name:
                        rec.P.set_param(p, v)
