"""The reference's exported generic functions, as module-level Python functions.

DiffusionMCMCTools.jl is driven through free functions dispatched on the container type
(exports at /root/reference/src/DiffusionMCMCTools.jl:28-60; GuidedProposals' ``GP.set_obs!``,
``GP.recompute_guiding_term!``, ``GP.loglikhd`` extended at src/biblock.jl:273-291,
src/block_collection.jl:198-221, src/sampling_unit.jl:100-109).  The same names here (``!``
dropped, ``°`` spelled ``_prop``, ``GP.`` functions under :data:`GP`) take the same objects
— :class:`~.api.BiBlock`, its views ``bb.b`` / ``bb.b_prop``, :class:`~.api.BlockCollection`,
:class:`~.api.BlockEnsemble`, :class:`~.api.SamplingUnit` — so a caller's loop reads like the
reference tutorials, e.g. docs/src/tutorials/biblock/inference.md:44-49::

    def accept_reject_proposal_param(bb, mcmciter, θ, θ°):
        accepted = rng.exponential(1.0) > -(bb.b_prop.ll - bb.b.ll)
        accepted and swap_XX(bb)
        accepted and swap_PP(bb)
        save_ll(bb, mcmciter)
        accepted and swap_ll(bb)
        return accepted, (θ° if accepted else θ).copy()

Every call is one libdmt C-ABI call over the blocks the object covers (no per-segment
calls); results are those of the methods in api.py.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .api import BiBlock, Block, BlockCollection, BlockEnsemble, SamplingUnit, _BlockRange
from .models import canonical_name

__all__ = ["draw_proposal_path", "accept_reject_proposal_path", "loglikhd", "loglikhd_prop",
           "recompute_path", "find_W_for_X", "fetch_ll", "fetch_ll_prop", "save_ll", "set_ll",
           "set_accepted", "swap_paths", "swap_XX", "swap_WW", "swap_PP", "swap_ll",
           "ll_of_accepted", "accpt_rate", "set_proposal_law", "num_recordings", "Val", "GP"]


def _blocks(x, what):
    if not isinstance(x, _BlockRange):
        raise TypeError(f"{what}: expected a BiBlock, BlockCollection or BlockEnsemble, got "
                        f"{type(x).__name__}")
    return x


def _range_of(b: Block):
    bb = b.bb
    return bb._ens, bb._layout, bb._b0, bb._b1


# ------------------------------------------------------------------ imputation and MH
def draw_proposal_path(x, **kw):
    """``draw_proposal_path!`` of a SamplingUnit (src/sampling_unit.jl:118-120; returns
    (success, ll)) or of a BiBlock / BlockCollection / BlockEnsemble (src/biblock.jl:78-92,
    src/block_collection.jl:46, src/block_ensemble.jl:50)."""
    if isinstance(x, SamplingUnit):
        return x.draw_proposal_path(**kw)
    _blocks(x, "draw_proposal_path").draw_proposal_path(**kw)


def accept_reject_proposal_path(x, mcmciter, **kw):
    """``accept_reject_proposal_path!(x, mcmciter)`` (src/biblock.jl:121-127)."""
    return _blocks(x, "accept_reject_proposal_path").accept_reject_proposal_path(mcmciter, **kw)


def loglikhd(x):
    """``loglikhd!(b)`` of a Block view (src/block.jl:152) or of blocks
    (``loglikhd!(bb)`` = the accepted b, src/biblock.jl:240)."""
    if isinstance(x, Block):
        e, lay, b0, b1 = _range_of(x)
        e.loglikhd(lay, x.unit, b0, b1)
        return
    _blocks(x, "loglikhd").loglikhd()


def loglikhd_prop(x):
    """``loglikhd°!(x)`` (src/biblock.jl:248, src/block_collection.jl:132)."""
    _blocks(x, "loglikhd_prop").loglikhd_prop()


def recompute_path(x, WW=None, skip=0):
    """``recompute_path!(bb.b°, bb.b.WW; skip)`` (src/block.jl:159-187, called by
    set_proposal_law! at src/biblock.jl:343): u° re-solved under its laws with u's Wiener
    path.  ``x`` is the proposal view ``bb.b_prop`` (``WW``, if given, must be ``bb.b.WW`` — the
    only Wiener path the reference passes) or a block range (the same for every block)."""
    if isinstance(x, Block):
        if x.unit != L.UPROP:
            raise ValueError("recompute_path: the device re-solves the proposal b° with b.WW "
                             "(src/biblock.jl:343); pass bb.b_prop")
        return x.bb.recompute_path(skip=skip)
    return _blocks(x, "recompute_path").recompute_path(skip=skip)


def find_W_for_X(x):
    """``find_W_for_X!`` (src/block.jl:118-131; BiBlock :300 = of ``bb.b``)."""
    if isinstance(x, Block):
        if x.unit != L.U:
            raise ValueError("find_W_for_X: the reference calls it on the accepted b "
                             "(src/biblock.jl:300)")
        x = x.bb
    _blocks(x, "find_W_for_X").find_W_for_X()


# ------------------------------------------------------------------ log-likelihood bookkeeping
def fetch_ll(x):
    """``fetch_ll`` (src/block_collection.jl:144, src/block_ensemble.jl:140)."""
    return _blocks(x, "fetch_ll").fetch_ll()


def fetch_ll_prop(x):
    """``fetch_ll°`` (src/block_collection.jl:156, src/block_ensemble.jl:152)."""
    return _blocks(x, "fetch_ll_prop").fetch_ll_prop()


def save_ll(x, i):
    """``save_ll!(x, i)``: of a Block view ``ll_history[i] = ll`` (src/block.jl:94), of blocks
    both b and b° (src/biblock.jl:256-259)."""
    if isinstance(x, Block):
        set_ll(x, i, x.ll)
        return
    _blocks(x, "save_ll").save_ll(i)


def set_ll(b, i, v):
    """``set_ll!(b, i, v)`` (src/block.jl:86) of a Block view."""
    if not isinstance(b, Block):
        raise TypeError("set_ll: expected a Block view (bb.b or bb.b_prop)")
    b.bb.set_ll(i, v, unit=b.unit)


def set_accepted(bb, i, v):
    """``set_accepted!(bb, i, v)`` (src/biblock.jl:135)."""
    _blocks(bb, "set_accepted").set_accepted(i, v)


def swap_paths(x):
    _blocks(x, "swap_paths").swap_paths()


def swap_XX(x):
    _blocks(x, "swap_XX").swap_XX()


def swap_WW(x):
    _blocks(x, "swap_WW").swap_WW()


def swap_PP(x):
    _blocks(x, "swap_PP").swap_PP()


def swap_ll(x):
    _blocks(x, "swap_ll").swap_ll()


def ll_of_accepted(x, i):
    """``ll_of_accepted(x, i)`` (src/biblock.jl:222-224, broadcasts)."""
    return _blocks(x, "ll_of_accepted").ll_of_accepted(i)


def accpt_rate(x, rng):
    """``accpt_rate(x, range)`` (src/biblock.jl:232): ``rng`` = the 1-based iterations, e.g.
    ``range(i - 99, i + 1)`` for Julia's ``(i-99):i``."""
    return _blocks(x, "accpt_rate").accpt_rate(rng)


def num_recordings(x):
    return x.num_recordings()


# ------------------------------------------------------------------ parameter updates
def _get(o, k):
    return o[k] if isinstance(o, dict) else getattr(o, k)


def _pairs(pn_block):
    """Every (θ° index, law parameter name) pair a block's ``ParamNamesBlock`` (or the
    tutorials' hand-made NamedTuple) updates, over its four law collections and their
    auxiliary laws (DD.set_parameters!(bb.b°.PP / P_last / P_excl / Pb_excl, θ°, pnames.…),
    src/biblock.jl:366-369)."""
    out = {}
    for coll in ("PP", "P_last", "P_excl", "Pb_excl"):
        u = _get(pn_block, coll)
        obs = _get(u, "updt_obs") if (isinstance(u, dict) and "updt_obs" in u) or hasattr(u, "updt_obs") else ()
        if any(len(list(o)) for o in obs):
            raise NotImplementedError(
                "set_proposal_law: observation parameters (updt_obs) are not updated on the "
                "device; the observations are uploaded once (dmt_upload_obs)")
        pairs = list(_get(u, "updt"))
        for ua in _get(u, "updt_aux"):
            pairs += list(ua)
        for idx, name in pairs:
            name = canonical_name(name)
            if out.get(name, idx) != idx:
                raise ValueError(f"parameter {name} is updated from two entries of θ°")
            out[name] = int(idx)
    return out


def _theta_map(pn_block, θ):
    θ = np.atleast_1d(np.asarray(θ, dtype=np.float64))
    return {name: float(θ[idx - 1]) for name, idx in _pairs(pn_block).items()}


def set_proposal_law(x, θ_prop, pnames, critical_change=None, skip=0):
    """``set_proposal_law!(x, θ°, pnames, critical_change; skip)`` (src/biblock.jl:334-344,
    src/block_collection.jl:264-276, src/block_ensemble.jl:242-255): u°'s laws ← u's with the
    parameters ``pnames`` names set from θ° (``pnames``: a ParamNamesBlock, or the tutorials'
    NamedTuple of PP / P_last / P_excl / Pb_excl with ``updt`` pairs ``(idx, name)``, for a
    BiBlock; ``pnames.blocks[i]`` for a BlockCollection; ``pnames.recordings[r].blocks[i]`` for a
    BlockEnsemble), the guiding term of b° recomputed, then ``recompute_path!(b°, b.WW; skip)``.

    ``critical_change`` (Bool / per block / per recording per block, as the reference
    broadcasts it): omitted — the reference's default GP.is_critical_update — recomputes the
    guiding term of the blocks whose auxiliary law changed (a recomputation of an unchanged law
    reproduces its guiding term bit for bit); True recomputes every block's; False keeps b°'s
    guiding term unless equalizing b°'s law with b's changed the auxiliary law
    (src/biblock.jl:340-342, 361-362).  Observation parameters
    (``updt_obs``, DD.set_parameters!(PP, θ°, updt, updt_aux, updt_obs), :373-375) are not
    device state here — a non-empty ``updt_obs`` raises.  One device call covers all blocks
    whose θ° → name maps and flags agree (every tutorial: a single call).  Returns per-block
    success."""
    if isinstance(x, BiBlock):
        groups = [(x, _theta_map(pnames, θ_prop))]
    elif isinstance(x, BlockCollection):
        groups = [(bb, _theta_map(pb, θ_prop)) for bb, pb in zip(x.blocks, _get(pnames, "blocks"))]
    elif isinstance(x, BlockEnsemble):
        groups = [(bb, _theta_map(pb, θ_prop))
                  for bc, pr in zip(x.recordings, _get(pnames, "recordings"))
                  for bb, pb in zip(bc.blocks, _get(pr, "blocks"))]
    else:
        raise TypeError("set_proposal_law: expected a BiBlock, BlockCollection or BlockEnsemble")
    ccs = [None] * len(groups) if critical_change is None else _flags(critical_change, len(groups))
    if all(m == groups[0][1] for _, m in groups) and all(c == ccs[0] for c in ccs):
        ok, _ = x.set_proposal_law(theta=groups[0][1], skip=skip, critical_change=ccs[0])
        return ok
    return np.concatenate([bb.set_proposal_law(theta=m, skip=skip, critical_change=c)[0]
                           for (bb, m), c in zip(groups, ccs)])


def _flags(cc, n):
    """critical_change as one Bool per block: a Bool, a per-block vector, or per recording
    a per-block vector (the reference's BlockCollection / BlockEnsemble broadcasts)."""
    if isinstance(cc, (bool, np.bool_)):
        return [bool(cc)] * n
    flat = []
    for v in cc:
        if isinstance(v, (bool, np.bool_, int, np.integer)):
            flat.append(bool(v))
        else:
            flat += [bool(u) for u in v]
    if len(flat) != n:
        raise ValueError(f"critical_change: {len(flat)} flags for {n} blocks")
    return flat


# ------------------------------------------------------------------ GuidedProposals' methods
def Val(x):
    """``Val(:P_only)`` / ``Val(:P°_only)`` flags of recompute_guiding_term!."""
    return str(x).lstrip(":")


class _GP:
    """``GP.*`` methods the reference extends (``GP.set_obs!``, ``GP.recompute_guiding_term!``,
    ``GP.loglikhd``, ``GP.equalize_obs_params!``)."""

    @staticmethod
    def set_obs(x):
        """``GP.set_obs!`` (src/biblock.jl:273-280, src/block_collection.jl:198,
        src/block_ensemble.jl:192)."""
        _blocks(x, "set_obs").set_obs()

    @staticmethod
    def recompute_guiding_term(x, flag=None):
        """``GP.recompute_guiding_term!`` of a SamplingUnit (src/sampling_unit.jl:100-102), a
        Block view (``recompute_guiding_term!(bb.b)``, src/block.jl:102-110), a BiBlock (b then
        b°, src/biblock.jl:288-291) or a collection / ensemble with an optional
        ``Val(:P_only)`` / ``Val(:P°_only)`` (src/block_collection.jl:208-221)."""
        if isinstance(x, SamplingUnit):
            x.recompute_guiding_term()
            return
        if isinstance(x, Block):
            e, lay, b0, b1 = _range_of(x)
            e.recompute_guiding_term(lay, b0, b1, unit=x.unit)
            return
        only = None if flag is None else {"P_only": "P_only", "P°_only": "P°_only",
                                          "Pprop_only": "P°_only"}[Val(flag)]
        _blocks(x, "recompute_guiding_term").recompute_guiding_term(only=only)

    @staticmethod
    def loglikhd(u):
        """``GP.loglikhd(u::SamplingUnit)`` (src/sampling_unit.jl:109): a value."""
        if not isinstance(u, SamplingUnit):
            raise TypeError("GP.loglikhd: expected a SamplingUnit (sp.u / sp.u_prop)")
        return u.loglikhd()

    @staticmethod
    def equalize_obs_params(bb):
        return _blocks(bb, "equalize_obs_params").equalize_obs_params()


GP = _GP()
