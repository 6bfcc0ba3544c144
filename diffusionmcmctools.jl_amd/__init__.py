"""diffusionmcmctools.jl_amd — MI355X-native guided-bridge imputation engine.

Drop-in for the hot path of DiffusionMCMCTools.jl (draw_proposal_path! /
accept_reject_proposal_path! / loglikhd! / recompute_path! / fetch_ll over
BiBlock, BlockCollection, BlockEnsemble).  Compute runs in libdmt.so (HIP, gfx950)
behind the C-ABI of include/dmt.h; this package is the host-side mirror of the
reference's interface (``api``), the low-level handle wrapper (``engine``) and the
set-up helpers (``models``, ``workloads``).  There is no CPU fallback.

Import it as ``import diffusionmcmctools_amd`` (root-level loader; the directory name
contains a dot).
"""
from . import _lib  # noqa: F401  (raises ImportError if libdmt.so is missing)
from ._lib import DMTError, version  # noqa: F401
from .engine import Ensemble, comm_unique_id, combine_rank_partials, guiding_linear, guiding_linear_td, guiding_linear_tda, read_snapshots  # noqa: F401
from .api import (BiBlock, Block, BlockCollection, BlockEnsemble,  # noqa: F401
                  SamplingEnsemble, SamplingPair, SamplingUnit)
from .functions import *  # noqa: F401,F403  (the reference's generic functions)
from .functions import __all__ as _fn_all
from .param_names import (AllObservations, ParamNamesAllObs, ParamNamesBlock,  # noqa: F401
                          ParamNamesRecording, ParamNamesUnit)

__all__ = ["Ensemble", "DMTError", "version", "comm_unique_id", "combine_rank_partials", "guiding_linear", "guiding_linear_td", "guiding_linear_tda", "read_snapshots",
           "SamplingEnsemble", "SamplingPair", "SamplingUnit", "BlockEnsemble",
           "BlockCollection", "BiBlock", "Block", "AllObservations", "ParamNamesUnit",
           "ParamNamesBlock", "ParamNamesRecording", "ParamNamesAllObs"] + list(_fn_all)
