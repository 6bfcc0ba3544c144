"""C5 (Lorenz fp32, 2000 steps) draw time against the number of recordings: 0.25, 0.5 and 1
wave per SIMD of the lane kernel (16 384, 32 768, 65 536 recordings = 256, 512, 1 024 tiles).
Flat time up to 1 024 waves = the chip's idle SIMDs, not the per-wave stream, set C5's rate."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L
from diffusionmcmctools_amd import workloads as W

out = []
for B in [int(b) for b in (sys.argv[1:] or ["16384", "32768", "65536"])]:
    w = W.c5_lorenz(B=B)
    w.meta["hist_len"] = 64
    ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=3,
                       grid_shared=w.grid_shared)
    lay = W.fill(ens, w, init_Z=False)
    ens.loglikhd(lay, L.U, 0, B)
    ens.mcmc_run(lay, 0, B, 1, 3)
    ens.sync()
    ens.set_timing(True, kernels=[L.K_DRAW])
    ens.mcmc_run(lay, 0, B, 4, 10)
    ens.sync()
    ms, n = ens.get_timing(L.K_DRAW)
    ens.set_timing(False)
    rec = {"recordings": B, "waves": B // 64, "draw_us": ms / n * 1e3, "draws": n,
           "GBps": 72.0 * B * 2000 / (ms / n * 1e-3) / 1e9}
    print(json.dumps(rec), flush=True)
    out.append(rec)
    del ens
