#!/usr/bin/env python3
"""Kernel-level timing of draw_proposal for a workload/mapping/mode (device events)."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L, workloads as W

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--mapping", default="wave")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--parity", action="store_true", help="host normals (no device RNG)")
ap.add_argument("--B", type=int, default=0)
ap.add_argument("--accept", action="store_true", help="accept_reject after every draw")
ap.add_argument("--step", action="store_true", help="use dmt_mcmc_step")
ap.add_argument("--accept-all", action="store_true", help="accept_reject with E = +inf (all accept)")
ap.add_argument("--sync", action="store_true", help="synchronise after every call")
ap.add_argument("--mix", type=float, default=0.0,
                help="before timing, accept a random fraction of the blocks (mixed selectors)")
a = ap.parse_args()
kw = {"B": a.B} if a.B else {}
w = {"c2": W.c2_ou2d, "c3": W.c3_fhn, "c5": W.c5_lorenz, "c1": W.c1_ou1d}[a.config](**kw)
mp = {"auto": 0, "lane": 1, "wave": 2}[a.mapping]
ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                   grid_shared=w.grid_shared, mapping=mp)
w.meta["hist_len"] = a.iters + 2
lay = W.fill(ens, w, init_Z=False)
B = w.nblocks
Z = np.random.default_rng(0).standard_normal((w.steps_per_iter, w.m)) if a.parity else None
ens.draw_proposal(lay, 0, B, Z=Z, iter=1)
if a.mix > 0:
    acc = np.random.default_rng(1).random(B) < a.mix
    ens.accept_reject(lay, 0, B, 1, E=np.where(acc, np.inf, -np.inf))
ens.sync()
ens.set_timing(True)
t0 = time.perf_counter()
for i in range(a.iters):
    if a.step:
        ens.mcmc_step(lay, 0, B, i + 2)
        continue
    ens.draw_proposal(lay, 0, B, Z=Z, iter=i + 2)
    if a.accept:
        ens.accept_reject(lay, 0, B, i + 2)
    if a.accept_all:
        ens.accept_reject(lay, 0, B, i + 2, E=np.full(B, np.inf))
    if a.sync:
        ens.sync()
ens.sync()
el = time.perf_counter() - t0
ms, n = ens.get_timing(L.K_DRAW)
print(json.dumps({"config": a.config, "mapping": a.mapping, "parity": a.parity,
                  "accept": a.accept, "step": a.step, "sync": a.sync, "accept_all": a.accept_all,
                  "diag": os.environ.get("DMT_DIAG", "0"), "B": B,
                  "kernel_us": ms / n * 1e3, "wall_us_per_call": el / a.iters * 1e6,
                  "gsteps_per_s": w.steps_per_iter / (ms / n * 1e-3) / 1e9}))
