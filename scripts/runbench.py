#!/usr/bin/env python3
"""Device time of dmt_mcmc_run (persistent kernels) per iteration for several run lengths, and
the wall time of the call (kernel-variant comparisons: DMT_LIB_PATH=build_variants/…)."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L, workloads as W

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--runs", default="5,20,100,500")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
w = {"c2": W.c2_ou2d, "c1": W.c1_ou1d}[a.config]()
runs = [int(x) for x in a.runs.split(",")]
w.meta["hist_len"] = sum(runs) * a.reps + 10
ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                   grid_shared=w.grid_shared)
lay = W.fill(ens, w, init_Z=False)
B = w.nblocks
ens.loglikhd(lay, L.U, 0, B)
it = 1
ens.mcmc_run(lay, 0, B, it, 5); it += 5
out = {"lib": os.environ.get("DMT_LIB_PATH", "libdmt.so")}
for n in runs:
    best = None
    for _ in range(a.reps):
        ens.sync()
        ens.set_timing(True, kernels=[L.K_DRAW])
        t0 = time.perf_counter()
        ens.mcmc_run(lay, 0, B, it, n); it += n
        ens.sync()
        el = time.perf_counter() - t0
        ms, k = ens.get_timing(L.K_DRAW)
        r = (ms * 1e3 / n, el * 1e6 / n)
        best = r if best is None or r[0] < best[0] else best
    out[str(n)] = {"kernel_us_per_iter": best[0], "wall_us_per_iter": best[1]}
print(json.dumps(out))
