#!/usr/bin/env python3
"""Host-side cost of one dmt_mcmc_run call at the driver's bench config (C2, 20 iterations):
wall time of the call (+ the bench's trailing sync) against the kernel's dispatch-event time,
with event timing on / off, and the cost of an idle dmt_sync.  Medians over --reps calls."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L, workloads as W

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--runs", default="1,20")
a = ap.parse_args()
w = W.c2_ou2d()
runs = [int(x) for x in a.runs.split(",")]
w.meta["hist_len"] = 4 * sum(runs) * a.reps + 100
ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                   grid_shared=w.grid_shared)
lay = W.fill(ens, w, init_Z=False)
B = w.nblocks
ens.loglikhd(lay, L.U, 0, B)
it = 1
ens.mcmc_run(lay, 0, B, it, 5); it += 5
out = {}
for n in runs:
    for timing in (True, False):
        walls, kern, calls = [], [], []
        for _ in range(a.reps):
            ens.sync()
            ens.set_timing(timing, kernels=[L.K_DRAW])
            ens.sync()
            t0 = time.perf_counter()
            ens.mcmc_run(lay, 0, B, it, n); it += n
            t1 = time.perf_counter()
            ens.sync()
            t2 = time.perf_counter()
            walls.append((t2 - t0) * 1e6)
            calls.append((t1 - t0) * 1e6)
            if timing:
                ms, _ = ens.get_timing(L.K_DRAW)
                kern.append(ms * 1e3)
        out[f"n{n}_timing{int(timing)}"] = {
            "wall_us": float(np.median(walls)), "call_us": float(np.median(calls)),
            "kernel_us": float(np.median(kern)) if kern else None}
ens.set_timing(False)
t = []
for _ in range(a.reps):
    t0 = time.perf_counter(); ens.sync(); t.append((time.perf_counter() - t0) * 1e6)
out["idle_sync_us"] = float(np.median(t))
print(json.dumps(out))
