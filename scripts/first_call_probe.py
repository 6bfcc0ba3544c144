#!/usr/bin/env python3
"""The bench's timed region repeated: after bench.py's set-up and warmup, time several
consecutive single dmt_mcmc_run calls of --steps iterations exactly as bench.py times its one
call (barrier, set_timing, barrier, call, barrier), to see whether the first is slower than the
rest and by how much of it is kernel time (dispatch events) vs host."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L, workloads as W

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--reps", type=int, default=8)
ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep before each timed call")
a = ap.parse_args()
w = W.c2_ou2d()
w.meta["hist_len"] = a.warmup + a.steps * a.reps + 10
ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=0xD1FF,
                   grid_shared=w.grid_shared)
lay = W.fill(ens, w, init_Z=False)
B = w.nblocks
ens.loglikhd(lay, L.U, 0, B)
if a.warmup:
    ens.mcmc_run(lay, 0, B, 1, a.warmup)
ens.sync()
it = a.warmup + 1
out = []
for r in range(a.reps):
    if a.idle_ms:
        time.sleep(a.idle_ms * 1e-3)
    ens.set_timing(True, kernels=[L.K_DRAW])
    ens.sync()
    t0 = time.perf_counter()
    ens.mcmc_run(lay, 0, B, it, a.steps)
    ens.sync()
    el = time.perf_counter() - t0
    it += a.steps
    k_ms, _ = ens.get_timing(L.K_DRAW)
    ens.set_timing(False)
    out.append({"wall_us": el * 1e6, "kernel_us": k_ms * 1e3})
print(json.dumps({"steps": a.steps, "idle_ms": a.idle_ms, "calls": out}))
