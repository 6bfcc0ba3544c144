#!/usr/bin/env python3
"""Host-side time of the driver's C2 call (dmt_mcmc_run of 20 iterations + dmt_sync): wall time
per call against the kernel's own duration, with the line's HIP events off, on (stream events)
and on as dispatch events (DMT_DISPATCH_EVENTS=1 is read at dmt_create, so that mode runs as a
separate process: --dispatch)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import diffusionmcmctools_amd as dmt  # noqa: E402
from diffusionmcmctools_amd import _lib as L  # noqa: E402
from diffusionmcmctools_amd import workloads as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--calls", type=int, default=40)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
w = W.c2_ou2d()
w.meta["hist_len"] = 10 + a.iters * (3 * a.calls + 2)
ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                   grid_shared=w.grid_shared)
lay = W.fill(ens, w, init_Z=False)
B = w.nblocks
ens.loglikhd(lay, L.U, 0, B)
done = 0
ens.mcmc_run(lay, 0, B, 1, 5)
done = 5
out = {"dispatch_events": os.environ.get("DMT_DISPATCH_EVENTS", "0")}
for mode in ("off", "events", "off2"):
    walls, py = [], []
    ens.set_timing(mode == "events", kernels=[L.K_DRAW])
    for _ in range(a.calls):
        ens.sync()
        t0 = time.perf_counter()
        ens.mcmc_run(lay, 0, B, done + 1, a.iters)
        t1 = time.perf_counter()
        ens.sync()
        t2 = time.perf_counter()
        walls.append((t2 - t0) * 1e6)
        py.append((t1 - t0) * 1e6)
        done += a.iters
    row = {"wall_us_median": float(np.median(walls)), "wall_us_min": float(np.min(walls)),
           "mcmc_run_return_us_median": float(np.median(py))}
    if mode == "events":
        ms, n = ens.get_timing(L.K_DRAW)
        row["kernel_us_events"] = ms * 1e3 / a.calls
    ens.set_timing(False)
    out[mode] = row
print(json.dumps(out), flush=True)
