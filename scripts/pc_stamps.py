#!/usr/bin/env python3
"""Where the fixed time of one C2 k_mcmc_resident_pc launch goes: device wall-clock stamps
(100 MHz) per workgroup from a -DDMT_PC_STAMPS build (DMT_LIB_PATH=build_variants/
libdmt_stamps.so): entry (0), consumer set-up done (1), producer first draw + propose done (2),
B1 of iteration 0 passed (3), loop end (4), tree tail end (5), consumer: law record and
loglikhd_obs done (6), per-step constants loaded (7) (before its own normals).  Prints the spread over the
workgroups of each stage relative to the launch's first entry, for a few launches of
--iters iterations, beside the HIP-event kernel time."""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import diffusionmcmctools_amd as dmt  # noqa: E402
from diffusionmcmctools_amd import _lib as L  # noqa: E402
from diffusionmcmctools_amd import workloads as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--launches", type=int, default=5)
a = ap.parse_args()

w = W.c2_ou2d()
w.meta["hist_len"] = 10 + a.iters * (a.launches + 1)
ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=5,
                   grid_shared=w.grid_shared)
lay = W.fill(ens, w, init_Z=False)
B = w.nblocks
ens.loglikhd(lay, L.U, 0, B)
ens.mcmc_run(lay, 0, B, 1, 5)
fn = L.lib.dmt_probe_pc_stamps
fn.argtypes = [C.c_void_p, C.c_int64]
nwg = (B + 3) // 4
done = 5
out = []
for k in range(a.launches):
    ens.sync()
    ens.set_timing(True, kernels=[L.K_DRAW])
    ens.mcmc_run(lay, 0, B, done + 1, a.iters)
    ens.sync()
    ms, n = ens.get_timing(L.K_DRAW)
    ens.set_timing(False)
    done += a.iters
    st = np.zeros(8192 * 8, dtype=np.uint64)
    assert fn(st.ctypes.data, st.size) == 0
    s = st[:nwg * 8].reshape(nwg, 8).astype(np.int64)
    t0 = s[:, 0].min()
    rel = (s[:, :8] - t0) * 0.01  # µs
    row = {"launch": k, "event_kernel_us": round(ms * 1e3, 2),  # one launch (n counts iterations)
           "span_us": float((s[:, 5].max() - t0) * 0.01)}
    for j, name in enumerate(["entry", "cons_setup", "prod_first_draw", "b1_iter0", "loop_end",
                              "tail_end", "cons_law_obs", "cons_step_consts"]):
        v = rel[:, j]
        row[name] = {"min": round(float(v.min()), 2), "med": round(float(np.median(v)), 2),
                     "max": round(float(v.max()), 2)}
    row["loop_us_med"] = round(float(np.median(rel[:, 4] - rel[:, 3])), 2)
    row["per_iter_us_med"] = round(row["loop_us_med"] / a.iters, 3)
    out.append(row)
    print(json.dumps(row), flush=True)

# per-iteration stamps of workgroup 0 (the last launch): durations in µs per iteration
fi = L.lib.dmt_probe_pc_iter_stamps
fi.argtypes = [C.c_void_p]
it = np.zeros(64 * 8, dtype=np.uint64)
assert fi(it.ctypes.data) == 0
t = it.reshape(64, 8).astype(np.int64)[:a.iters]
d = lambda i, j: np.median((t[:, j] - t[:, i]) * 0.01)  # noqa: E731
cyc = np.median(np.diff(t[:, 0]) * 0.01)
print(json.dumps({"wg0_iteration_us": round(float(cyc), 3),
                  "cons_B1_to_decision": round(float(d(0, 1)), 3),
                  "cons_decision_to_B2_arrive": round(float(d(1, 2)), 3),
                  "cons_B2_wait": round(float(d(2, 3)), 3),
                  "prod_B1_to_B2_arrive (W stores + draw)": round(float(d(4, 5)), 3),
                  "prod_B2_wait": round(float(d(5, 6)), 3),
                  "prod_B2_to_B1_arrive (propose)": round(float(d(6, 7)), 3),
                  "cons_B2_to_next_B1_pass": round(float(np.median((t[1:, 0] - t[:-1, 3]) * 0.01)), 3)}))
