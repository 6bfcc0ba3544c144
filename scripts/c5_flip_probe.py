#!/usr/bin/env python3
"""Locate MH decisions of the bench's CPU leg that differ from the device (C5 fp32): runs the
bench workload, then one iteration on the CPU leg's path (oracle, sequential loop, the device's
streams) and on the device, and prints every block whose decision, ll° or proposal differs."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import bench
import oracle as orc
import diffusionmcmctools_amd as dmt
from diffusionmcmctools_amd import _lib as L

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 30
w = bench.build_workload(cfg, 0)
w.meta["hist_len"] = warm + 4
ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=bench.ens_seed,
                   device=0, grid_shared=w.grid_shared)
lay = dmt.workloads.fill(ens, w, init_Z=False)
B = w.nblocks
npts = w.n_points[0][0]
ens.loglikhd(lay, L.U, 0, B)
ens.mcmc_run(lay, 0, B, 1, warm)
it = warm + 1
X = ens.download_paths(L.U, 0)
Wp = ens.download_paths(L.U, 2)  # increments as held (DMT_PATH_DW)
ll = ens.get_block_state(lay, L.BLK_LL, 0, B)
rho = np.full(B, w.rho)
out = {}
for seq in (True, False):
    Xo, Wo, llp, nfail = orc.draw_terminal_blocks(
        w.model.kind, w.d, w.m, npts, w.laws, w.t, w.H, w.F, X, Wp, rho, Z=None,
        seed=bench.ens_seed, it=it, salt=0, prec=w.precision, nthreads=16, t_shared=True,
        H_shared=w.H_shared, sequential=seq)
    out[seq] = (Xo, llp, nfail)
E = orc.exp1_range(bench.ens_seed, 0, B, it, 0)
ens.mcmc_run(lay, 0, B, it, 1)
dev_acc = ens.get_block_state(lay, L.BLK_ACC_HIST, 0, B, hist_len=w.meta["hist_len"])[it - 1].astype(bool)
dev_llp = ens.get_block_state(lay, L.BLK_LLPROP_HIST, 0, B, hist_len=w.meta["hist_len"])[it - 1]
dev_ll = ens.get_block_state(lay, L.BLK_LL_HIST, 0, B, hist_len=w.meta["hist_len"])[it - 1]
Xo, llp, nfail = out[True]
cpu_acc = E > -(llp - ll)
diff = np.flatnonzero(cpu_acc != dev_acc)
llp_diff = np.flatnonzero(~((llp == dev_llp) | (np.isnan(llp) & np.isnan(dev_llp))))
print(json.dumps({"config": cfg, "iteration": it, "blocks": B,
                  "decision_diffs": diff.tolist()[:20], "llp_diffs": int(llp_diff.size),
                  "llp_diff_blocks": llp_diff.tolist()[:20],
                  "seq_vs_canonical_llp_equal": bool(np.array_equal(out[True][1], out[False][1], equal_nan=True)),
                  "ll_state_equal": bool(np.array_equal(ll, dev_ll, equal_nan=True))}))
for b in llp_diff[:10]:
    print(int(b), "cpu llp", repr(float(llp[b])), "dev llp", repr(float(dev_llp[b])), "ll", repr(float(ll[b])),
          "E", repr(float(E[b])), "cpu acc", bool(cpu_acc[b]), "dev acc", bool(dev_acc[b]), "nfail", nfail)
ens.close()
