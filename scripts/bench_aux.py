#!/usr/bin/env python3
"""Timing of the §8(f) kernels at C3 scale (65 536 FHN blocks × 1 000 steps, fp64, one GPU):
find_W_for_X! (k_invsolve), loglikhd! (k_pathll) and recompute_guiding_term! (the device
backward filter) — HIP dispatch events, one JSON line per kernel with its algorithmic bytes
and the HBM roofline fraction (the filter is fp64-compute-bound: flops are not counted)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--N", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import _lib as L
    from diffusionmcmctools_amd import workloads as W
    from diffusionmcmctools_amd.models import packed
    w = W.c3_fhn(B=a.B, N=a.N)
    ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=3,
                       grid_shared=w.grid_shared)
    lay = W.fill(ens, w, init_Z=False)
    nb = w.nblocks
    steps = w.steps_per_iter
    s = 8
    out = []

    def timed(kind, fn):
        ens.sync()
        ens.set_timing(True, kernels=[kind])
        for _ in range(a.reps):
            fn()
        ens.sync()
        ms, n = ens.get_timing(kind)
        ens.set_timing(False)
        return ms / max(n, 1) * 1e-3

    # find_W_for_X!: read X (d) + H (hp) + F (d), write W (m) per step
    t = timed(L.K_RECOMPUTE, lambda: ens.find_W_for_X(lay, 0, nb))
    byt = s * (w.d + w.d * (w.d + 1) // 2 + w.d + w.m) * steps
    out.append(dict(kernel="k_invsolve (find_W_for_X!)", us=t * 1e6, bytes=byt,
                    GBs=byt / t / 1e9, frac=byt / t / 1e9 / PEAK, steps_per_s=steps / t))
    # loglikhd!: read X (d) + H (hp) + F (d) per step
    t = timed(L.K_PATHLL, lambda: ens.loglikhd(lay, L.U, 0, nb))
    byt = s * (w.d + w.d * (w.d + 1) // 2 + w.d) * steps
    out.append(dict(kernel="k_pathll (loglikhd!)", us=t * 1e6, bytes=byt, GBs=byt / t / 1e9,
                    frac=byt / t / 1e9 / PEAK, steps_per_s=steps / t))
    # recompute_guiding_term!: write H (hp) + F (d) per point; fp64 compute-bound
    G = nb
    hp = w.d * (w.d + 1) // 2
    v = w.meta["v"]
    Hobs = np.tile(packed(np.array([[100.0, 0.0], [0.0, 0.0]])), (G, 1))
    Fobs = np.stack([np.array([100.0 * v[b], 0.0]) for b in range(G)])
    cobs = np.zeros(G)
    ens.upload_obs(Hobs, Fobs, cobs)
    t = timed(L.K_RECOMPUTE, lambda: ens.recompute_guiding_term(lay, 0, nb, L.U))
    byt = s * (hp + w.d) * (steps + nb)
    out.append(dict(kernel="k_filter_scan + k_filter_chain (recompute_guiding_term!)", us=t * 1e6, bytes=byt,
                    GBs=byt / t / 1e9, frac=byt / t / 1e9 / PEAK, points_per_s=(steps + nb) / t,
                    bound="fp64 VALU (exact transition per step, one combine per point)"))
    for o in out:
        o.update(config=f"C3 FHN {nb} blocks x {a.N} steps fp64")
        print(json.dumps(o))


if __name__ == "__main__":
    main()
