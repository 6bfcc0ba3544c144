#!/usr/bin/env python3
"""Benchmark of the guided-bridge imputation hot path on MI355X.

One "step" = one MCMC iteration over the whole per-GPU BlockEnsemble:
  draw_proposal_path!(be)            (pCN + guided Euler–Maruyama + Girsanov weight, device RNG)
  accept_reject_proposal_path!(be,i) (per-block MH test, selector swaps, histories)
  fetch_ll(be) + accepted count      (deterministic reduction; RCCL all-gather over ranks)
i.e. the caller loop of /root/reference/docs/src/tutorials/biblock/smoothing.md:40-44 at
BlockEnsemble level (src/block_ensemble.jl:50,63-67,140).  Throughput unit: bridge-segment
Euler steps (one grid increment of one segment) per second, whole job.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5]
Multi-GPU: launched by torch.distributed.run, one rank per GPU, weak scaling: rank r owns
recording shard r of a global ensemble of N x B blocks (RNG keyed by global segment ids,
diffusionmcmctools.jl_amd/shard.py); the only collective is fetch_ll's RCCL all-gather of
3 doubles per iteration.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0
EXTRA_ITERS = 5  # untimed iterations after the timed region (accept-kernel event timing)  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    "c2": ("C2: 2D OU guided bridge, 1024 blocks x 500 Euler steps per GPU, fp64", "f64"),
    "c3": ("C3/C4: FitzHugh-Nagumo guided bridge, 65536 blocks x 1000 Euler steps per GPU, fp64", "f64"),
    "c5": ("C5: Lorenz-63 guided bridge, 32768 blocks x 2000 Euler steps per GPU, fp32", "f32"),
}


def build_workload(name, rank):
    from diffusionmcmctools_amd import workloads as W
    if name == "c2":
        return W.c2_ou2d(block_offset=rank)
    if name == "c3":
        return W.c3_fhn(block_offset=rank)
    if name == "c5":
        return W.c5_lorenz(block_offset=rank)
    raise SystemExit(f"unknown config {name}")


def algorithmic_bytes_per_step(w):
    """s·(2m [read W, write W°] + d [write X°] + d [read F] + h [read H]),
    h = d(d+1)/2 for per-block guiding tables, 0 when H is shared; shared grid ignored."""
    s = 8 if w.precision == 0 else 4
    h = 0 if w.H_shared else w.d * (w.d + 1) // 2
    return s * (2 * w.m + 2 * w.d + h)


def measured_traffic(config, kernel_substr):
    """HBM bytes per launch of the draw kernel from the newest committed PMC summary
    (profiles/rNN_traffic_<config>.json, scripts/pmc_traffic.py: separate FETCH_SIZE and
    WRITE_SIZE rocprofv3 passes, calibrated with scripts/calib_stream); None if absent."""
    import glob
    # run tags go r01, r01b … r01z, r01aa …: newest = longest tag, then the last in order
    def tag(p):
        t = os.path.basename(p).split("_traffic_")[0]
        return (len(t), t)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{config}.json")), key=tag)
    for path in reversed(files):
        with open(path) as f:
            t = json.load(f)
        if kernel_substr in t.get("kernel", ""):
            return t["traffic_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(w, ens, lay, budget_s=12.0):
    """The oracle's OpenMP restatement (oracle/dmt_oracle.c) timed on this host on a bounded
    sample: whole MCMC iterations (draw + MH accept) of the same per-GPU workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    from diffusionmcmctools_amd import _lib as L
    nthreads = max(1, min(16, os.cpu_count() or 1))
    B = w.nblocks
    npts = w.n_points[0][0]
    X = ens.download_paths(L.U, 0)
    Wc = ens.download_paths(L.U, 1).reshape(B, npts, w.m)  # cumulative Wiener paths
    Wp = Wc.copy()                                          # the oracle holds increments
    Wp[:, 1:] = Wc[:, 1:] - Wc[:, :-1]
    Wp = Wp.reshape(B * npts, w.m)
    ens.loglikhd(lay, L.U, 0, B)
    ll = ens.get_block_state(lay, L.BLK_LL, 0, B)
    rho = np.full(B, w.rho)
    prec = w.precision
    rng = np.random.default_rng(0)
    res = {}
    for nt in sorted({1, nthreads}):
        it = 0
        acc_n = 0
        Xa, Wa, lla = X.copy(), Wp.copy(), ll.copy()
        t0 = time.perf_counter()
        while True:
            it += 1
            Xo, Wo, llp, _ = orc.draw_terminal_blocks(
                w.model.kind, w.d, w.m, npts, w.laws, w.t, w.H, w.F, Xa, Wa, rho, Z=None,
                seed=1234, it=it, salt=0, prec=prec, nthreads=nt, t_shared=True,
                H_shared=w.H_shared, sequential=True)
            E = rng.exponential(1.0, B)
            acc = E > -(llp - lla)
            sel = np.repeat(acc, npts)
            Xa = np.where(sel[:, None], Xo, Xa)
            Wa = np.where(sel[:, None], Wo, Wa)
            lla = np.where(acc, llp, lla)
            acc_n += int(acc.sum())
            el = time.perf_counter() - t0
            if (el > budget_s / 2 and it >= 2) or it >= 10000:
                break
        res[nt] = (w.steps_per_iter * it / el, it, acc_n / (B * it))
    v, its, ar = res[nthreads]
    v1 = res[1][0]
    return {"value": v, "unit": "steps/s", "cores": nthreads, "kind": "port",
            "sample": f"{its} full MCMC iterations (draw + MH accept) of the same per-GPU workload "
                      f"({B} blocks x {npts - 1} steps), step-by-step Euler loop, same "
                      f"Philox/Box-Muller normals, OpenMP over blocks",
            "value_1thread": v1, "accept_rate": ar}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--mapping", default="auto", choices=["auto", "lane", "wave"],
                    help="thread mapping of the Euler recursion (DESIGN.md §2)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only; the data path is RCCL in libdmt

    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import _lib as L
    from diffusionmcmctools_amd import workloads as W

    w = build_workload(args.config, rank)
    w.meta["hist_len"] = args.warmup + args.steps + EXTRA_ITERS
    mapping = {"auto": L.MAP_AUTO, "lane": L.MAP_LANE, "wave": L.MAP_WAVE}[args.mapping]
    ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision,
                       seed=0xD1FF, device=local_rank, grid_shared=w.grid_shared,
                       mapping=mapping)
    # rank r holds recording shard r of the global ensemble: RNG streams keyed by global
    # segment ids (shard.py), so the N-GPU job equals one ensemble of N x B blocks
    ens.set_shard(rank * ens.G)
    lay = W.fill(ens, w, init_Z=False)
    B = w.nblocks
    if world > 1:
        uid = [dmt.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ens.comm_init(world, rank, uid[0])
    ens.loglikhd(lay, L.U, 0, B)

    # one step = draw_proposal_path!(be); accept_reject_proposal_path!(be, i); fetch_ll(be).
    # The K timed steps are queued back to back on the device (dmt_mcmc_run: no host round
    # trip per iteration; every iteration's fetch_ll values come back at the end).

    def barrier():
        ens.sync()
        if dist is not None:
            dist.barrier()

    if args.warmup:
        ens.mcmc_run(lay, 0, B, 1, args.warmup)
    barrier()
    # HIP events around the dominant (draw) kernel over the timed region, on libdmt's stream
    ens.set_timing(True, kernels=[L.K_DRAW])
    barrier()
    t0 = time.perf_counter()
    res = ens.mcmc_run(lay, 0, B, args.warmup + 1, args.steps)
    barrier()
    el = time.perf_counter() - t0
    n_acc = float(res[:, 2].sum())
    k_ms, k_n = ens.get_timing(L.K_DRAW)  # k_n counts iterations (persistent) or launches
    persist = w.model.kind == L.MODEL_OU and os.environ.get("DMT_MCMC_PERSIST", "1") != "0"
    a_ms = a_n = 0
    if not persist:
        # the accept+reduce kernel, timed on a few extra iterations after the timed region
        ens.set_timing(True, kernels=[L.K_ACCEPT])
        ens.mcmc_run(lay, 0, B, args.warmup + args.steps + 1, EXTRA_ITERS)
        a_ms, a_n = ens.get_timing(L.K_ACCEPT)
    ens.set_timing(False)
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    steps_total = w.steps_per_iter * args.steps * world
    value = steps_total / el
    # launches of the dominant kernel in the timed region: one per iteration, or (persistent,
    # dmt_mcmc_run) one per chunk of iterations (dmt_runtime.hip: ≤ 64 MiB of partials)
    it_per_launch = min(args.steps, max(1, (64 << 20) // (24 * B))) if persist else 1
    launches = -(-args.steps // it_per_launch)
    k_avg_s = (k_ms / launches) * 1e-3          # average launch duration
    k_iter_s = (k_ms / max(args.steps, 1)) * 1e-3
    bytes_iter = algorithmic_bytes_per_step(w) * w.steps_per_iter
    bytes_launch = bytes_iter * it_per_launch
    achieved = bytes_launch / k_avg_s / 1e9 if k_avg_s > 0 else 0.0
    accept_rate = n_acc / (B * world * args.steps)  # n_acc is already global (fetch_ll over ranks)
    # the mapping libdmt resolves for MAP_AUTO (kAutoWaveMaxRecordings, dmt_internal.h)
    wave = args.mapping == "wave" or (args.mapping == "auto" and len(w.n_points) <= 8192)
    # single-segment blocks of <= 512 steps, d <= 2: register-resident kernels (dmt_internal.h)
    short1 = (w.model.kind == L.MODEL_OU and w.d <= 2
              and all(len(r) == 1 and r[0] - 1 <= 512 for r in w.n_points))
    resident = persist and short1 and os.environ.get("DMT_MCMC_RESIDENT", "1") != "0"
    if resident:  # linear drift: all K iterations in one k_mcmc_resident launch (dmt_mcmc_run)
        wave, kname = True, "k_mcmc_resident"
    elif persist:  # linear drift: all K iterations in one k_mcmc_scan launch (dmt_mcmc_run)
        wave, kname = True, "k_mcmc_scan"
    elif short1 and os.environ.get("DMT_SCAN_RESIDENT", "1") != "0":  # one launch per iteration
        wave, kname = True, "k_block_resident"
    elif w.model.kind == L.MODEL_OU:  # linear drift: the affine-scan kernel per iteration
        wave, kname = True, "k_block_scan"
    else:
        kname = "k_block_wave" if wave else "k_block<"
    traffic, traffic_src = measured_traffic(args.config, kname)  # HBM bytes per iteration
    if traffic is not None:
        traffic *= it_per_launch
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(w, ens, lay, budget_s=args.cpu_budget)
        desc, dtype = WORKLOADS[args.config]
        line = {
            "metric": "bridge-segment Euler steps/sec/GPU; accept-rate vs CPU ref",
            "value": value,
            "unit": "steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (seeded, SURVEY.md §8(d) configs; no reference checkpoints/datasets)",
            "config": {"workload": desc, "blocks_per_gpu": B,
                       "euler_steps_per_block": w.steps_per_iter // B, "rho": w.rho,
                       "parallelism": f"blockensemble-shard x{world}",
                       "mapping": ("scan-resident" if resident else
                                   "scan-persistent" if persist else
                                   "scan-resident-per-iteration" if kname == "k_block_resident" else
                                   "scan" if kname == "k_block_scan" else
                                   "wave" if wave else "lane"),
                       "rng": "device Philox4x32-10 + Box-Muller (perf mode)"},
            "per_gpu": value / world,
            "accept_rate": accept_rate,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": kname + (" (draw_proposal_path! + accept_reject_proposal_path! "
                                            "of every iteration of the launch)" if persist else
                                            " (draw_proposal_path!)"),
                         "kernel_avg_us": k_avg_s * 1e6,
                         "kernel_us_per_iteration": k_iter_s * 1e6,
                         "iterations_per_launch": it_per_launch,
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "algorithmic_bytes_per_iteration": bytes_iter,
                         "bytes_per_step": algorithmic_bytes_per_step(w)},
            "accept_kernel_avg_us": (a_ms / a_n) * 1e3 if a_n else None,
            "cpu_baseline": cpu,
        }
        if cpu is not None:
            line["accept_rate_cpu"] = cpu["accept_rate"]
        print(json.dumps(line))
    ens.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
