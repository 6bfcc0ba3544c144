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
Multi-GPU: one process per GPU, weak scaling: rank r owns recording shard r of a global
ensemble of N x B blocks (RNG keyed by global segment ids, diffusionmcmctools.jl_amd/shard.py);
the only collective is fetch_ll's RCCL all-gather of 3 doubles per iteration.  Under
torch.distributed.run the ranks come from RANK/LOCAL_RANK/WORLD_SIZE; run directly with
--gpus N > 1 (WORLD_SIZE unset), this process spawns the N ranks itself before touching a GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
EXTRA_ITERS = 5        # untimed iterations after the timed region (accept-kernel event timing)
CPU_MAX_ITERS = 4000   # bound of the CPU-baseline sample (history slots reserved for it)

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


def _newest(pattern):
    """Committed profile files matching a glob, newest run tag first (tags r01, r01b … r01z,
    r01aa …, r02a …: ordered by round, then tag length, then name)."""
    import glob

    def tag(p):
        t = os.path.basename(p).split("_")[0]
        return (t[:3], len(t), t)
    return sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=tag, reverse=True)


_TREE = None


def tree_digest():
    """Digest of the library sources this bench runs from (scripts/provenance.py)."""
    global _TREE
    if _TREE is None:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import provenance
        _TREE = provenance.csrc_digest(ROOT)
    return _TREE


# the draw kernels a timed call can dispatch, as committed summaries name them (lane kernels with
# their template bracket so that k_block< does not match k_block_pk<)
DRAW_KERNELS = ("k_mcmc_resident_pc", "k_mcmc_resident", "k_mcmc_scan", "k_block_resident",
                "k_block_scan", "k_block_wave", "k_block_ps_pk<", "k_block_pk<", "k_block<")


def dispatched_kernel(recent):
    """The family of the most recent draw kernel among libdmt's recently launched kernels
    (demangled names, most recent first), or None."""
    for name in recent:
        m = re.search(r"\bdmt::(k_\w+)<", name)
        if not m:
            continue
        base = m.group(1)
        for fam in DRAW_KERNELS:
            if fam.rstrip("<") == base:
                return fam
    return None


def committed_summary(kind, config, kernel_substr):
    """The newest committed profile summary of `kind` (traffic: scripts/pmc_traffic.py, kstats:
    scripts/kstats_summary.py, issue: scripts/issue_summary.py) for this config and kernel,
    used only if it measured THIS source tree (its csrc_sha16 equals tree_digest()).  Returns
    (summary with "source" set, None), or (None, the newest matching file's name) when that
    file measured another tree, or (None, None) when there is none."""
    for path in _newest(f"r*_{kind}_{config}.json"):
        with open(path) as f:
            t = json.load(f)
        k = t.get("kernel", "")
        if not k or kernel_substr not in k and k not in kernel_substr:
            continue
        rel = os.path.relpath(path, ROOT)
        if t.get("csrc_sha16") != tree_digest():
            return None, rel
        t = dict(t)
        t["source"] = rel
        return t, None
    return None, None


def host_cpu_info():
    """nproc, the CPUs this process may run on, OMP_NUM_THREADS and the lscpu model name."""
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"nproc": os.cpu_count(), "affinity": affinity,
            "omp_num_threads": int(omp) if omp and omp.isdigit() else None, "model": model}


def cpu_baseline(w, ens, lay, iter0, budget_s=12.0):
    """The oracle's OpenMP restatement (oracle/dmt_oracle.c) timed on this host on a bounded
    sample of whole MCMC iterations (draw + MH accept) of the same per-GPU workload, from the
    device's current state and with the device's streams: iteration it draws the normals of
    key (it, salt 0) and the Exp(1) variables of the same key — exactly what the device's next
    dmt_mcmc_run(iter0, …) draws.  The CPU leg runs the reference's sequential Euler loop
    (oracle sequential=True), the device the canonical parallel affine scan (OU) or the same
    recursion (FHN, Lorenz); the device then runs the same iterations and the per-block MH
    decisions are compared.  Threads: every CPU this process may use, capped by
    OMP_NUM_THREADS (the GPU box's CPU share) when that is set."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    from diffusionmcmctools_amd import _lib as L
    info = host_cpu_info()
    nthreads = info["affinity"] or 1
    if info["omp_num_threads"]:
        nthreads = min(nthreads, info["omp_num_threads"])
    B = w.nblocks
    npts = w.n_points[0][0]
    X = ens.download_paths(L.U, 0)
    Wp = ens.download_paths(L.U, 2)  # the Wiener increments exactly as the device holds them
    ll = ens.get_block_state(lay, L.BLK_LL, 0, B)
    rho = np.full(B, w.rho)
    prec = w.precision

    def run(nt, max_it, budget, record, max_it_min=2):
        Xa, Wa, lla = X.copy(), Wp.copy(), ll.copy()
        decisions = []
        it, acc_n = 0, 0
        t0 = time.perf_counter()
        while it < max_it:
            key = iter0 + it
            Xo, Wo, llp, _ = orc.draw_terminal_blocks(
                w.model.kind, w.d, w.m, npts, w.laws, w.t, w.H, w.F, Xa, Wa, rho, Z=None,
                seed=ens_seed, it=key, salt=0, prec=prec, nthreads=nt, t_shared=True,
                H_shared=w.H_shared, sequential=True)
            E = orc.exp1_range(ens_seed, 0, B, key, 0)
            acc = E > -(llp - lla)
            sel = np.repeat(acc, npts)
            Xa = np.where(sel[:, None], Xo, Xa)
            Wa = np.where(sel[:, None], Wo, Wa)
            lla = np.where(acc, llp, lla)
            acc_n += int(acc.sum())
            it += 1
            if record:
                decisions.append(acc)
            if time.perf_counter() - t0 > budget and it >= max_it_min:
                break
        el = time.perf_counter() - t0
        return w.steps_per_iter * it / el, it, acc_n / (B * it), decisions

    v1, its1, _, _ = run(1, 5, 0.0, False, 5)  # single-thread rate: 5 whole iterations
    v, its, ar, dec = run(nthreads, CPU_MAX_ITERS, budget_s, True)
    # the device runs the same iterations from the same state (untimed) and records decisions
    ens.mcmc_run(lay, 0, B, iter0, its)
    hist = ens.get_block_state(lay, L.BLK_ACC_HIST, 0, B, hist_len=w.meta["hist_len"])
    dev = hist[iter0 - 1: iter0 - 1 + its].astype(bool)
    cpu = np.array(dec)
    same = dev == cpu
    first = int(np.argmin(same.all(axis=1))) if not same.all() else None
    return {"value": v, "unit": "steps/s", "cores": nthreads, "kind": "port",
            "sample": f"{its} full MCMC iterations (draw + MH accept) of the same per-GPU "
                      f"workload ({B} blocks x {npts - 1} steps) from the device's state after "
                      f"iteration {iter0 - 1}, the device's Philox normal and Exp(1) streams "
                      f"(keys {iter0}..{iter0 + its - 1}), sequential Euler loop, OpenMP over "
                      f"blocks",
            "value_1thread": v1, "iterations_1thread": its1, "accept_rate": ar,
            "decisions_identical": int(same.sum()), "decisions_total": int(same.size),
            "first_differing_iteration": None if first is None else iter0 + first,
            "accept_rate_device_same_iterations": float(dev.mean()),
            "host": info}


ens_seed = 0xD1FF


def separate_calls(ens, lay, B, iter0, n, global_, python=True):
    """The reference's unchanged caller loop, every call separate — draw_proposal_path!(be);
    accept_reject_proposal_path!(be, i); fetch_ll(be); fetch_ll°(be) — issued as C-ABI calls
    from C (csrc/dmt_callbench.c: what a Julia caller's ccalls cost) and, for comparison, from
    Python through ctypes (the Python mirror).  Returns µs per iteration of both loops and the
    C loop's per-iteration (fetch_ll, fetch_ll°, accepted count)."""
    import ctypes as C
    from diffusionmcmctools_amd import _lib as L
    lib = C.CDLL(os.path.join(ROOT, "diffusionmcmctools.jl_amd", "libdmt_callbench.so"))
    out = np.empty((n, 3))
    sec = C.c_double()
    st = lib.dmt_callbench_loop(ens.handle, C.c_int32(lay), C.c_int64(0), C.c_int64(B),
                                C.c_int64(iter0), C.c_int64(n), C.c_int32(1 if global_ else 0),
                                out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(sec))
    if st != 0:
        raise RuntimeError(f"dmt_callbench_loop failed at step {st}: {L.lib.dmt_last_error()}")
    c_us = sec.value / n * 1e6
    if not python:
        return c_us, None, out
    t0 = time.perf_counter()
    for i in range(iter0 + n, iter0 + 2 * n):
        ens.draw_proposal(lay, 0, B, salt=L.RNG_AUTO, want_success="lazy")
        ens.accept_reject(lay, 0, B, i, salt=L.RNG_AUTO)
        ens.fetch_ll(lay, 0, B, i, local=not global_)
        ens.fetch_ll(lay, 0, B, 0, local=not global_)
    py_us = (time.perf_counter() - t0) / n * 1e6
    return c_us, py_us, out


def rank_diagnostics(dist, world, k_ms, allgather_us, rccl_nranks):
    """Per-rank timing spread of an N-GPU run (rank 0 prints it): the slowest and fastest rank's
    draw-kernel time over the timed region, the RCCL all-gather's cost per fetch_ll call and
    the communicator size, so that a scaling loss shows whether it is skew or the collective.
    Gathered over the gloo control plane (also in --dry-run, with null values)."""
    vals = [None] * world
    dist.all_gather_object(vals, {"kernel_ms": k_ms, "allgather_us": allgather_us})
    ks = [v["kernel_ms"] for v in vals if v["kernel_ms"] is not None]
    ag = [v["allgather_us"] for v in vals if v["allgather_us"] is not None]
    return {"ranks": world, "rccl_nranks": rccl_nranks,
            "kernel_ms_max": max(ks) if ks else None, "kernel_ms_min": min(ks) if ks else None,
            "kernel_skew": (max(ks) / min(ks) if ks and min(ks) > 0 else None),
            "allgather_us_per_call_max": max(ag) if ag else None,
            "per_rank": vals}


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv):
    """--gpus N with WORLD_SIZE unset: start N rank processes (one per GPU) with the
    torch.distributed environment set, before this process touches any GPU; rank 0 prints the
    result line.  Returns the worst exit code."""
    port = free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--mapping", default="auto", choices=["auto", "lane", "wave"],
                    help="thread mapping of the Euler recursion (DESIGN.md §2)")
    ap.add_argument("--dry-run", action="store_true",
                    help="rendezvous the ranks and exit before any GPU work (launcher test)")
    ap.add_argument("--repeats", type=int, default=5,
                    help="extra timed runs of the same K steps after the timed region: their "
                         "median and mean ms/step are reported beside the headline")
    ap.add_argument("--api", default="run", choices=["run", "calls"],
                    help="run: the K steps as one dmt_mcmc_run call (headline); calls: the "
                         "caller's loop of separate draw / accept / fetch_ll C calls as value")
    ap.add_argument("--calls-iters", type=int, default=200,
                    help="iterations of the separate-call loop measured beside the headline")
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only; the data path is RCCL in libdmt
        assert dist.get_world_size() == world
    if args.dry_run:
        diag = None
        if dist is not None:
            dist.barrier()
            diag = rank_diagnostics(dist, world, None, None, None)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": world,
                              "rank_diagnostics": diag}))
        if dist is not None:
            dist.destroy_process_group()
        return 0

    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import _lib as L
    from diffusionmcmctools_amd import workloads as W

    w = build_workload(args.config, rank)
    w.meta["hist_len"] = (args.warmup + args.steps * (3 + max(args.repeats, 0)) + EXTRA_ITERS +
                          CPU_MAX_ITERS + 2 * args.calls_iters)
    mapping = {"auto": L.MAP_AUTO, "lane": L.MAP_LANE, "wave": L.MAP_WAVE}[args.mapping]
    ens = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision,
                       seed=ens_seed, device=local_rank, grid_shared=w.grid_shared,
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
    rccl_nranks = ens.comm_size()
    if world > 1 and rccl_nranks != world:
        raise SystemExit(f"bench.py: RCCL communicator has {rccl_nranks} ranks, expected {world}")
    ens.loglikhd(lay, L.U, 0, B)

    # one step = draw_proposal_path!(be); accept_reject_proposal_path!(be, i); fetch_ll(be).
    # The K timed steps are queued back to back on the device (dmt_mcmc_run: no host round
    # trip per iteration; every iteration's fetch_ll values come back at the end).

    def barrier():
        ens.sync()
        if dist is not None:
            dist.barrier()

    # W untimed warm-up steps, issued as separate one-iteration calls (the host path warms over
    # the first calls: DESIGN.md §6), and the timed call's result buffer made beforehand
    for it in range(1, args.warmup + 1):
        ens.mcmc_run(lay, 0, B, it, 1)
    ens.prepare_run(args.steps)
    barrier()
    # The timed region holds the K steps and nothing else: no timing events (they cost ≈ 10 µs
    # of event completion per call); the kernel's own duration comes from the
    # same K steps re-run with HIP events right after it (below) and from rocprofv3.
    t0 = time.perf_counter()
    if args.api == "calls":
        # the caller's loop of separate C calls (deferred draw fused with its accept, fetch_ll
        # from the fused tree), timed by the same clock as the headline; the untimed Python
        # comparison loop of separate_calls runs after it
        _, _, res = separate_calls(ens, lay, B, args.warmup + 1, args.steps, world > 1,
                                   python=False)
    else:
        res = ens.mcmc_run(lay, 0, B, args.warmup + 1, args.steps, copy=False)
    barrier()
    el = time.perf_counter() - t0
    recent = L.recent_kernels()  # the kernels the timed call dispatched (dmt_recent_kernels)
    n_acc = float(res[:, 2].sum())  # read before any later run of this length reuses the buffer
    done = args.warmup + args.steps  # iterations run so far
    # The dominant kernel's launch duration: HIP events recorded on libdmt's stream around the
    # launches of the same K steps, run twice right after the timed region (same launch shape,
    # same state; the first event-recording call is not the one averaged alone).
    ens.set_timing(True, kernels=[L.K_DRAW])
    for _ in range(2):
        if args.api == "calls":
            separate_calls(ens, lay, B, done + 1, args.steps, world > 1, python=False)
        else:
            ens.mcmc_run(lay, 0, B, done + 1, args.steps)
        done += args.steps
    ens.sync()
    k_ms, k_n = ens.get_timing(L.K_DRAW)  # k_n counts iterations (persistent) or launches
    k_ms /= 2.0  # per K steps
    persist = w.model.kind == L.MODEL_OU and os.environ.get("DMT_MCMC_PERSIST", "1") != "0"
    a_ms = a_n = 0
    if not persist:
        # the accept+reduce kernel, timed on a few extra iterations
        ens.set_timing(True, kernels=[L.K_ACCEPT])
        ens.mcmc_run(lay, 0, B, done + 1, EXTRA_ITERS)
        a_ms, a_n = ens.get_timing(L.K_ACCEPT)
        done += EXTRA_ITERS
    ens.set_timing(False)
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # repeats of the same K steps (median and mean beside the headline)
    rep_ms = []
    for _ in range(max(args.repeats, 0)):
        barrier()
        t1 = time.perf_counter()
        ens.mcmc_run(lay, 0, B, done + 1, args.steps)
        barrier()
        rep_ms.append((time.perf_counter() - t1) / args.steps * 1e3)
        done += args.steps
    # the caller's separate-call loop beside the fused headline
    calls = None
    if args.calls_iters > 0 and args.api == "run":
        c_us, py_us, _ = separate_calls(ens, lay, B, done + 1, args.calls_iters, world > 1)
        done += 2 * args.calls_iters
        calls = {"loop": "draw_proposal_path!(be); accept_reject_proposal_path!(be, i); "
                         "fetch_ll(be); fetch_ll°(be) as separate C-ABI calls",
                 "us_per_iteration_c": c_us, "us_per_iteration_python_ctypes": py_us,
                 "steps_per_s_c": w.steps_per_iter / (c_us * 1e-6),
                 "iterations": args.calls_iters,
                 "fused_launch_per_iteration": os.environ.get("DMT_DEFER", "1") != "0"}
    diag = None
    if dist is not None:
        # all-gather cost per call: global (collective) minus local fetch_ll, 20 calls each
        ens.sync()
        t1 = time.perf_counter()
        for _ in range(20):
            ens.fetch_ll(lay, 0, B, 0, local=True)
        loc = time.perf_counter() - t1
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(20):
            ens.fetch_ll(lay, 0, B, 0)
        glob = time.perf_counter() - t1
        diag = rank_diagnostics(dist, world, k_ms, (glob - loc) / 20 * 1e6, rccl_nranks)

    steps_total = w.steps_per_iter * args.steps * world
    value = steps_total / el
    # launches of the dominant kernel in the timed region: one per iteration, or (persistent,
    # dmt_mcmc_run) one per chunk of iterations (dmt_runtime.hip: ≤ 64 MiB of partials)
    it_per_launch = (min(args.steps, max(1, (64 << 20) // (24 * B)))
                     if persist and args.api == "run" else 1)
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
    if resident:  # linear drift: all K iterations in one k_mcmc_resident(_pc) launch (dmt_mcmc_run)
        wave = True
        kname = ("k_mcmc_resident_pc" if os.environ.get("DMT_MCMC_PC", "1") != "0"
                 else "k_mcmc_resident")
    elif persist:  # linear drift: all K iterations in one k_mcmc_scan launch (dmt_mcmc_run)
        wave, kname = True, "k_mcmc_scan"
    elif short1 and os.environ.get("DMT_SCAN_RESIDENT", "1") != "0":  # one launch per iteration
        wave, kname = True, "k_block_resident"
    elif w.model.kind == L.MODEL_OU:  # linear drift: the affine-scan kernel per iteration
        wave, kname = True, "k_block_scan"
    elif wave:
        kname = "k_block_wave"
    else:  # lane mapping: fp32 ensembles on lane packets (dmt_create; DMT_PATH_PACKETS=0: rows),
        # with fewer recording tiles than SIMDs on producer/consumer waves (DMT_LANE_SPLIT=0: one)
        pk = w.precision == L.F32 and os.environ.get("DMT_PATH_PACKETS", "1") != "0"
        split = (os.environ.get("DMT_LANE_SPLIT", "-1") != "0"
                 and all(len(r) == 1 for r in w.n_points) and B // 64 < 1024)
        kname = ("k_block_ps_pk<" if pk and split else "k_block_pk<" if pk else "k_block<")
    # the draw kernel the library actually dispatched in the timed call, when it reports one
    # (the restatement above is the fallback for a library without dmt_recent_kernels)
    kname = dispatched_kernel(recent) or kname
    # committed profile summaries of THIS source tree only (scripts/provenance.py)
    tr, traffic_stale = committed_summary("traffic", args.config, kname)
    traffic = tr["traffic_bytes_per_unit"] * it_per_launch if tr else None  # per launch
    traffic_src = tr["source"] if tr else None
    issue, issue_stale = committed_summary("issue", args.config, kname)
    rp, rp_stale = committed_summary("kstats", args.config, kname)
    rp_us = None
    if rp is not None and rp.get("units_per_launch", 1) == it_per_launch:  # same launch shape
        rp_us = rp["avg_us"]
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(w, ens, lay, done + 1, budget_s=args.cpu_budget)
        desc, dtype = WORKLOADS[args.config]
        frac = achieved / PEAK_HBM_GBS
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
                       "rccl_nranks": rccl_nranks,
                       "mapping": ("scan-resident" if resident else
                                   "scan-persistent" if persist else
                                   "scan-resident-per-iteration" if kname == "k_block_resident" else
                                   "scan" if kname == "k_block_scan" else
                                   "wave" if wave else
                                   "lane-packets" if kname in ("k_block_pk<", "k_block_ps_pk<")
                                   else "lane"),
                       "rng": "device Philox4x32-10 + Box-Muller (perf mode)"},
            "per_gpu": value / world,
            "accept_rate": accept_rate,
            # bound: what the counters show for this kernel (issue summary), HBM otherwise
            "roofline": {"bound": (issue or {}).get("bound", "hbm"), "achieved": achieved,
                         "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": frac, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": kname + (" (draw_proposal_path! + accept_reject_proposal_path! "
                                            "+ fetch_ll of every iteration of the launch)" if persist else
                                            " (draw_proposal_path!)"),
                         "kernel_avg_us": k_avg_s * 1e6,
                         # the same kernel's average dispatch in the committed rocprofv3 trace of
                         # this config (the profiler's clock; the line's own figure is HIP events)
                         "kernel_avg_us_rocprof": rp_us,
                         "frac_rocprof": (bytes_launch / (rp_us * 1e-6) / 1e9 / PEAK_HBM_GBS
                                          if rp_us else None),
                         "rocprof_source": (rp or {}).get("source"),
                         "kernel_timing": ("HIP events on libdmt's stream around the same K "
                                           "steps, re-run twice right after the timed region"),
                         "source_tree": tree_digest(),
                         # newest committed summaries that measured another tree (not quoted)
                         "stale_summaries": {k: v for k, v in (("traffic", traffic_stale),
                                                               ("issue", issue_stale),
                                                               ("kstats", rp_stale)) if v},
                         "kernel_us_per_iteration": k_iter_s * 1e6,
                         "iterations_per_launch": it_per_launch,
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "algorithmic_bytes_per_iteration": bytes_iter,
                         "bytes_per_step": algorithmic_bytes_per_step(w),
                         "hbm_frac_from_traffic": (traffic / k_avg_s / 1e9 / PEAK_HBM_GBS
                                                   if traffic and k_avg_s > 0 else None),
                         "limiter": (issue or {}).get("limiter"),
                         "issue": issue},
            "accept_kernel_avg_us": (a_ms / a_n) * 1e3 if a_n else None,
            "api": args.api,
            "repeats": {"n": len(rep_ms),
                        "ms_per_step_median": float(np.median(rep_ms)) if rep_ms else None,
                        "ms_per_step_mean": float(np.mean(rep_ms)) if rep_ms else None,
                        "value_median": (w.steps_per_iter * world / (np.median(rep_ms) * 1e-3)
                                         if rep_ms else None)},
            "separate_calls": calls,
            "rank_diagnostics": diag,
            "cpu_baseline": cpu,
        }
        if cpu is not None:
            line["accept_rate_cpu"] = cpu["accept_rate"]
            line["decisions_identical"] = cpu["decisions_identical"]
            line["decisions_total"] = cpu["decisions_total"]
        print(json.dumps(line), flush=True)
    ens.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
