"""Multi-rank sharding on CPU (gloo, world_size 2): a BlockEnsemble split into recording
shards, each rank keyed by global segment ids (set_shard) and combining fetch_ll partials in
rank order, reproduces the unsharded ensemble bit for bit (shard.py).  The
numerics run on the oracle backend here; the GPU test drives two libdmt shards on one device."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B_LOCAL, N, ITERS, SEED = 8, 40, 3, 77


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(ens, lay, nb):
    """Perf-mode MCMC iterations (device-RNG streams), returning per-iteration partials."""
    ens.loglikhd(lay, 0, 0, nb)
    parts = []
    for i in range(1, ITERS + 1):
        ens.draw_proposal(lay, 0, nb, Z=None, iter=i)
        ens.accept_reject(lay, 0, nb, i)
        parts.append(ens.fetch_ll(lay, 0, nb, i))
    ll = ens.get_block_state(lay, 0, 0, nb)
    return parts, ll


def _worker(rank, world, port, out_dir):
    import sys
    for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import oracle as orc
    from diffusionmcmctools_amd import workloads as W
    from diffusionmcmctools_amd import shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    w = W.c2_ou2d(B=B_LOCAL, N=N, block_offset=rank)
    w.meta["hist_len"] = ITERS
    ens = orc.OracleEnsemble(w.model.kind, w.d, w.m, w.n_points, prec=w.precision, seed=SEED,
                             grid_shared=w.grid_shared)
    ens.set_shard(shard.segment_base([len(r) for r in w.n_points] * world, rank * B_LOCAL))
    lay = W.fill(ens, w, init_Z=True)
    parts, ll = _run(ens, lay, w.nblocks)
    glob = [shard.combine_partials(p) for p in parts]
    np.save(os.path.join(out_dir, f"ll{rank}.npy"), ll)
    np.save(os.path.join(out_dir, f"glob{rank}.npy"), np.array(glob))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_helpers():
    from diffusionmcmctools_amd import shard
    assert [shard.shard_range(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
    assert shard.segment_base([4, 6, 5], 2) == 10
    assert shard.rank_tree([1.0, 2.0, 3.0]) == (1.0 + 2.0) + (3.0 + 0.0)


@pytest.mark.parametrize("nranks", [1, 2, 3, 6, 8])
def test_rank_combine_host_path_matches_rank_tree(dmt, nranks):
    """libdmt's host combination of all-gathered partials (dmt_combine_rank_partials: the code
    finish_reduction and mcmc_run_collect run after ncclAllGather) against shard.rank_tree,
    bit for bit, for every iteration and component: synthetic partials of mixed magnitudes and
    signs (so that any other summation order would round differently), -inf and 0."""
    from diffusionmcmctools_amd import shard
    rng = np.random.default_rng(nranks)
    n_iter = 7
    allp = rng.standard_normal((nranks, n_iter, 3)) * 10.0 ** rng.integers(-8, 9, (nranks, n_iter, 3))
    allp[:, :, 2] = rng.integers(0, 1 << 20, (nranks, n_iter))  # accepted counts
    allp[0, 3, 1] = -np.inf
    allp[-1, 4, 0] = 0.0
    out = dmt.combine_rank_partials(allp)
    assert out.shape == (n_iter, 3)
    for i in range(n_iter):
        for c in range(3):
            want = shard.rank_tree(allp[:, i, c])
            got = out[i, c]
            assert (got == want) or (np.isnan(got) and np.isnan(want)), (nranks, i, c, got, want)
            assert np.signbit(got) == np.signbit(want)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_rank_combine_of_power_of_two_shards_is_the_global_tree(dmt, orc, nranks):
    """Power-of-two blocks per rank: each rank's fetch_ll subtree, combined by libdmt's host
    step, equals the single-ensemble tree over all blocks — the property that
    makes an N-GPU job bit-identical to one ensemble.  Block values from a real oracle run."""
    from diffusionmcmctools_amd import workloads as W
    B = 16
    g = W.concat_workloads([W.c2_ou2d(B=B, N=30, block_offset=r) for r in range(nranks)])
    g.meta["hist_len"] = 2
    ens = orc.OracleEnsemble(g.model.kind, g.d, g.m, g.n_points, prec=g.precision, seed=SEED,
                             grid_shared=g.grid_shared)
    lay = W.fill(ens, g, init_Z=True)
    nb = g.nblocks
    ens.loglikhd(lay, 0, 0, nb)
    ens.draw_proposal(lay, 0, nb, Z=None, iter=1)
    ens.accept_reject(lay, 0, nb, 1)
    want = ens.fetch_ll(lay, 0, nb, 1)
    per_rank = np.array([ens.fetch_ll(lay, r * B, (r + 1) * B, 1) for r in range(nranks)])
    got = dmt.combine_rank_partials(per_rank)[0]
    np.testing.assert_array_equal(got, np.asarray(want, dtype=np.float64))


def test_two_rank_shards_match_unsharded(tmp_path):
    import torch.multiprocessing as mp
    import oracle as orc
    from diffusionmcmctools_amd import workloads as W
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    ws = [W.c2_ou2d(B=B_LOCAL, N=N, block_offset=r) for r in range(world)]
    g = W.concat_workloads(ws)
    g.meta["hist_len"] = ITERS
    ens = orc.OracleEnsemble(g.model.kind, g.d, g.m, g.n_points, prec=g.precision, seed=SEED,
                             grid_shared=g.grid_shared)
    lay = W.fill(ens, g, init_Z=True)
    parts, ll = _run(ens, lay, g.nblocks)
    ll_sharded = np.concatenate([np.load(tmp_path / f"ll{r}.npy") for r in range(world)])
    np.testing.assert_array_equal(ll_sharded, ll)
    for r in range(world):
        glob = np.load(tmp_path / f"glob{r}.npy")
        np.testing.assert_array_equal(glob, np.array(parts, dtype=np.float64))


@pytest.mark.gpu
def test_gpu_shards_match_unsharded():
    """Two libdmt shards (set_shard) on one GPU vs one ensemble holding both: identical paths,
    ll and decisions; host rank tree of the shard partials == the unsharded fetch_ll."""
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import workloads as W
    from diffusionmcmctools_amd import shard
    world, B = 2, 256
    ws = [W.c2_ou2d(B=B, N=100, block_offset=r) for r in range(world)]
    g = W.concat_workloads(ws)
    for w in ws + [g]:
        w.meta["hist_len"] = ITERS

    def make(w, base):
        e = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=SEED,
                         grid_shared=w.grid_shared)
        e.set_shard(base)
        return e, W.fill(e, w, init_Z=True)

    shards = [make(w, r * B) for r, w in enumerate(ws)]
    full, lay = make(g, 0)
    res_s = [_run(e, l, B) for e, l in shards]
    parts, ll = _run(full, lay, g.nblocks)
    np.testing.assert_array_equal(np.concatenate([r[1] for r in res_s]), ll)
    for i in range(ITERS):
        comb = tuple(shard.rank_tree([res_s[r][0][i][c] for r in range(world)]) for c in range(3))
        assert comb == tuple(float(x) for x in parts[i])
    X = np.concatenate([e.download_paths(1, 0) for e, _ in shards])
    np.testing.assert_array_equal(X, full.download_paths(1, 0))


@pytest.mark.gpu
def test_gpu_fhn_lane_shards_match_unsharded():
    """C3's per-rank scale on the lane mapping: two FHN shards of 32 768 blocks × 1000 steps
    (set_shard: global segment ids key the device streams) against one ensemble of 65 536 —
    identical paths, ll, decisions and rank-tree fetch_ll over dmt_mcmc_run (the
    per-iteration kernels k_block / k_block_ps + k_accept_reduce)."""
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import workloads as W
    from diffusionmcmctools_amd import shard
    from diffusionmcmctools_amd import _lib as L
    world, B, n = 2, 32768, 3
    ws = [W.c3_fhn(B=B, T_burn=0.05, block_offset=r) for r in range(world)]
    g = W.concat_workloads(ws)
    for w in ws + [g]:
        w.meta["hist_len"] = n

    def make(w, base):
        e = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=SEED,
                         grid_shared=w.grid_shared, mapping=L.MAP_LANE)
        e.set_shard(base)
        lay = W.fill(e, w, init_Z=True)
        e.loglikhd(lay, 0, 0, w.nblocks)
        return e, lay

    shards = [make(w, r * B) for r, w in enumerate(ws)]
    full, lay = make(g, 0)
    res_s = [e.mcmc_run(l, 0, B, 1, n, salt=3) for e, l in shards]
    res_f = full.mcmc_run(lay, 0, g.nblocks, 1, n, salt=3)
    for i in range(n):
        comb = tuple(shard.rank_tree([res_s[r][i][c] for r in range(world)]) for c in range(3))
        assert comb == tuple(float(x) for x in res_f[i])
    for what in (L.BLK_LL, L.BLK_LLPROP):
        np.testing.assert_array_equal(
            np.concatenate([e.get_block_state(l, what, 0, B) for e, l in shards]),
            full.get_block_state(lay, what, 0, g.nblocks))
    np.testing.assert_array_equal(
        np.concatenate([e.get_block_state(l, L.BLK_ACC_HIST, 0, B, hist_len=n)
                        for e, l in shards], axis=1),
        full.get_block_state(lay, L.BLK_ACC_HIST, 0, g.nblocks, hist_len=n))
    for unit in (L.U, L.UPROP):
        X = np.concatenate([e.download_paths(unit, 0) for e, _ in shards])
        np.testing.assert_array_equal(X, full.download_paths(unit, 0))
    for e, _ in shards + [(full, lay)]:
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("persist", ["1", "0"])
def test_rccl_allgather_path_single_rank(monkeypatch, persist):
    """The RCCL path of fetch_ll / dmt_mcmc_run (ncclCommInitRank, ncclAllGather, the host
    rank-order tree) on a one-rank communicator (DMT_COMM_FORCE): results identical to the
    communicator-free path, for the persistent and the per-iteration MCMC kernels."""
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import workloads as W
    monkeypatch.setenv("DMT_COMM_FORCE", "1")
    monkeypatch.setenv("DMT_MCMC_PERSIST", persist)
    w = W.c2_ou2d(B=300, N=100)
    w.meta["hist_len"] = 12
    ens = []
    for k in range(2):
        e = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=SEED,
                         grid_shared=w.grid_shared)
        lay = W.fill(e, w)
        if k == 1:
            e.comm_init(1, 0, dmt.comm_unique_id())
        e.loglikhd(lay, 0, 0, w.nblocks)
        ens.append(e)
    r = [e.mcmc_run(lay, 0, w.nblocks, 1, 10) for e in ens]
    np.testing.assert_array_equal(r[0], r[1])
    f = [e.fetch_ll(lay, 0, w.nblocks, 10) for e in ens]
    assert f[0] == f[1]
    for e in ens:
        e.close()



def test_collection_level_calls_are_rank_local():
    """A BiBlock's or BlockCollection's fused mcmc_step / mcmc_run and fetch_ll are this
    rank's (src/block_collection.jl:144,156): they reach libdmt as the *_local entry points
    (no collective, so one rank may call them alone); only the BlockEnsemble's are global."""
    import oracle as orc
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import workloads as W
    w = W.c2_ou2d(B=4, N=20)
    w.meta["hist_len"] = 6
    calls = []

    class Recorder(orc.OracleEnsemble):
        depth = 0

        def _rec(self, name, local, fn, *a, **k):
            if Recorder.depth == 0:  # the API's calls, not the oracle's own nested ones
                calls.append((name, local))
            Recorder.depth += 1
            try:
                return fn(*a, local=local, **k)
            finally:
                Recorder.depth -= 1

        def mcmc_run(self, *a, local=False, **k):
            return self._rec("run", local, super().mcmc_run, *a, **k)

        def mcmc_step(self, *a, local=False, **k):
            return self._rec("step", local, super().mcmc_step, *a, **k)

        def fetch_ll(self, *a, local=False, **k):
            return self._rec("fetch", local, super().fetch_ll, *a, **k)

    eng = Recorder(w.model.kind, w.d, w.m, w.n_points, prec=w.precision, seed=1,
                   grid_shared=w.grid_shared)
    se = dmt.SamplingEnsemble(w.model, w.n_points, _engine=eng)
    W.fill(eng, w, init_Z=True)
    be = dmt.BlockEnsemble(se, [[range(0, 1)]] * 4, rho=0.5, ll_hist_len=6)
    for x, local in ((be.recordings[1], True), (be.recordings[2].blocks[0], True), (be, False)):
        calls.clear()
        x.mcmc_run(1, 2)
        x.mcmc_step(3)
        x.fetch_ll()
        assert calls[:2] == [("run", local), ("step", local)], calls
        if not isinstance(x, dmt.BiBlock):  # a BiBlock reads its ll directly
            assert ("fetch", local) in calls[2:], calls


def _gpu_worker(rank, world, port, out_dir, B):
    """One rank process: its libdmt shard on device 0 (both ranks share the one GPU of the
    box), fetch_ll partials combined over gloo with the rank-order tree (shard.rank_tree)."""
    import sys
    for p in (ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import workloads as W
    from diffusionmcmctools_amd import shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    w = W.c3_fhn(B=B, N=200, T_burn=0.05, block_offset=rank)
    w.meta["hist_len"] = ITERS
    e = dmt.Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=SEED,
                     grid_shared=w.grid_shared)
    e.set_shard(rank * B)
    lay = W.fill(e, w, init_Z=True)
    e.loglikhd(lay, 0, 0, B)
    res = e.mcmc_run(lay, 0, B, 1, ITERS, salt=3, local=True)   # this rank's partials
    allres = [None] * world
    dist.all_gather_object(allres, res.tolist())
    comb = [[shard.rank_tree([allres[r][i][c] for r in range(world)]) for c in range(3)]
            for i in range(ITERS)]
    np.save(os.path.join(out_dir, f"X{rank}.npy"), e.download_paths(0, 0))
    if rank == 0:
        np.save(os.path.join(out_dir, "comb.npy"), np.array(comb))
    e.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_two_rank_processes_match_unsharded(tmp_path):
    """Two rank PROCESSES (gloo control plane, world size 2), each with its own libdmt handle
    on the box's one GPU holding one recording shard: paths and the rank-tree fetch_ll of every
    iteration equal one process's unsharded ensemble bit for bit — the multi-process form of
    the N-GPU job on real hardware (the RCCL all-gather itself needs one GPU per rank)."""
    import torch.multiprocessing as mp
    import diffusionmcmctools_amd as dmt
    from diffusionmcmctools_amd import workloads as W
    world, B = 2, 256  # power-of-two blocks per rank: the rank tree is a subtree split
    mp.start_processes(_gpu_worker, args=(world, _free_port(), str(tmp_path), B), nprocs=world,
                       join=True, start_method="spawn")
    g = W.concat_workloads([W.c3_fhn(B=B, N=200, T_burn=0.05, block_offset=r)
                            for r in range(world)])
    g.meta["hist_len"] = ITERS
    e = dmt.Ensemble(g.model.kind, g.d, g.m, g.n_points, precision=g.precision, seed=SEED,
                     grid_shared=g.grid_shared)
    lay = W.fill(e, g, init_Z=True)
    e.loglikhd(lay, 0, 0, g.nblocks)
    full = e.mcmc_run(lay, 0, g.nblocks, 1, ITERS, salt=3)
    np.testing.assert_array_equal(np.load(tmp_path / "comb.npy"), full)
    X = np.concatenate([np.load(tmp_path / f"X{r}.npy") for r in range(world)])
    np.testing.assert_array_equal(X, e.download_paths(0, 0))
    e.close()
