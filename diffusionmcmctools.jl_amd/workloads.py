"""Synthetic workloads of BASELINE.json's configs, seeded.

Each builder returns a ``Workload``: reference-layout host arrays (time grid, guiding-term
tables, law records, initial state, normals for the initial draw) plus the block layout.
The same arrays feed libdmt (``load_device``) and the CPU oracle in tests.

  C1  1D OU bridge, 1 block × 200 steps (CPU-scale plumbing case)
  C2  2D OU bridge, 1 024 blocks × 500 steps, fp64          (bench headline)
  C3  FitzHugh–Nagumo, 65 536 blocks × 1 000 steps, fp64
  C4  C3 sharded over ranks (65 536 blocks per GPU)
  C5  Lorenz-63, fp32, 262 144 blocks × 2 000 steps (32 768 per GPU on 8)
"""
from __future__ import annotations

import math
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .models import (FHN, OU, Lorenz, Observation, packed, standard_guid_prop_time_transf,
                     guiding_chain)


@dataclass
class Workload:
    name: str
    model: object
    precision: int
    n_points: list            # per recording, per segment
    t: np.ndarray             # shared grid (Q0) or flat (P)
    grid_shared: bool
    H: np.ndarray             # shared (Q0 × hp) or flat (P × hp)
    H_shared: bool
    F: np.ndarray             # P × d
    laws: np.ndarray          # G × LAW_STRIDE
    X0: np.ndarray            # P × d  (only each recording's first point matters)
    Z0: np.ndarray            # S × m  normals of the initial (fresh) draw
    rho: float
    n_blocks: np.ndarray = None
    seg_first: np.ndarray = None
    seg_last: np.ndarray = None
    last: np.ndarray = None
    meta: dict = field(default_factory=dict)

    @property
    def d(self):
        return self.model.d

    @property
    def m(self):
        return self.model.m

    @property
    def nblocks(self):
        return int(np.sum(self.n_blocks))

    @property
    def steps_per_iter(self):
        return int(sum(n - 1 for r in self.n_points for n in r))


def _terminal_layout(w: Workload):
    R = len(w.n_points)
    w.n_blocks = np.ones(R, dtype=np.int32)
    w.seg_first = np.zeros(R, dtype=np.int32)
    w.seg_last = np.array([len(r) - 1 for r in w.n_points], dtype=np.int32)
    w.last = np.ones(R, dtype=np.uint8)


def _single_segment_workload(name, model, prec, B, t, auxes, infos, x0s, rho, seed_z, H_shared,
                             threads=16):
    """B recordings × 1 segment, shared grid t.  auxes/infos: per block (or one shared aux)."""
    d, m = model.d, model.m
    hp = d * (d + 1) // 2
    npts = t.size
    if H_shared:
        # H depends only on the aux law and the observation operator/noise: one table.
        (H, F0, c0), = guiding_chain([auxes[0]], [t], [infos[0]])
        Hs = H
        Fs = np.empty((B, npts, d))
        cs = np.empty(B)
        # F, c depend on v: recompute per block (cheap for the OU configs)
        def one(b):
            (_, F, c), = guiding_chain([auxes[0]], [t], [infos[b]])
            Fs[b] = F
            cs[b] = c[0]
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, range(B)))
        Hflat = Hs
    else:
        Hb = np.empty((B, npts, hp))
        Fs = np.empty((B, npts, d))
        cs = np.empty(B)

        def one(b):
            (H, F, c), = guiding_chain([auxes[b]], [t], [infos[b]])
            Hb[b], Fs[b], cs[b] = H, F, c[0]
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, range(B)))
        Hflat = Hb.reshape(B * npts, hp)
    laws = np.stack([model.law_record(auxes[b if len(auxes) > 1 else 0], cs[b]) for b in range(B)])
    X0 = np.zeros((B, npts, d))
    X0[:, 0, :] = x0s
    rng = np.random.default_rng(seed_z)
    Z0 = rng.standard_normal((B * (npts - 1), m))
    w = Workload(name, model, prec, [[npts]] * B, t, True, Hflat, H_shared,
                 Fs.reshape(B * npts, d), laws, X0.reshape(B * npts, d), Z0, rho)
    _terminal_layout(w)
    return w


def c1_ou1d(N=200):
    """1D OU θ=1, μ=0, σ=0.5 on [0,1], x0=0, one obs v=0.3 (Σ=0.01); aux OU θ̃=0.5."""
    model = OU([[1.0]], [0.0], [[0.5]])
    aux = model.aux(Theta_t=[[0.5]])
    t = standard_guid_prop_time_transf(0.0, 1.0, 1.0 / N)
    ob = Observation(1.0, np.array([0.3]), np.eye(1), 0.01 * np.eye(1))
    return _single_segment_workload("C1-ou1d", model, L.F64, 1, t, [aux], [ob.info()],
                                    np.zeros((1, 1)), 0.5, 100, H_shared=True)


def c2_ou2d(B=1024, N=500, seed=1, block_offset=0):
    """2D OU Θ=[[1,.3],[-.3,.8]], μ=0, σ=0.5I, aux Θ̃=diag(.5,.5); B blocks × N steps on [0,1];
    x0 ~ N(0,I) (seed), v = x0 + N(0, 0.1² I), Σ = 0.01 I; ρ = 0.9."""
    model = OU([[1.0, 0.3], [-0.3, 0.8]], [0.0, 0.0], 0.5 * np.eye(2))
    aux = model.aux(Theta_t=np.diag([0.5, 0.5]))
    t = standard_guid_prop_time_transf(0.0, 1.0, 1.0 / N)
    rng = np.random.default_rng([seed, block_offset])
    x0 = rng.standard_normal((B, 2))
    v = x0 + 0.1 * np.random.default_rng([seed + 1, block_offset]).standard_normal((B, 2))
    infos = [Observation(1.0, v[b], np.eye(2), 0.01 * np.eye(2)).info() for b in range(B)]
    w = _single_segment_workload("C2-ou2d", model, L.F64, B, t, [aux], infos, x0, 0.9,
                                 [seed + 2, block_offset], H_shared=True)
    w.meta.update(v=v)
    return w


def _fhn_states(model, B, seed, T_burn=1.0, dt_burn=1e-3, T_obs=0.1, dt_obs=1e-4):
    """Start points from a burned-in target run; end values from a fine forward simulation
    over the observation interval (vectorised Euler–Maruyama over B chains)."""
    rng = np.random.default_rng(seed)
    x = np.tile(np.array([-0.9, -1.0]), (B, 1))

    def run(x, T, h):
        for _ in range(int(round(T / h))):
            y, v = x[:, 0], x[:, 1]
            dy = (y - y ** 3 - v + model.s) / model.eps
            dv = model.gamma * y - v + model.beta
            x = np.stack([y + dy * h, v + dv * h + model.sg * math.sqrt(h) * rng.standard_normal(B)], 1)
        return x
    x0 = run(x, T_burn, dt_burn)
    xT = run(x0, T_obs, dt_obs)
    return x0, xT, rng


def c3_fhn(B=65536, N=1000, seed=100, block_offset=0, T_burn=1.0):
    """FHN θ=(0.1,-0.8,1.5,0,0.3), obs L=[1 0], Σ=0.01, interval 0.1, N steps (dt=1e-4 before
    the time change); aux = FHN linearised at the observed end value; ρ = 0.96."""
    model = FHN(0.1, -0.8, 1.5, 0.0, 0.3)
    x0, xT, rng = _fhn_states(model, B, [seed, block_offset], T_burn=T_burn)
    v = xT[:, 0] + 0.1 * rng.standard_normal(B)
    t = standard_guid_prop_time_transf(0.0, 0.1, 0.1 / N)
    auxes = [model.aux(v[b]) for b in range(B)]
    Lm = np.array([[1.0, 0.0]])
    infos = [Observation(0.1, np.array([v[b]]), Lm, 0.01 * np.eye(1)).info() for b in range(B)]
    w = _single_segment_workload("C3-fhn", model, L.F64, B, t, auxes, infos, x0, 0.96,
                                 [seed + 1, block_offset], H_shared=False)
    w.meta.update(v=v)
    return w


def c5_lorenz(B=32768, N=2000, seed=7, block_offset=0, T=0.2):
    """Lorenz-63 (10, 28, 8/3), σ = I, fp32; full-state obs Σ = 0.1 I at T; aux linearised at
    the observation; ρ = 0.9."""
    model = Lorenz(10.0, 28.0, 8.0 / 3.0, (1.0, 1.0, 1.0))
    rng = np.random.default_rng([seed, block_offset])
    x = rng.standard_normal((B, 3)) * 5 + np.array([0.0, 0.0, 25.0])
    h = 1e-3
    for _ in range(500):  # burn-in onto the attractor
        x0_, x1_, x2_ = x[:, 0], x[:, 1], x[:, 2]
        dx = np.stack([10 * (x1_ - x0_), x0_ * (28 - x2_) - x1_, x0_ * x1_ - 8 / 3 * x2_], 1)
        x = x + dx * h + math.sqrt(h) * rng.standard_normal((B, 3))
    x0 = x.copy()
    for _ in range(int(round(T / 1e-4))):
        x0_, x1_, x2_ = x[:, 0], x[:, 1], x[:, 2]
        dx = np.stack([10 * (x1_ - x0_), x0_ * (28 - x2_) - x1_, x0_ * x1_ - 8 / 3 * x2_], 1)
        x = x + dx * 1e-4 + math.sqrt(1e-4) * rng.standard_normal((B, 3))
    v = x + math.sqrt(0.1) * rng.standard_normal((B, 3))
    t = standard_guid_prop_time_transf(0.0, T, T / N)
    auxes = [model.aux(v[b]) for b in range(B)]
    infos = [Observation(T, v[b], np.eye(3), 0.1 * np.eye(3)).info() for b in range(B)]
    w = _single_segment_workload("C5-lorenz", model, L.F32, B, t, auxes, infos, x0, 0.9,
                                 [seed + 1, block_offset], H_shared=False)
    w.meta.update(v=v)
    return w


CONFIGS = {"c1": c1_ou1d, "c2": c2_ou2d, "c3": c3_fhn, "c5": c5_lorenz}


def load_device(w: Workload, seed=0, device=0, init_Z=True, mapping=L.MAP_AUTO):
    """Create a libdmt ensemble holding the workload; initial paths by a fresh draw of u
    (init_paths!, src/sampling_unit.jl:83-87) with the workload's normals (or the device
    stream when init_Z is False), then u° = deepcopy(u) (src/sampling_pair.jl:51)."""
    from .engine import Ensemble
    ens = Ensemble(w.model.kind, w.d, w.m, w.n_points, precision=w.precision, seed=seed,
                   device=device, grid_shared=w.grid_shared, mapping=mapping)
    fill(ens, w, init_Z=init_Z)
    return ens


def fill(ens, w: Workload, init_Z=True):
    """Upload a workload into an Ensemble-like object (libdmt Ensemble or OracleEnsemble)."""
    ens.upload_grid(w.t)
    ens.upload_law(L.U, L.LAW_PP, H=w.H, F=w.F, laws=w.laws, H_shared=w.H_shared)
    ens.set_paths(L.U, X=w.X0)
    ens.draw_unit(L.U, Z=w.Z0 if init_Z else None, iter=0, salt=0xFFFF)
    X = ens.download_paths(L.U, 0)
    W = ens.download_paths(L.U, 1)
    ens.set_paths(L.UPROP, X=X, W=W)
    lay = ens.create_layout(w.n_blocks, w.seg_first, w.seg_last, w.last,
                            np.full(w.nblocks, w.rho), hist_len=w.meta.get("hist_len", 0))
    return lay


def concat_workloads(ws):
    """The global workload whose recording shards are ``ws`` (in rank order).  Shared grids
    and shared guiding tables must agree between shards."""
    w0 = ws[0]
    for w in ws[1:]:
        assert w.grid_shared == w0.grid_shared and w.H_shared == w0.H_shared
        if w0.grid_shared:
            assert np.array_equal(w.t, w0.t)
        if w0.H_shared:
            assert np.array_equal(w.H, w0.H)
    cat = lambda k: np.concatenate([getattr(w, k) for w in ws])  # noqa: E731
    g = Workload(w0.name, w0.model, w0.precision, [r for w in ws for r in w.n_points],
                 w0.t if w0.grid_shared else cat("t"), w0.grid_shared,
                 w0.H if w0.H_shared else cat("H"), w0.H_shared, cat("F"), cat("laws"),
                 cat("X0"), cat("Z0"), w0.rho)
    g.n_blocks, g.seg_first, g.seg_last, g.last = (cat(k) for k in
                                                   ("n_blocks", "seg_first", "seg_last", "last"))
    return g
