"""Thin object wrapper of one libdmt ensemble handle (reference-layout host arrays).

Host arrays follow the reference's in-memory layout (include/dmt.h): a segment's path is
``double[npts][d]`` (Julia ``Vector{SVector{d,Float64}}``) and segments are concatenated
recording-major.  Every call goes straight to the HIP library.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class Ensemble:
    """Device containers of a SamplingEnsemble (u and u°) plus its block layouts."""

    def __init__(self, model: int, d: int, m: int, n_points, precision: int = L.F64,
                 seed: int = 0, device: int = 0, grid_shared: bool = False,
                 mapping: int = L.MAP_AUTO):
        # n_points: list (per recording) of lists (per segment) of grid-point counts
        self.model, self.d, self.m, self.precision = int(model), int(d), int(m), int(precision)
        self.hp = self.d * (self.d + 1) // 2
        self.nseg = np.array([len(r) for r in n_points], dtype=np.int32)
        self.npts = np.array([int(n) for r in n_points for n in r], dtype=np.int32)
        self.R = len(self.nseg)
        self.G = len(self.npts)
        self.rec_seg0 = np.concatenate([[0], np.cumsum(self.nseg)]).astype(np.int64)
        self.pt_off = np.concatenate([[0], np.cumsum(self.npts)[:-1]]).astype(np.int64)
        self.st_off = (self.pt_off - np.arange(self.G)).astype(np.int64)
        self.P = int(self.npts.sum())
        self.S = self.P - self.G
        self.grid_shared = bool(grid_shared)
        self.Q0 = int(self.npts[: self.nseg[0]].sum())
        self._h = C.c_void_p()
        self._run_out = {}  # dmt_mcmc_run result buffers by run length (mcmc_run)
        self._hist_len = {0: 0}  # history length of each layout (dmt_get_block_state fills all)
        mdl = L.dmt_model(self.model, self.precision, self.d, self.m)
        st = L.dmt_structure(self.R, L.i32p(self.nseg), L.i32p(self.npts))
        cfg = L.dmt_config(int(seed) & (2**64 - 1), int(device), 1 if grid_shared else 0,
                           int(mapping))
        self.mapping = int(mapping)
        L.call("dmt_create", C.byref(self._h), C.byref(mdl), C.byref(st), C.byref(cfg))

    # ---------------------------------------------------------------- lifetime
    def close(self):
        if self._h:
            L.lib.dmt_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---------------------------------------------------------------- uploads
    def upload_grid(self, t):
        t = np.ascontiguousarray(t, dtype=np.float64)
        want = self.Q0 if self.grid_shared else self.P
        if t.size != want:
            raise ValueError(f"grid needs {want} values, got {t.size}")
        L.call("dmt_upload_grid", self._h, L.f64p(t))

    def upload_law(self, unit, kind, H=None, F=None, laws=None, H_shared=False):
        H = None if H is None else np.ascontiguousarray(H, dtype=np.float64)
        F = None if F is None else np.ascontiguousarray(F, dtype=np.float64)
        laws = None if laws is None else np.ascontiguousarray(laws, dtype=np.float64)
        if H is not None:
            want = (self.Q0 if H_shared else self.P) * self.hp
            if H.size != want:
                raise ValueError(f"H needs {want} values, got {H.size}")
        if F is not None and F.size != self.P * self.d:
            raise ValueError("F has the wrong size")
        if laws is not None and laws.size != self.G * L.LAW_STRIDE:
            raise ValueError("laws has the wrong size")
        L.call("dmt_upload_law", self._h, unit, kind, L.f64p(H), 1 if H_shared else 0,
               L.f64p(F), L.f64p(laws))

    def upload_aux(self, kind, aux):
        """dmt_upload_aux(_a): per-point B̃(t_i), β̃(t_i) ([P][d·d + d]) — or B̃, β̃, ã(t_i) packed
        ([P][d·d + d + d(d+1)/2]) — of the laws of `kind` (u and u° alike) for segments whose
        record has LAW_AUXTD set (2: ã from the table too); None removes the table."""
        if aux is None:
            L.call("dmt_upload_aux", self._h, int(kind), None)
            return
        aux = np.ascontiguousarray(aux, dtype=np.float64)
        nb = self.d * self.d + self.d
        na = nb + self.d * (self.d + 1) // 2
        if aux.size not in (self.P * nb, self.P * na):
            raise ValueError("aux needs P·(d·d + d) or P·(d·d + d + d(d+1)/2) values")
        L.call("dmt_upload_aux_a", self._h, int(kind), L.f64p(aux), aux.size // self.P)

    def set_paths(self, unit, X=None, W=None):
        X = None if X is None else np.ascontiguousarray(X, dtype=np.float64)
        W = None if W is None else np.ascontiguousarray(W, dtype=np.float64)
        if X is not None and X.size != self.P * self.d:
            raise ValueError("X has the wrong size")
        if W is not None and W.size != self.P * self.m:
            raise ValueError("W has the wrong size")
        L.call("dmt_set_paths", self._h, unit, L.f64p(X), L.f64p(W))

    def download_paths(self, unit, what):
        C_ = self.d if what == 0 else self.m
        out = np.empty((self.P, C_), dtype=np.float64)
        L.call("dmt_download_paths", self._h, unit, what, L.f64p(out))
        return out

    def XX(self, unit=L.U):
        return self.download_paths(unit, 0)

    # ---------------------------------------------------------------- path snapshots
    def snapshot_reserve(self, n_slots, what_mask=1):
        """HBM ring of n_slots path copies: what_mask 1 = XX, 2 = WW, 3 = both."""
        L.call("dmt_snapshot_reserve", self._h, int(what_mask), int(n_slots))
        self._snap_slots = int(n_slots)

    def snapshot_take(self, slot, mcmciter=0, unit=L.U):
        """deepcopy(unit.XX) (docs/src/tutorials/biblock/smoothing.md:55), on the device."""
        L.call("dmt_snapshot_take", self._h, int(unit), int(slot), int(mcmciter))

    def snapshot_download(self, slot, what=0):
        C_ = self.d if what == 0 else self.m
        out = np.empty((self.P, C_), dtype=np.float64)
        it = C.c_int64()
        L.call("dmt_snapshot_download", self._h, int(what), int(slot), L.f64p(out), C.byref(it))
        return out, it.value

    def snapshot_write(self, path, s0, s1):
        L.call("dmt_snapshot_write", self._h, str(path).encode(), int(s0), int(s1))

    def WW(self, unit=L.U):
        return self.download_paths(unit, 1)

    # ---------------------------------------------------------------- hot path
    def _Z(self, Z):
        if Z is None:
            return None
        Z = np.ascontiguousarray(Z, dtype=np.float64)
        if Z.size != self.S * self.m:
            raise ValueError(f"Z needs {self.S * self.m} values (steps × m), got {Z.size}")
        return Z

    def draw_unit(self, unit, r0=0, r1=None, Z=None, iter=0, salt=0):
        r1 = self.R if r1 is None else r1
        ll = np.empty(r1 - r0, dtype=np.float64)
        ok = np.empty(r1 - r0, dtype=np.uint8)
        Z = self._Z(Z)
        L.call("dmt_draw_unit", self._h, unit, r0, r1, L.f64p(Z), int(iter), int(salt),
               L.f64p(ll), L.u8p(ok))
        return ll, ok.astype(bool)

    def create_layout(self, n_blocks, seg_first, seg_last, last, rho, hist_len=0):
        nb = np.ascontiguousarray(n_blocks, dtype=np.int32)
        sf = np.ascontiguousarray(seg_first, dtype=np.int32)
        sl = np.ascontiguousarray(seg_last, dtype=np.int32)
        lt = np.ascontiguousarray(last, dtype=np.uint8)
        rh = np.ascontiguousarray(rho, dtype=np.float64)
        lid = C.c_int32()
        L.call("dmt_create_layout", self._h, L.i32p(nb), L.i32p(sf), L.i32p(sl), L.u8p(lt),
               L.f64p(rh), int(hist_len), C.byref(lid))
        self._hist_len[lid.value] = int(hist_len)
        return lid.value

    def layout_size(self, layout):
        n = C.c_int64()
        L.call("dmt_layout_size", self._h, layout, C.byref(n))
        return n.value

    def draw_proposal(self, layout, b0, b1, Z=None, iter=0, salt=0, want_success=False):
        """``want_success``: True → the flags (the draw runs now); "lazy" → a LazyFlags that
        reads them (dmt_draw_success) only when used, so the draw may be deferred and fused
        with the accept_reject that follows (include/dmt.h, deferred draws)."""
        eager = want_success is True
        ok = np.empty(b1 - b0, dtype=np.uint8) if eager else None
        Z = self._Z(Z)
        L.call("dmt_draw_proposal", self._h, layout, b0, b1, L.f64p(Z), int(iter), int(salt),
               L.u8p(ok))
        if want_success == "lazy":
            return LazyFlags(self, layout, b0, b1)
        return None if ok is None else ok.astype(bool)

    def draw_success(self, layout, b0, b1):
        """Success flags of the last draw over blocks [b0, b1)."""
        ok = np.empty(b1 - b0, dtype=np.uint8)
        L.call("dmt_draw_success", self._h, layout, b0, b1, L.u8p(ok))
        return ok.astype(bool)

    def accept_reject(self, layout, b0, b1, mcmciter, E=None, salt=0, want_acc=False):
        acc = np.empty(b1 - b0, dtype=np.uint8) if want_acc else None
        if E is not None:
            E = np.ascontiguousarray(E, dtype=np.float64)
            if E.size != b1 - b0:
                raise ValueError("E needs one value per block")
        L.call("dmt_accept_reject", self._h, layout, b0, b1, L.f64p(E), int(mcmciter), int(salt),
               L.u8p(acc))
        return None if acc is None else acc.astype(bool)

    def loglikhd(self, layout, unit, b0, b1):
        L.call("dmt_loglikhd", self._h, layout, unit, b0, b1)

    def recompute_path(self, layout, b0, b1, skip=0, want_success=False):
        ok = np.empty(b1 - b0, dtype=np.uint8) if want_success else None
        L.call("dmt_recompute_path", self._h, layout, b0, b1, int(skip), L.u8p(ok))
        return None if ok is None else ok.astype(bool)

    def find_W_for_X(self, layout, b0, b1):
        """find_W_for_X!: u.WW ← the increments reproducing u.XX under u's laws."""
        L.call("dmt_find_W_for_X", self._h, layout, b0, b1)

    def upload_obs(self, Hobs, Fobs, cobs, artificial_noise=1e-11):
        """Information of the observation at each segment end (packed H, F, c) for the
        device backward filter."""
        Hobs = np.ascontiguousarray(Hobs, dtype=np.float64)
        Fobs = np.ascontiguousarray(Fobs, dtype=np.float64)
        cobs = np.ascontiguousarray(cobs, dtype=np.float64)
        if Hobs.size != self.G * self.hp or Fobs.size != self.G * self.d or cobs.size != self.G:
            raise ValueError("observation information has the wrong size")
        L.call("dmt_upload_obs", self._h, L.f64p(Hobs), L.f64p(Fobs), L.f64p(cobs),
               float(artificial_noise))

    def download_law(self, unit, kind, H_shared=False):
        """(H, F, laws) of a unit's PP / PPb laws in the reference layout."""
        Hn = (self.Q0 if H_shared else self.P) * self.hp
        H = np.empty(Hn)
        F = np.empty(self.P * self.d)
        laws = np.empty(self.G * L.LAW_STRIDE)
        L.call("dmt_download_law", self._h, unit, kind, L.f64p(H), L.f64p(F), L.f64p(laws))
        return H.reshape(-1, self.hp), F.reshape(-1, self.d), laws.reshape(self.G, L.LAW_STRIDE)

    def set_obs(self, layout, b0, b1):
        L.call("dmt_set_obs", self._h, layout, b0, b1)

    def recompute_guiding_term(self, layout, b0, b1, unit=L.U):
        L.call("dmt_recompute_guiding_term", self._h, layout, b0, b1, unit)

    def set_proposal_law(self, layout, b0, b1, params, skip=0, critical_change=None):
        """set_proposal_law!(bb, θ°, pnames, critical_change; skip) on the device: params is
        {name index: value} (DMT_PAR_*); critical_change None: recompute the guiding term where
        the auxiliary law changed, True: everywhere, False: only where equalizing u°'s law with
        u's changed it (dmt_set_proposal_law_cc).  Returns (success[b1-b0], critical[b1-b0])."""
        idx = np.ascontiguousarray(np.fromiter(params.keys(), dtype=np.int32, count=len(params)))
        val = np.ascontiguousarray(np.fromiter(params.values(), dtype=np.float64, count=len(params)))
        ok = np.empty(b1 - b0, dtype=np.uint8)
        crit = np.empty(b1 - b0, dtype=np.uint8)
        cc = -1 if critical_change is None else (1 if critical_change else 0)
        L.call("dmt_set_proposal_law_cc", self._h, layout, b0, b1, len(params),
               idx.ctypes.data_as(C.c_void_p), val.ctypes.data_as(C.c_void_p), int(skip), cc,
               ok.ctypes.data_as(C.c_void_p), crit.ctypes.data_as(C.c_void_p))
        return ok.astype(bool), crit.astype(bool)

    def swap(self, layout, what, b0, b1):
        L.call("dmt_swap", self._h, layout, int(what), b0, b1)

    def save_ll(self, layout, b0, b1, mcmciter):
        L.call("dmt_save_ll", self._h, layout, b0, b1, int(mcmciter))

    def set_accepted(self, layout, b0, b1, mcmciter, v):
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(v, dtype=np.uint8), (b1 - b0,)))
        L.call("dmt_set_accepted", self._h, layout, b0, b1, int(mcmciter), L.u8p(v))

    def get_block_state(self, layout, what, b0, b1, hist_len=None):
        if what in (L.BLK_LL, L.BLK_LLPROP):
            out = np.empty(b1 - b0, dtype=np.float64)
        else:
            have = self._hist_len.get(layout)
            if hist_len is None:
                hist_len = have
            if hist_len is None or (have is not None and hist_len != have):
                raise ValueError(f"layout {layout} holds {have} history rows, not {hist_len}")
            dt = np.uint8 if what == L.BLK_ACC_HIST else np.float64
            out = np.empty((hist_len, b1 - b0), dtype=dt)
        L.call("dmt_get_block_state", self._h, layout, what, b0, b1, out.ctypes.data_as(C.c_void_p))
        return out

    def set_ll(self, layout, unit, b0, b1, mcmciter, values):
        """set_ll!(b, i, v) (src/block.jl:82-86) for blocks [b0, b1) of unit u (bb.b) or u°."""
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(values, dtype=np.float64), (b1 - b0,)))
        L.call("dmt_set_ll", self._h, layout, int(unit), b0, b1, int(mcmciter), L.f64p(v))

    def set_block_state(self, layout, what, b0, b1, values):
        dt = np.uint8 if what == L.BLK_ACC_HIST else np.float64
        v = np.ascontiguousarray(values, dtype=dt)
        L.call("dmt_set_block_state", self._h, layout, what, b0, b1, v.ctypes.data_as(C.c_void_p))

    def fetch_ll(self, layout, b0, b1, mcmciter=0, local=False):
        """(Σ ll, Σ ll°, accepted count of ``mcmciter``) over blocks [b0, b1).  With a
        communicator the sums run over every rank (a collective: BlockEnsemble level) unless
        ``local`` (BiBlock / BlockCollection level: this rank's blocks only)."""
        a, b, n = C.c_double(), C.c_double(), C.c_int64()
        L.call("dmt_fetch_ll_local" if local else "dmt_fetch_ll", self._h, layout, b0, b1,
               int(mcmciter), C.byref(a), C.byref(b), C.byref(n))
        return a.value, b.value, n.value

    def mcmc_step(self, layout, b0, b1, mcmciter, salt=0, local=False):
        """draw_proposal (device RNG) + accept_reject + fetch_ll in one call; ``local``: this
        rank's sums only (BiBlock / BlockCollection level, no collective)."""
        a, b, n = C.c_double(), C.c_double(), C.c_int64()
        L.call("dmt_mcmc_step_local" if local else "dmt_mcmc_step", self._h, layout, b0, b1, int(mcmciter), int(salt), C.byref(a),
               C.byref(b), C.byref(n))
        return a.value, b.value, n.value

    def mcmc_run(self, layout, b0, b1, iter0, n_iter, salt=0, local=False, copy=True):
        """n_iter mcmc_step iterations without host synchronisation in between; returns
        (n_iter, 3): fetch_ll, fetch_ll°, accepted count per iteration (``local``: this rank's
        sums, no collective).  ``copy=False`` returns the handle's result buffer for this run
        length itself (valid until the next run of the same length)."""
        n = int(n_iter)
        buf = self._run_out.get(n)
        if buf is None:
            buf = self.prepare_run(n)
        st = L.fast["dmt_mcmc_run_local" if local else "dmt_mcmc_run"](
            self._h, layout, b0, b1, iter0, n, salt, buf[1])
        if st:
            L.check(st)
        return buf[0].copy() if copy else buf[0]

    def prepare_run(self, n_iter):
        """The result buffer of mcmc_run calls of n_iter iterations (one per run length, its
        address taken once), created ahead of a timed call."""
        n = int(n_iter)
        if n not in self._run_out:
            arr = np.empty((n, 3), dtype=np.float64)
            self._run_out[n] = (arr, arr.ctypes.data)
        return self._run_out[n]

    def set_run_snapshots(self, every, slot0=0):
        """Snapshot u inside every later mcmc_run after each iteration k with k % every == 0
        (slots slot0, slot0 + 1, … of snapshot_reserve, a ring); every = 0: off."""
        L.call("dmt_set_run_snapshots", self._h, int(every), int(slot0))

    # ---------------------------------------------------------------- misc
    def sync(self):
        st = L.fast["dmt_sync"](self._h)
        if st:
            L.check(st)

    def set_service(self, enable=True, idle_ms=2.0):
        """The resident MCMC service's switch and idle window (dmt_set_service); idle_ms = 0
        or enable = False: off — no launch waits on the device between calls."""
        L.call("dmt_set_service", self._h, 1 if enable else 0, float(idle_ms))

    def service_stats(self):
        """(starts, relaunches, posts, waits, off) of the resident service (dmt_service_stats)."""
        st = (C.c_uint64 * 5)()
        L.call("dmt_service_stats", self._h, st)
        return dict(zip(("starts", "relaunches", "posts", "waits", "off"), map(int, st)))

    def set_timing(self, on=True, kernels=None):
        """Event timing of kernel classes ``kernels`` (iterable of K_*; default all)."""
        mask = 0 if not on else (-1 if kernels is None else sum(1 << k for k in kernels))
        L.call("dmt_set_timing", self._h, int(mask))

    def get_timing(self, kernel):
        ms, n = C.c_double(), C.c_int64()
        L.call("dmt_get_timing", self._h, kernel, C.byref(ms), C.byref(n))
        return ms.value, n.value

    def memory_bytes(self):
        n = C.c_int64()
        L.call("dmt_memory_bytes", self._h, C.byref(n))
        return n.value

    def comm_init(self, nranks, rank, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        L.call("dmt_comm_init", self._h, int(nranks), int(rank), buf)

    def comm_size(self):
        """Ranks of the communicator as RCCL reports them (1 without one)."""
        n = C.c_int32()
        L.call("dmt_comm_size", self._h, C.byref(n))
        return n.value

    def rng_counter(self):
        """Next value of the handle's DMT_RNG_AUTO stream counter."""
        n = C.c_uint64()
        L.call("dmt_rng_counter", self._h, C.byref(n))
        return n.value

    def set_rng_counter(self, value):
        L.call("dmt_set_rng_counter", self._h, int(value))

    def rng_state(self):
        """(next counter value, key of the last auto draw, accept pending) — checkpoint."""
        n, last, pend = C.c_uint64(), C.c_uint64(), C.c_uint8()
        L.call("dmt_rng_state", self._h, C.byref(n), C.byref(last), C.byref(pend))
        return n.value, last.value, bool(pend.value)

    def set_rng_state(self, state):
        n, last, pend = state
        L.call("dmt_set_rng_state", self._h, int(n), int(last), 1 if pend else 0)

    def set_shard(self, seg_base):
        """This handle holds a shard whose local segment 0 is global segment ``seg_base``."""
        L.call("dmt_set_shard", self._h, int(seg_base))


class LazyFlags:
    """The success flags a draw returns, read from the device only when used (bool(), indexing,
    iteration, numpy conversion): the draw itself may still be deferred (include/dmt.h)."""

    def __init__(self, ens, layout, b0, b1):
        self._args, self._v = (ens, layout, b0, b1), None

    def _get(self):
        if self._v is None:
            ens, layout, b0, b1 = self._args
            self._v = ens.draw_success(layout, b0, b1)
        return self._v

    def __array__(self, dtype=None, copy=None):
        v = self._get()
        return v if dtype is None else v.astype(dtype)

    def __len__(self):
        return len(self._get())

    def __iter__(self):
        return iter(self._get())

    def __getitem__(self, k):
        return self._get()[k]

    def __bool__(self):
        return bool(self._get().all())

    def all(self):
        return bool(self._get().all())

    def __eq__(self, other):
        return self._get() == other

    def __repr__(self):
        return f"LazyFlags({self._get()!r})"


def comm_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    L.call("dmt_comm_unique_id", buf)
    return bytes(buf)


def combine_rank_partials(all_partials):
    """The host step of the multi-rank fetch_ll / dmt_mcmc_run (dmt_combine_rank_partials):
    ``all_partials[r][i][c]`` = rank r's partial c of iteration i, as the RCCL all-gather leaves
    them; returns ``[n_iter][3]``, the rank-order tree of ``shard.rank_tree`` per entry."""
    a = np.ascontiguousarray(all_partials, dtype=np.float64)
    if a.ndim == 2:
        a = a[:, None, :]
    nranks, n_iter = a.shape[0], a.shape[1]
    out = np.empty((n_iter, 3))
    L.call("dmt_combine_rank_partials", L.f64p(a.reshape(-1)), nranks, n_iter, L.f64p(out))
    return out


def guiding_linear(Bt, beta, at_packed, t, HT_packed, FT, cT):
    """Exact discrete backward filter on one segment (host; dmt_guiding_linear)."""
    d = len(beta)
    hp = d * (d + 1) // 2
    t = np.ascontiguousarray(t, dtype=np.float64)
    n = t.size
    H = np.empty((n, hp))
    F = np.empty((n, d))
    c = np.empty(n)
    L.call("dmt_guiding_linear", d, L.f64p(np.ascontiguousarray(Bt, dtype=np.float64).ravel()),
           L.f64p(np.ascontiguousarray(beta, dtype=np.float64)),
           L.f64p(np.ascontiguousarray(at_packed, dtype=np.float64)), n, L.f64p(t),
           L.f64p(np.ascontiguousarray(HT_packed, dtype=np.float64)),
           L.f64p(np.ascontiguousarray(FT, dtype=np.float64)), float(cT), L.f64p(H), L.f64p(F),
           L.f64p(c))
    return H, F, c


def guiding_linear_td(aux, at_packed, t, HT_packed, FT, cT):
    """The host filter of a time-dependent auxiliary drift (dmt_guiding_linear_td):
    aux[npts][d·d + d] = B̃(t_i), β̃(t_i), step i taking its left point's row."""
    t = np.ascontiguousarray(t, dtype=np.float64)
    n = t.size
    aux = np.ascontiguousarray(aux, dtype=np.float64).reshape(n, -1)
    d = {2: 1, 6: 2, 12: 3}[aux.shape[1]]
    hp = d * (d + 1) // 2
    H = np.empty((n, hp))
    F = np.empty((n, d))
    c = np.empty(n)
    L.call("dmt_guiding_linear_td", d, L.f64p(aux),
           L.f64p(np.ascontiguousarray(at_packed, dtype=np.float64)), n, L.f64p(t),
           L.f64p(np.ascontiguousarray(HT_packed, dtype=np.float64)),
           L.f64p(np.ascontiguousarray(FT, dtype=np.float64)), float(cT), L.f64p(H), L.f64p(F),
           L.f64p(c))
    return H, F, c


def guiding_linear_tda(aux, t, HT_packed, FT, cT):
    """The host filter of a time-dependent auxiliary law with time-dependent ã too
    (dmt_guiding_linear_tda): aux[npts][d·d + d + d(d+1)/2] = B̃, β̃, ã packed."""
    t = np.ascontiguousarray(t, dtype=np.float64)
    n = t.size
    aux = np.ascontiguousarray(aux, dtype=np.float64).reshape(n, -1)
    d = {3: 1, 9: 2, 18: 3}[aux.shape[1]]
    hp = d * (d + 1) // 2
    H = np.empty((n, hp))
    F = np.empty((n, d))
    c = np.empty(n)
    L.call("dmt_guiding_linear_tda", d, L.f64p(aux), n, L.f64p(t),
           L.f64p(np.ascontiguousarray(HT_packed, dtype=np.float64)),
           L.f64p(np.ascontiguousarray(FT, dtype=np.float64)), float(cT), L.f64p(H), L.f64p(F),
           L.f64p(c))
    return H, F, c


def debug_philox(seed, ctr, device=0):
    ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
    out = np.empty_like(ctr)
    L.call("dmt_debug_philox", device, int(seed), L.u32p(ctr), ctr.shape[0], L.u32p(out))
    return out


def debug_normals(seed, ctr, device=0):
    ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
    out = np.empty((ctr.shape[0], 2), dtype=np.float64)
    L.call("dmt_debug_normals", device, int(seed), L.u32p(ctr), ctr.shape[0], L.f64p(out))
    return out


# ---------------------------------------------------------------- snapshot files
SNAPSHOT_HEADER = np.dtype([("magic", "S8"), ("version", "<u4"), ("what_mask", "<u4"),
                            ("d", "<i4"), ("m", "<i4"), ("grid_shared", "<i4"),
                            ("precision", "<i4"), ("n_recordings", "<i8"), ("n_segments", "<i8"),
                            ("n_points", "<i8"), ("n_t", "<i8"), ("n_slots", "<i8"),
                            ("seg_base", "<i8")])


def read_snapshots(path, mmap=True):
    """Reads a dmt_snapshot_write file (layout: include/dmt.h, dmt_snapshot_header).  Returns a
    dict: header fields, ``n_points`` (per recording, per segment), ``t``, ``mcmciter`` and
    ``unit`` per slot, ``X`` [slots][P][d] and/or ``W`` [slots][P][m] (memory-mapped), and
    ``paths(slot, r)`` = recording r's XX as a list of per-segment [npts][d] arrays (the
    reference's ``Vector{Trajectory}``)."""
    hd = np.fromfile(path, dtype=SNAPSHOT_HEADER, count=1)[0]
    if hd["magic"] != b"DMTPATH1" or hd["version"] != 1:
        raise ValueError(f"{path}: not a DMTPATH1 snapshot file")
    R, G, P, nt, ns = (int(hd[k]) for k in ("n_recordings", "n_segments", "n_points", "n_t", "n_slots"))
    d, m, mask = int(hd["d"]), int(hd["m"]), int(hd["what_mask"])
    off = SNAPSHOT_HEADER.itemsize
    nseg = np.fromfile(path, dtype="<i4", count=R, offset=off); off += 4 * R
    npts = np.fromfile(path, dtype="<i4", count=G, offset=off); off += 4 * G
    t = np.fromfile(path, dtype="<f8", count=nt, offset=off); off += 8 * nt
    per = (P * d if mask & 1 else 0) + (P * m if mask & 2 else 0)
    rec = np.dtype([("mcmciter", "<i8"), ("unit", "<i8"), ("paths", "<f8", (per,))])
    slots = (np.memmap(path, dtype=rec, mode="r", offset=off, shape=(ns,)) if mmap and ns
             else np.fromfile(path, dtype=rec, count=ns, offset=off))
    out = {k: hd[k].item() for k in SNAPSHOT_HEADER.names if k != "magic"}
    seg0 = np.concatenate([[0], np.cumsum(nseg)])
    out["n_points"] = [npts[seg0[r]:seg0[r + 1]].tolist() for r in range(R)]
    out["t"] = t
    out["mcmciter"] = np.asarray(slots["mcmciter"])
    out["unit"] = np.asarray(slots["unit"])
    body = slots["paths"]
    if mask & 1:
        out["X"] = body[:, : P * d].reshape(ns, P, d)
    if mask & 2:
        o = P * d if mask & 1 else 0
        out["W"] = body[:, o: o + P * m].reshape(ns, P, m)
    pt0 = np.concatenate([[0], np.cumsum(npts)])

    def paths(slot, r, what="X"):
        A = out[what][slot]
        return [A[pt0[g]:pt0[g + 1]] for g in range(seg0[r], seg0[r + 1])]
    out["paths"] = paths
    return out

