"""Oracle for the guided-bridge hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and the cpu_baseline leg of bench.py import this
module; the product (libdmt, diffusionmcmctools.jl_amd) never does.

Two parts:
  * a ctypes binding of liboracle.so (oracle/dmt_oracle.c): the per-segment numerical
    restatement (canonical arithmetic, see the C file header);
  * ``OracleEnsemble``: a pure-Python restatement of the reference's CONTAINER semantics,
    following the Julia sources line by line: SamplingPair u/u° with per-segment
    containers (src/sampling_pair.jl:36-55), Block views (src/block.jl:49-79), BiBlock
    imputation/accept/swaps/histories (src/biblock.jl:78-259), BlockCollection /
    BlockEnsemble broadcasting (src/block_collection.jl, src/block_ensemble.jl).
    Swaps exchange Python object references between u and u°, exactly as the Julia
    code swaps container references.

Parity status: "parity unpinned" against the reference itself (no Julia, upstream
GuidedProposals/DiffusionDefinition not vendored, empty reference tests); pinned by
the analytic known-answer tests in tests/test_oracle_kat.py and the independent
numpy restatement in oracle/np_oracle.py.  See DESIGN.md §4.
"""
from __future__ import annotations

import copy
import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("DMT_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")  # measurement variants

LAW_STRIDE = 64
L_C0 = 49
L_BT, L_TRACE, L_A, L_SIGMA, L_ANCHOR, L_AUXLIN = 31, 50, 25, 16, 60, 63
L_AUXTD = 15   # time-dependent auxiliary law flag (include/dmt.h DMT_LAW_AUXTD)
L_GSTALE = 14  # u°'s guiding term left stale by critical_change = false (DMT_LAW_GSTALE)
MODEL_OU = 0


def set_law_params(model, d, rec, params):
    """DD.set_parameters! on one law record + the fields derived from θ (FHN: σ, a and — for an
    auxiliary law linearised at its anchor — B̃, β̃, a − ã = 0; Lorenz: B̃, β̃; OU: Θ, μ only).
    Plain Python float arithmetic (IEEE double, no contraction) in the order the device's
    k_set_prop_law uses; restates DESIGN.md §3's set_proposal_law! derivation.  In place."""
    for p, v in params.items():
        v = float(v)
        if model == 1:  # FHN (eps, s, gamma, beta, sigma)
            if p == 0:
                rec[4], rec[0] = v, 1.0 / v
            elif p == 4:
                rec[5] = v
            else:
                rec[p] = v
        elif model == 2:  # Lorenz (s, r, beta)
            rec[p] = v
        else:  # OU: Theta (row-major), mu
            rec[p if p < d * d else 9 + (p - d * d)] = v
    if model == 1:
        sg = float(rec[5])
        rec[L_SIGMA], rec[L_SIGMA + 1] = 0.0, sg
        rec[L_A], rec[L_A + 1], rec[L_A + 2] = 0.0 * 0.0, 0.0 * sg, sg * sg
        if rec[L_AUXLIN] != 0.0:
            e, y = float(rec[4]), float(rec[L_ANCHOR])
            yy = y * y
            rec[L_BT:L_BT + 4] = [(1.0 - 3.0 * yy) / e, -1.0 / e, float(rec[2]), -1.0]
            rec[40:42] = [(float(rec[1]) + 2.0 * (yy * y)) / e, float(rec[3])]
            rec[43:46] = 0.0
            rec[L_TRACE] = 0.0
    elif model == 2 and rec[L_AUXLIN] != 0.0:
        s_, r_, b_ = (float(rec[i]) for i in range(3))
        x0, x1, x2 = (float(rec[L_ANCHOR + i]) for i in range(3))
        J = [-s_, s_, 0.0, r_ - x2, -1.0, -x0, x1, x0, -b_]
        f = [s_ * (x1 - x0), x0 * (r_ - x2) - x1, x0 * x1 - b_ * x2]
        rec[L_BT:L_BT + 9] = J
        rec[40:43] = [f[i] - ((J[3 * i] * x0 + J[3 * i + 1] * x1) + J[3 * i + 2] * x2)
                      for i in range(3)]


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def _load():
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    d_, i_, i64, u32, u64 = C.c_double, C.c_int, C.c_int64, C.c_uint32, C.c_uint64
    P = C.c_void_p
    for sfx, R in (("f64", C.c_double), ("f32", C.c_float)):
        f = getattr(lib, f"orc_solve_segment_{sfx}")
        f.argtypes = [i_, i_, i_, P, i_, P, P, P, P, P, P, P]
        f.restype = i_
        f = getattr(lib, f"orc_invsolve_segment_{sfx}")
        f.argtypes = [i_, i_, i_, P, i_, P, P, P, P, P]
        f.restype = None
        f = getattr(lib, f"orc_path_ll_segment_{sfx}")
        f.argtypes = [i_, i_, i_, P, i_, P, P, P, P]
        f.restype = R
        f = getattr(lib, f"orc_obs_term_{sfx}")
        f.argtypes = [i_, P, P, P, P]
        f.restype = R
        f = getattr(lib, f"orc_pcn_segment_{sfx}")
        f.argtypes = [i_, i_, P, P, P, R, R, P]
        f.restype = None
        for nm in ("orc_w_to_increments", "orc_w_from_increments"):
            f = getattr(lib, f"{nm}_{sfx}")
            f.argtypes = [i_, i_, P, P]
            f.restype = None
        f = getattr(lib, f"orc_normals_segment_{sfx}")
        f.argtypes = [u64, u32, u32, u32, i_, i_, P]
        f.restype = None
        f = getattr(lib, f"orc_draw_terminal_blocks_{sfx}")
        f.argtypes = [i_, i_, i_, i64, i_, P, i64, P, i64, P, i64, P, i64, P, P, P, u64, i64,
                      u32, P, P, P, P, i_]
        f.restype = i_
    lib.orc_normal_pair_f64.argtypes = [u64, u32, u32, u32, u32, P, P]
    lib.orc_normal_pair_f64.restype = None
    lib.orc_exp1.argtypes = [u64, u32, u32, u32]
    lib.orc_exp1.restype = d_
    lib.orc_exp1_range.argtypes = [u64, u32, C.c_int64, u32, u32, C.c_void_p]
    lib.orc_exp1_range.restype = None
    lib.orc_set_sequential_ou.argtypes = [i_]
    lib.orc_set_sequential_ou.restype = None
    lib.orc_set_ll_skip.argtypes = [i_]
    lib.orc_set_ll_skip.restype = None
    lib.orc_backward_filter_segment.argtypes = [i_, P, P, P, i_, P, P, P, d_, P, P, P]
    lib.orc_backward_filter_segment.restype = i_
    lib.orc_backward_filter_segment_td.argtypes = [i_, P, P, i_, P, P, P, d_, P, P, P]
    lib.orc_backward_filter_segment_td.restype = i_
    lib.orc_backward_filter_segment_tda.argtypes = [i_, P, i_, P, P, P, d_, P, P, P]
    lib.orc_backward_filter_segment_tda.restype = i_
    lib.orc_set_aux.argtypes = [P]
    lib.orc_set_aux.restype = None
    lib.orc_rng_log.argtypes = [d_]
    lib.orc_rng_log.restype = d_
    lib.orc_bm_log.argtypes = [d_]
    lib.orc_bm_log.restype = d_
    lib.orc_philox_raw.argtypes = [u64, P, P]
    lib.orc_philox_raw.restype = None
    return lib


lib = _load()


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _dt(prec):
    return np.float64 if prec == 0 else np.float32


def _sfx(prec):
    return "f64" if prec == 0 else "f32"


# ------------------------------------------------------------------ per-segment numerics
class _aux_rows:
    """The segment's time-dependent auxiliary coefficients (rows [npts][d·d + d + d(d+1)/2] =
    B̃, β̃, ã packed, doubles) for the C calls inside the block (orc_set_aux), or nothing."""

    def __init__(self, aux):
        self.aux = None if aux is None else np.ascontiguousarray(aux, dtype=np.float64)

    def __enter__(self):
        if self.aux is not None:
            lib.orc_set_aux(_p(self.aux))

    def __exit__(self, *exc):
        if self.aux is not None:
            lib.orc_set_aux(None)


def solve_segment(model, d, m, law, t, H, F, W, y1, prec=0, aux=None):
    dt = _dt(prec)
    t, H, F, W = (np.ascontiguousarray(a, dtype=dt) for a in (t, H, F, W))
    y1 = np.ascontiguousarray(y1, dtype=dt)
    law = np.ascontiguousarray(law, dtype=np.float64)
    n = t.size
    X = np.empty((n, d), dtype=dt)
    ll = np.zeros(1, dtype=dt)
    with _aux_rows(aux):
        ok = getattr(lib, f"orc_solve_segment_{_sfx(prec)}")(model, d, m, _p(law), n, _p(t), _p(H),
                                                              _p(F), _p(W), _p(y1), _p(X), _p(ll))
    return X, dt(ll[0]), bool(ok)


LOG2PI = float.fromhex("0x1.d67f1c864beb4p+0")


def backward_filter_segment(d, Bt, beta, at_packed, t, HT_packed, FT, cT):
    """Exact discrete backward filter of a linear auxiliary law over one grid (double):
    returns H (npts × hp packed), F (npts × d), c (npts)."""
    t = np.ascontiguousarray(t, dtype=np.float64)
    n = t.size
    hp = d * (d + 1) // 2
    H = np.empty((n, hp)); F = np.empty((n, d)); c = np.empty(n)
    args = [np.ascontiguousarray(a, dtype=np.float64) for a in (Bt, beta, at_packed, HT_packed, FT)]
    ok = lib.orc_backward_filter_segment(d, _p(args[0]), _p(args[1]), _p(args[2]), n, _p(t),
                                         _p(args[3]), _p(args[4]), float(cT), _p(H), _p(F), _p(c))
    if not ok:
        raise FloatingPointError("singular I + HK in the backward filter")
    return H, F, c


def backward_filter_segment_td(d, aux, at_packed, t, HT_packed, FT, cT):
    """The same filter for a time-dependent auxiliary drift: aux[npts][d·d + d] = B̃(t_i), β̃(t_i),
    step i taking its left point's row (dmt_guiding_linear_td, dmt_upload_aux)."""
    t = np.ascontiguousarray(t, dtype=np.float64)
    n = t.size
    hp = d * (d + 1) // 2
    H = np.empty((n, hp)); F = np.empty((n, d)); c = np.empty(n)
    args = [np.ascontiguousarray(a, dtype=np.float64) for a in (aux, at_packed, HT_packed, FT)]
    assert args[0].shape == (n, d * d + d)
    ok = lib.orc_backward_filter_segment_td(d, _p(args[0]), _p(args[1]), n, _p(t), _p(args[2]),
                                            _p(args[3]), float(cT), _p(H), _p(F), _p(c))
    if not ok:
        raise FloatingPointError("singular I + HK in the backward filter")
    return H, F, c


def backward_filter_segment_tda(d, aux, t, HT_packed, FT, cT):
    """The filter with a time-dependent ã too: aux[npts][d·d + d + d(d+1)/2] = B̃, β̃, ã packed,
    step i taking the trapezoidal averages of rows i and i + 1 (dmt_guiding_linear_tda)."""
    t = np.ascontiguousarray(t, dtype=np.float64)
    n = t.size
    hp = d * (d + 1) // 2
    H = np.empty((n, hp)); F = np.empty((n, d)); c = np.empty(n)
    args = [np.ascontiguousarray(a, dtype=np.float64) for a in (aux, HT_packed, FT)]
    assert args[0].shape == (n, d * d + d + hp)
    ok = lib.orc_backward_filter_segment_tda(d, _p(args[0]), n, _p(t), _p(args[1]), _p(args[2]),
                                             float(cT), _p(H), _p(F), _p(c))
    if not ok:
        raise FloatingPointError("singular I + HK in the backward filter")
    return H, F, c


def invsolve_segment(model, d, m, law, t, H, F, X, prec=0):
    """DD.invsolve!: Wiener increments (row 0 = W(t0) = 0) reproducing X under the law."""
    dt = _dt(prec)
    t, H, F, X = (np.ascontiguousarray(a, dtype=dt) for a in (t, H, F, X))
    law = np.ascontiguousarray(law, dtype=np.float64)
    W = np.empty((t.size, m), dtype=dt)
    getattr(lib, f"orc_invsolve_segment_{_sfx(prec)}")(model, d, m, _p(law), t.size, _p(t), _p(H),
                                                      _p(F), _p(X), _p(W))
    return W


def path_ll_segment(model, d, m, law, t, H, F, X, prec=0, aux=None):
    dt = _dt(prec)
    t, H, F, X = (np.ascontiguousarray(a, dtype=dt) for a in (t, H, F, X))
    law = np.ascontiguousarray(law, dtype=np.float64)
    with _aux_rows(aux):
        return dt(getattr(lib, f"orc_path_ll_segment_{_sfx(prec)}")(model, d, m, _p(law), t.size,
                                                                     _p(t), _p(H), _p(F), _p(X)))


def obs_term(d, law, H0, F0, x, prec=0):
    dt = _dt(prec)
    H0, F0, x = (np.ascontiguousarray(a, dtype=dt) for a in (H0, F0, x))
    law = np.ascontiguousarray(law, dtype=np.float64)
    return dt(getattr(lib, f"orc_obs_term_{_sfx(prec)}")(d, _p(law), _p(H0), _p(F0), _p(x)))


def pcn_segment(m, t, W, Z, rho, srho, prec=0):
    dt = _dt(prec)
    t, W, Z = (np.ascontiguousarray(a, dtype=dt) for a in (t, W, Z))
    Wo = np.empty((t.size, m), dtype=dt)
    getattr(lib, f"orc_pcn_segment_{_sfx(prec)}")(m, t.size, _p(t), _p(W), _p(Z), rho, srho,
                                                  _p(Wo))
    return Wo


def w_to_increments(W, prec=0):
    """Cumulative Wiener path (npts × m) -> row 0 = W(t0), row i+1 = increment i."""
    dt = _dt(prec)
    W = np.ascontiguousarray(W, dtype=dt)
    out = np.empty_like(W)
    getattr(lib, f"orc_w_to_increments_{_sfx(prec)}")(W.shape[1], W.shape[0], _p(W), _p(out))
    return out


def w_from_increments(dW, prec=0):
    dt = _dt(prec)
    dW = np.ascontiguousarray(dW, dtype=dt)
    out = np.empty_like(dW)
    getattr(lib, f"orc_w_from_increments_{_sfx(prec)}")(dW.shape[1], dW.shape[0], _p(dW), _p(out))
    return out


def normals_segment(seed, g, it, salt, nsteps, m, prec=0):
    Z = np.empty(nsteps * m, dtype=_dt(prec))
    getattr(lib, f"orc_normals_segment_{_sfx(prec)}")(seed, g, it & 0xFFFFFFFF, salt, nsteps, m,
                                                      _p(Z))
    return Z.reshape(nsteps, m)


def normal_pair(seed, ctr):
    """Box–Muller pair of one Philox block (fp64), counter ctr = (c0, c1, c2, c3)."""
    z0, z1 = C.c_double(), C.c_double()
    lib.orc_normal_pair_f64(seed, *[int(v) for v in ctr], C.byref(z0), C.byref(z1))
    return z0.value, z1.value


def exp1(seed, blk, it, salt):
    return lib.orc_exp1(seed, blk, it & 0xFFFFFFFF, salt)


def exp1_range(seed, g0, n, it, salt):
    """exp1 of the blocks whose first segments are g0 … g0 + n - 1."""
    out = np.empty(int(n))
    lib.orc_exp1_range(C.c_uint64(seed), C.c_uint32(g0), C.c_int64(n), C.c_uint32(it & 0xFFFFFFFF),
                       C.c_uint32(salt), _p(out))
    return out


def philox_raw(seed, ctr):
    ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
    out = np.empty_like(ctr)
    for i in range(ctr.shape[0]):
        lib.orc_philox_raw(seed, _p(ctr[i]), _p(out[i]))
    return out


def unpacked(hp_vec, d):
    """Packed upper triangle (row-major) -> full symmetric d×d."""
    M = np.empty((d, d))
    k = 0
    for a in range(d):
        for b in range(a, d):
            M[a, b] = M[b, a] = hp_vec[k]
            k += 1
    return M


def packed_sym(M):
    d = M.shape[0]
    return np.array([M[a, b] for a in range(d) for b in range(a, d)])


def pairwise_tree(vals):
    """Complete adjacent-pair binary tree over vals padded with zeros to a power of two,
    canonicalised with + 0.0 (fetch_ll reduction order)."""
    v = [float(x) for x in vals]
    n2 = 1
    while n2 < len(v):
        n2 *= 2
    v = v + [0.0] * (n2 - len(v))
    while len(v) > 1:
        v = [v[2 * j] + v[2 * j + 1] for j in range(len(v) // 2)]
    return (v[0] if v else 0.0) + 0.0


def draw_terminal_blocks(model, d, m, npts, laws, t, H, F, Xacc, Wacc, rho, Z=None, seed=0,
                         it=0, salt=0, prec=0, nthreads=1, t_shared=True, H_shared=False,
                         sequential=False):
    """Whole-ensemble draw for single-segment terminal blocks, OpenMP over blocks
    (the timed CPU baseline).  Arrays in reference layout.  sequential=True: linear-drift
    segments by the plain Euler loop (the CPU algorithm), not the canonical scan."""
    lib.orc_set_sequential_ou(1 if sequential else 0)
    dt = _dt(prec)
    B = laws.shape[0]
    t = np.ascontiguousarray(t, dtype=dt)
    H = np.ascontiguousarray(H, dtype=dt)
    F = np.ascontiguousarray(F, dtype=dt)
    Xacc = np.ascontiguousarray(Xacc, dtype=dt)
    Wacc = np.ascontiguousarray(Wacc, dtype=dt)
    laws = np.ascontiguousarray(laws, dtype=np.float64)
    rho = np.ascontiguousarray(rho, dtype=np.float64)
    Zp = None if Z is None else np.ascontiguousarray(Z, dtype=dt)
    hp = d * (d + 1) // 2
    Xo = np.empty((B * npts, d), dtype=dt)
    Wo = np.empty((B * npts, m), dtype=dt)
    ll = np.empty(B)
    nfail = getattr(lib, f"orc_draw_terminal_blocks_{_sfx(prec)}")(
        model, d, m, B, npts, _p(laws), LAW_STRIDE, _p(t), 0 if t_shared else npts, _p(H),
        0 if H_shared else npts * hp, _p(F), npts * d, _p(Xacc), _p(Wacc),
        None if Zp is None else _p(Zp), seed, it, salt, _p(rho), _p(Xo), _p(Wo), _p(ll), nthreads)
    lib.orc_set_sequential_ou(0)
    return Xo, Wo, ll, nfail


# ------------------------------------------------------------------ container semantics
class _Law:
    __slots__ = ("H", "F", "rec")

    def __init__(self, H, F, rec):
        self.H, self.F, self.rec = H, F, rec


class _Unit:
    """SamplingUnit containers (src/sampling_unit.jl:48-53): PP, PPb, WW, XX per segment."""

    def __init__(self):
        self.PP, self.PPb, self.WW, self.XX = [], [], [], []


class _Block:
    def __init__(self, rec, g0, g1, term, rho, hist_len):
        self.rec, self.g0, self.g1, self.term = rec, g0, g1, bool(term)
        self.rho = float(rho)
        self.srho = math.sqrt(1.0 - self.rho * self.rho)
        self.ll = -math.inf   # src/block.jl:75
        self.llp = -math.inf
        self.ll_hist = np.zeros(hist_len)
        self.llp_hist = np.zeros(hist_len)
        self.acc_hist = np.zeros(hist_len, dtype=bool)


# Device random stream keys (include/dmt.h, "device random streams"): salt = RNG_AUTO takes the
# handle's stream counter k instead of the caller's (iter, salt), mapped to
# (k mod 2^32, SALT_LIMIT + k div 2^32).
RNG_AUTO = 0xFFFFFFFF
SALT_LIMIT = 0x40000000


def auto_key(k):
    return k & 0xFFFFFFFF, SALT_LIMIT + ((k >> 32) & (SALT_LIMIT - 1))


class OracleEnsemble:
    """Restatement of SamplingEnsemble + BlockEnsemble semantics on reference-layout data.
    Mirrors the libdmt call surface (diffusionmcmctools.jl_amd/engine.py) so tests can drive
    both with the same calls."""

    def __init__(self, model, d, m, n_points, prec=0, seed=0, grid_shared=False):
        self.model, self.d, self.m, self.prec, self.seed = model, d, m, prec, seed
        self.hp = d * (d + 1) // 2
        self.dt = _dt(prec)
        self.nseg = [len(r) for r in n_points]
        self.npts = [int(n) for r in n_points for n in r]
        self.R, self.G = len(self.nseg), len(self.npts)
        self.rec_seg0 = np.concatenate([[0], np.cumsum(self.nseg)]).astype(np.int64)
        self.pt_off = np.concatenate([[0], np.cumsum(self.npts)[:-1]]).astype(np.int64)
        self.st_off = self.pt_off - np.arange(self.G)
        self.P = int(sum(self.npts))
        self.S = self.P - self.G
        self.grid_shared = grid_shared
        self.Q0 = int(sum(self.npts[: self.nseg[0]]))
        self.t = [None] * self.G
        self.u, self.up = _Unit(), _Unit()
        for U_ in (self.u, self.up):
            for g in range(self.G):
                U_.XX.append(np.zeros((self.npts[g], d), dtype=self.dt))
                U_.WW.append(np.zeros((self.npts[g], m), dtype=self.dt))
            U_.PP = [None] * self.G
            U_.PPb = [None] * self.G
        self.layouts = []
        self.aux = [None, None]  # [kind] time-dependent auxiliary coefficients (upload_aux)
        self.seg_base = 0  # dmt_set_shard
        # RNG_AUTO counter: next key, the key of the last auto draw, armed for one auto accept
        self.rng_ctr, self.rng_last, self.rng_pending = 0, 0, False
        # internal layout 0: whole recordings, terminal, rho 0 (draw_proposal_path!(u))
        self.create_layout([1] * self.R, [0] * self.R, [n - 1 for n in self.nseg], [1] * self.R,
                           [0.0] * self.R, 0)

    def _seg_rows(self, arr, g, C_):
        a = np.asarray(arr, dtype=np.float64).reshape(-1, C_)
        return a[self.pt_off[g]: self.pt_off[g] + self.npts[g]].astype(self.dt)

    def _unit(self, unit):
        return self.u if unit == 0 else self.up

    # ---- uploads
    def upload_grid(self, t):
        t = np.asarray(t, dtype=np.float64)
        for g in range(self.G):
            if self.grid_shared:
                k = g - self.rec_seg0[np.searchsorted(self.rec_seg0, g, side="right") - 1]
                off = int(sum(self.npts[:k]))
                self.t[g] = t[off: off + self.npts[g]].astype(self.dt)
            else:
                self.t[g] = self._seg_rows(t, g, 1).ravel()

    def upload_law(self, unit, kind, H=None, F=None, laws=None, H_shared=False):
        me = self._unit(unit)
        other = self._unit(1 - unit)
        tab = me.PP if kind == 0 else me.PPb
        otab = other.PP if kind == 0 else other.PPb
        first = tab[0] is None
        for g in range(self.G):
            if tab[g] is None:
                tab[g] = _Law(None, None, None)
            lw = tab[g]
            if H is not None:
                if H_shared:
                    k = g - self.rec_seg0[np.searchsorted(self.rec_seg0, g, side="right") - 1]
                    off = int(sum(self.npts[self.rec_seg0[0]: self.rec_seg0[0] + k]))
                    Hs = np.asarray(H, dtype=np.float64).reshape(-1, self.hp)
                    lw.H = Hs[off: off + self.npts[g]].astype(self.dt)
                else:
                    lw.H = self._seg_rows(H, g, self.hp)
            if F is not None:
                lw.F = self._seg_rows(F, g, self.d)
            if laws is not None:
                lw.rec = np.asarray(laws, dtype=np.float64).reshape(self.G, LAW_STRIDE)[g].copy()
        if first:  # u° = deepcopy(u) (src/sampling_pair.jl:51)
            for g in range(self.G):
                otab[g] = copy.deepcopy(tab[g])

    def upload_aux(self, kind, aux):
        """dmt_upload_aux(_a): per-point B̃(t_i), β̃(t_i) ([P][d·d + d]) — or B̃, β̃, ã(t_i) packed
        ([P][d·d + d + d(d+1)/2]) — of the laws of `kind`, u and u° alike, held in the working
        precision (as the device holds them; ã zero where not given) for the segments whose
        record has auxtd set (2: ã from the table too); None removes them.  A linear drift (OU)
        takes them in G only (its recursion is the target law's)."""
        if aux is None:
            self.aux[kind] = None
            return
        nb = self.d * self.d + self.d
        na = nb + self.d * (self.d + 1) // 2
        a = np.asarray(aux, dtype=np.float64).reshape(self.P, -1)
        if a.shape[1] not in (nb, na):
            raise ValueError("aux needs d·d + d or d·d + d + d(d+1)/2 columns")
        full = np.zeros((self.P, na))
        full[:, :a.shape[1]] = a
        self.aux[kind] = full.astype(self.dt).astype(np.float64)

    def _aux_seg(self, bk, g):
        """The segment's rows of its law kind's table when its record is time-dependent."""
        kind = 1 if (not bk.term and g == bk.g1) else 0
        tab = self.aux[kind]
        lw = self._law(0, bk, g)
        if tab is None or lw.rec is None or lw.rec[L_AUXTD] == 0.0:
            return None
        return tab[self.pt_off[g]: self.pt_off[g] + self.npts[g]]

    def set_paths(self, unit, X=None, W=None):
        """Host W is cumulative (the reference's Wiener trajectories); held as increments."""
        me = self._unit(unit)
        for g in range(self.G):
            if X is not None:
                me.XX[g][...] = self._seg_rows(X, g, self.d)
            if W is not None:
                me.WW[g][...] = w_to_increments(self._seg_rows(W, g, self.m), self.prec)

    def download_paths(self, unit, what):
        me = self._unit(unit)
        if what == 0:
            return np.concatenate(me.XX).astype(np.float64)
        if what == 2:  # DMT_PATH_DW: the increments as held
            return np.concatenate(me.WW).astype(np.float64)
        return np.concatenate([w_from_increments(w, self.prec) for w in me.WW]).astype(np.float64)

    # ---- layouts (BlockEnsemble ranges)
    def create_layout(self, n_blocks, seg_first, seg_last, last, rho, hist_len=0):
        blocks, b = [], 0
        for r in range(self.R):
            for _ in range(n_blocks[r]):
                g0 = int(self.rec_seg0[r] + seg_first[b])
                g1 = int(self.rec_seg0[r] + seg_last[b])
                blocks.append(_Block(r, g0, g1, last[b], rho[b], hist_len))
                b += 1
        self.layouts.append(blocks)
        return len(self.layouts) - 1

    # ---- stream keys: the reference's draws take no key (global RNG, src/biblock.jl:94-99,122);
    # RNG_AUTO restates that with a per-handle counter, exactly as libdmt's draw_key/accept_key
    def _draw_key(self, it, salt, arm):
        if salt != RNG_AUTO:
            if salt >= SALT_LIMIT:
                raise ValueError("salt must be < SALT_LIMIT")
            return it, salt
        k = self.rng_ctr
        self.rng_ctr += 1
        self.rng_last, self.rng_pending = k, arm
        return auto_key(k)

    def _accept_key(self, mcmciter, salt):
        if salt != RNG_AUTO:
            if salt >= SALT_LIMIT:
                raise ValueError("salt must be < SALT_LIMIT")
            return mcmciter, salt
        if self.rng_pending:
            k = self.rng_last
        else:
            k = self.rng_ctr
            self.rng_ctr += 1
        self.rng_pending = False
        return auto_key(k)

    def rng_counter(self):
        return self.rng_ctr

    def set_rng_counter(self, v):
        self.rng_ctr, self.rng_pending = int(v), False

    def rng_state(self):
        return self.rng_ctr, self.rng_last, self.rng_pending

    def set_rng_state(self, st):
        self.rng_ctr, self.rng_last, self.rng_pending = int(st[0]), int(st[1]), bool(st[2])

    # ---- the hot path, restated
    def _Zseg(self, Z, g, it, salt):
        n = self.npts[g] - 1
        if Z is not None:
            Zf = np.asarray(Z, dtype=np.float64).reshape(-1, self.m)
            return Zf[self.st_off[g]: self.st_off[g] + n].astype(self.dt)
        return normals_segment(self.seed, g + self.seg_base, it, salt, n, self.m, self.prec)

    def _law(self, unit, bk, g):
        me = self._unit(unit)
        return me.PPb[g] if (not bk.term and g == bk.g1) else me.PP[g]

    def _solve_block(self, bk, law_unit, start_unit, w_unit, out_unit, mode, Z, it, salt):
        """mode: 'pcn' (rand! with ρ), 'given' (solve_and_ll! with W), 'fresh' (ρ = 0)."""
        dt = self.dt
        src = self._unit(start_unit)
        y1 = src.XX[bk.g0][0].copy()
        law0 = self._unit(law_unit).PP[bk.g0]
        ll = obs_term(self.d, law0.rec, law0.H[0], law0.F[0], y1, self.prec)
        x = y1
        ok_all = True
        out = self._unit(out_unit)
        win = self._unit(w_unit)
        for g in range(bk.g0, bk.g1 + 1):
            lw = self._law(law_unit, bk, g)
            t = self.t[g]
            if mode == "given":
                Wuse = win.WW[g]
            else:
                Zg = self._Zseg(Z, g, it, salt)
                if mode == "fresh":
                    Wuse = pcn_segment(self.m, t, np.zeros_like(win.WW[g]), Zg, dt(0.0), dt(1.0),
                                       self.prec)
                else:
                    Wuse = pcn_segment(self.m, t, win.WW[g], Zg, dt(bk.rho), dt(bk.srho),
                                       self.prec)
                out.WW[g][...] = Wuse
            aux = self._aux_seg(bk, g) if lw.rec[L_AUXTD] != 0.0 else None
            X, sl, ok = solve_segment(self.model, self.d, self.m, lw.rec, t, lw.H, lw.F, Wuse, x,
                                      self.prec, aux=aux)
            out.XX[g][...] = X
            if not ok:
                ok_all = False
                break
            ll = dt(ll + sl)
            x = X[-1].copy()
        return (float(ll) if ok_all else -math.inf), ok_all

    def draw_unit(self, unit, r0=0, r1=None, Z=None, iter=0, salt=0):
        """draw_proposal_path!(u::SamplingUnit), src/sampling_unit.jl:118-120."""
        r1 = self.R if r1 is None else r1
        iter, salt = self._draw_key(iter, salt, False)
        lls, oks = [], []
        for r in range(r0, r1):
            bk = self.layouts[0][r]
            ll, ok = self._solve_block(bk, unit, unit, unit, unit, "fresh", Z, iter, salt)
            lls.append(ll)
            oks.append(ok)
        return np.array(lls), np.array(oks)

    def draw_proposal(self, layout, b0, b1, Z=None, iter=0, salt=0, want_success=False):
        """draw_proposal_path!(bb::BiBlock), src/biblock.jl:78-106: proposal drawn under the
        ACCEPTED law bb.b.PP into bb.b°, starting at bb.b.XX[1].x[1]."""
        iter, salt = self._draw_key(iter, salt, True)
        return self._draw(layout, b0, b1, Z, iter, salt, want_success)

    def _draw(self, layout, b0, b1, Z, iter, salt, want_success=False):
        oks = []
        for bk in self.layouts[layout][b0:b1]:
            bk.llp, ok = self._solve_block(bk, 0, 0, 0, 1, "pcn", Z, iter, salt)
            oks.append(ok)
        return np.array(oks) if want_success else None

    def accept_reject(self, layout, b0, b1, mcmciter, E=None, salt=0, want_acc=False):
        """accept_reject_proposal_path!(bb, i), src/biblock.jl:121-127."""
        kit, ksalt = self._accept_key(mcmciter, salt)
        return self._accept(layout, b0, b1, mcmciter, E, kit, ksalt, want_acc)

    def _accept(self, layout, b0, b1, mcmciter, E, kit, ksalt, want_acc):
        accs = []
        for j, bk in enumerate(self.layouts[layout][b0:b1]):
            e = (float(E[j]) if E is not None
                 else exp1(self.seed, bk.g0 + self.seg_base, kit, ksalt))
            acc = e > -(bk.llp - bk.ll)
            if acc:  # swap_paths!: XX and WW element swaps (src/biblock.jl:148-173)
                for g in range(bk.g0, bk.g1 + 1):
                    self.u.XX[g], self.up.XX[g] = self.up.XX[g], self.u.XX[g]
                    self.u.WW[g], self.up.WW[g] = self.up.WW[g], self.u.WW[g]
            if len(bk.acc_hist):
                bk.acc_hist[mcmciter - 1] = acc   # set_accepted!
                bk.ll_hist[mcmciter - 1] = bk.ll  # save_ll! on b and b°
                bk.llp_hist[mcmciter - 1] = bk.llp
            if acc:
                bk.ll, bk.llp = bk.llp, bk.ll     # swap_ll!
            accs.append(acc)
        return np.array(accs) if want_acc else None

    def loglikhd(self, layout, unit, b0, b1):
        """loglikhd!(b) (src/block.jl:138-152): obs term + Girsanov sums on stored paths."""
        me = self._unit(unit)
        dt = self.dt
        for bk in self.layouts[layout][b0:b1]:
            law0 = me.PP[bk.g0]
            ll = obs_term(self.d, law0.rec, law0.H[0], law0.F[0], me.XX[bk.g0][0], self.prec)
            for g in range(bk.g0, bk.g1 + 1):
                lw = self._law(unit, bk, g)
                aux = self._aux_seg(bk, g) if lw.rec[L_AUXTD] != 0.0 else None
                ll = dt(ll + path_ll_segment(self.model, self.d, self.m, lw.rec, self.t[g], lw.H,
                                             lw.F, me.XX[g], self.prec, aux=aux))
            if unit == 0:
                bk.ll = float(ll)
            else:
                bk.llp = float(ll)

    def recompute_path(self, layout, b0, b1, skip=0, want_success=False):
        """recompute_path!(b°, b.WW; skip) (src/block.jl:159-187) under u°.PP: every
        segment's solve_and_ll!(…; skip) leaves its last `skip` Girsanov terms out."""
        assert skip >= 0
        oks = []
        lib.orc_set_ll_skip(int(skip))
        try:
            for bk in self.layouts[layout][b0:b1]:
                bk.llp, ok = self._solve_block(bk, 1, 1, 0, 1, "given", None, 0, 0)
                oks.append(ok)
        finally:
            lib.orc_set_ll_skip(0)
        return np.array(oks) if want_success else None

    # ---- guiding terms (recompute_guiding_term!, set_obs!)
    def upload_obs(self, Hobs, Fobs, cobs, artificial_noise=1e-11):
        self.obsH = np.asarray(Hobs, dtype=np.float64).reshape(self.G, self.hp).copy()
        self.obsF = np.asarray(Fobs, dtype=np.float64).reshape(self.G, self.d).copy()
        self.obsc = np.asarray(cobs, dtype=np.float64).reshape(self.G).copy()
        self.art_eps = float(artificial_noise)
        if not hasattr(self, "obsv"):
            self.obsv = np.zeros((self.G, self.d))

    def download_law(self, unit, kind, H_shared=False):
        me = self._unit(unit)
        tab = me.PP if kind == 0 else me.PPb
        H = np.concatenate([lw.H for lw in tab]).astype(np.float64)
        F = np.concatenate([lw.F for lw in tab]).astype(np.float64)
        laws = np.stack([lw.rec for lw in tab])
        return H, F, laws

    def set_proposal_law(self, layout, b0, b1, params, skip=0, critical_change=None):
        """set_proposal_law!(bb, θ°, pnames, critical_change; skip) (src/biblock.jl:334-345):
        u°'s law records ← u's except c(t0) (equalize_law_params!, :390-431), the named
        parameters ← θ° (DD.set_parameters!, :360-364), recompute_guiding_term!(b°) for the
        blocks whose auxiliary law changed (:342) — with critical_change = True for every block,
        with False only where the equalization itself changed it (:361-362) —
        recompute_path!(b°, b.WW) (:343).
        Returns (success, critical) per block."""
        assert skip >= 0
        crit = np.zeros(b1 - b0, dtype=bool)
        for j, bk in enumerate(self.layouts[layout][b0:b1]):
            for g in range(bk.g0, bk.g1 + 1):
                for kind in (0, 1):
                    tab_p = self.up.PP if kind == 0 else self.up.PPb
                    tab_u = self.u.PP if kind == 0 else self.u.PPb
                    if not tab_u or tab_u[g] is None or tab_u[g].rec is None:
                        continue
                    dst = tab_p[g].rec
                    old = dst[L_A:L_TRACE + 1].copy()
                    c0 = dst[L_C0]
                    old_stale = dst[L_GSTALE] != 0.0
                    dst[:] = tab_u[g].rec
                    dst[L_C0] = c0
                    eq = dst[L_A:L_TRACE + 1].copy()  # after equalize_law_params!, before θ°
                    set_law_params(self.model, self.d, dst, params)
                    used = kind == (1 if (not bk.term and g == bk.g1) else 0)
                    new = dst[L_A:L_TRACE + 1].copy()
                    new[L_C0 - L_A] = old[L_C0 - L_A]
                    eq[L_C0 - L_A] = old[L_C0 - L_A]
                    same = lambda x, y: x.view(np.uint64).tolist() == y.view(np.uint64).tolist()  # noqa: E731
                    aux_changed, eq_changed = not same(old, new), not same(old, eq)
                    # u°'s stale-guiding-term bit (libdmt DMT_LAW_GSTALE, k_set_prop_law)
                    if used and critical_change is True:
                        crit[j] = True
                        dst[L_GSTALE] = 0.0
                    elif used and critical_change is not None and not critical_change:
                        crit[j] |= eq_changed
                        dst[L_GSTALE] = 1.0 if (old_stale or aux_changed) and not eq_changed else 0.0
                    elif used:
                        crit[j] |= aux_changed or old_stale
                        dst[L_GSTALE] = 0.0
                    else:
                        dst[L_GSTALE] = 1.0 if old_stale else 0.0
        for j in np.flatnonzero(crit):
            self.recompute_guiding_term(layout, b0 + j, b0 + j + 1, unit=1)
        ok = self.recompute_path(layout, b0, b1, skip=skip, want_success=True)
        return ok, crit

    def set_obs(self, layout, b0, b1):
        """GP.set_obs!(bb) (src/biblock.jl:273-280): P_last of b and b° observes the accepted
        end point; an auxiliary law linearised at its anchor (FHN: y_T, Lorenz: x_T) is
        re-anchored there and re-derived (set_law_params with no parameter writes), so that
        b̃ matches b at the exact end point (set_obs!)."""
        na = {1: 1, 2: 3}.get(self.model, 0)
        for bk in self.layouts[layout][b0:b1]:
            if not bk.term:
                g = bk.g1
                self.obsv[g] = self.u.XX[g][-1].astype(np.float64)
                for unit in (self.u, self.up):
                    if not unit.PPb or unit.PPb[g] is None or unit.PPb[g].rec is None:
                        continue
                    rec = unit.PPb[g].rec
                    if na and rec[L_AUXLIN] != 0.0:
                        rec[L_ANCHOR:L_ANCHOR + na] = self.obsv[g, :na]
                        set_law_params(self.model, self.d, rec, {})

    def recompute_guiding_term(self, layout, b0, b1, unit=0):
        """GP.recompute_guiding_term!(b) (src/block.jl:102-110) for `unit`'s laws: segments
        backward from the block end, P_last with observation + artificial observation, the
        others with observation + the next segment's guiding term at its start."""
        d, hp = self.d, self.hp
        for bk in self.layouts[layout][b0:b1]:
            nxt = None
            for g in range(bk.g1, bk.g0 - 1, -1):
                lw = self._law(unit, bk, g)
                last_b = (not bk.term) and g == bk.g1
                HT = unpacked(self.obsH[g], d)
                FT = self.obsF[g].copy()
                cT = float(self.obsc[g])
                if last_b:
                    inv = 1.0 / self.art_eps
                    vv = 0.0
                    for p in range(d):
                        v = float(self.obsv[g, p])
                        HT[p, p] += inv
                        FT[p] += inv * v
                        vv += v * v
                    cT += 0.5 * inv * vv + 0.5 * d * (LOG2PI + lib.orc_rng_log(self.art_eps))
                elif g < bk.g1:
                    Hn, Fn, cn = nxt
                    HT = HT + Hn
                    FT = FT + Fn
                    cT += cn
                rec = lw.rec
                Bt = rec[31:31 + d * d]
                beta = rec[40:40 + d]
                at = rec[25:25 + hp] - rec[43:43 + hp]
                kind = 1 if last_b else 0
                if rec[L_AUXTD] == 2.0 and self.aux[kind] is not None:
                    rows = self.aux[kind][self.pt_off[g]: self.pt_off[g] + self.npts[g]]
                    H, F, c = backward_filter_segment_tda(d, rows, self.t[g].astype(np.float64),
                                                          packed_sym(HT), FT, cT)
                elif rec[L_AUXTD] != 0.0 and self.aux[kind] is not None:
                    rows = self.aux[kind][self.pt_off[g]: self.pt_off[g] + self.npts[g], :d * d + d]
                    H, F, c = backward_filter_segment_td(d, rows, at, self.t[g].astype(np.float64),
                                                         packed_sym(HT), FT, cT)
                else:
                    H, F, c = backward_filter_segment(d, Bt, beta, at, self.t[g].astype(np.float64),
                                                      packed_sym(HT), FT, cT)
                lw.H = H.astype(self.dt)
                lw.F = F.astype(self.dt)
                lw.rec[L_C0] = c[0]
                nxt = (unpacked(H[0], d), F[0].copy(), float(c[0]))

    def find_W_for_X(self, layout, b0, b1):
        """find_W_for_X!(b) (src/block.jl:118-131): u.WW[g] ← invsolve(u.XX[g], law of g)."""
        for bk in self.layouts[layout][b0:b1]:
            for g in range(bk.g0, bk.g1 + 1):
                lw = self._law(0, bk, g)
                self.u.WW[g][...] = invsolve_segment(self.model, self.d, self.m, lw.rec, self.t[g],
                                                     lw.H, lw.F, self.u.XX[g], self.prec)

    def swap(self, layout, what, b0, b1):
        for bk in self.layouts[layout][b0:b1]:
            for g in range(bk.g0, bk.g1 + 1):
                if what & 1:
                    self.u.XX[g], self.up.XX[g] = self.up.XX[g], self.u.XX[g]
                if what & 2:
                    self.u.WW[g], self.up.WW[g] = self.up.WW[g], self.u.WW[g]
                if what & 4:  # swap_PP! (src/biblock.jl:180-199)
                    self.u.PP[g], self.up.PP[g] = self.up.PP[g], self.u.PP[g]
                    if not bk.term:
                        self.u.PPb[g], self.up.PPb[g] = self.up.PPb[g], self.u.PPb[g]
            if what & 8:
                bk.ll, bk.llp = bk.llp, bk.ll

    def save_ll(self, layout, b0, b1, mcmciter):
        for bk in self.layouts[layout][b0:b1]:
            bk.ll_hist[mcmciter - 1] = bk.ll
            bk.llp_hist[mcmciter - 1] = bk.llp

    def set_ll(self, layout, unit, b0, b1, mcmciter, v):
        """set_ll!(b, i, v), src/block.jl:82-86 (b = bb.b for U, bb.b° for UPROP)."""
        v = np.broadcast_to(np.asarray(v, dtype=np.float64), (b1 - b0,))
        for j, bk in enumerate(self.layouts[layout][b0:b1]):
            (bk.ll_hist if unit == 0 else bk.llp_hist)[mcmciter - 1] = v[j]

    def set_accepted(self, layout, b0, b1, mcmciter, v):
        v = np.broadcast_to(np.asarray(v, dtype=bool), (b1 - b0,))
        for j, bk in enumerate(self.layouts[layout][b0:b1]):
            bk.acc_hist[mcmciter - 1] = v[j]

    def block_ll(self, layout, b0, b1):
        bks = self.layouts[layout][b0:b1]
        return np.array([b.ll for b in bks]), np.array([b.llp for b in bks])

    def histories(self, layout, b0, b1):
        bks = self.layouts[layout][b0:b1]
        return (np.stack([b.ll_hist for b in bks], 1), np.stack([b.llp_hist for b in bks], 1),
                np.stack([b.acc_hist for b in bks], 1))

    def set_shard(self, seg_base):
        self.seg_base = int(seg_base)

    def get_block_state(self, layout, what, b0, b1, hist_len=None):
        """Same contract as dmt_get_block_state (histories iteration-major)."""
        bks = self.layouts[layout][b0:b1]
        if what == 0:
            return np.array([b.ll for b in bks])
        if what == 1:
            return np.array([b.llp for b in bks])
        h = {2: "ll_hist", 3: "llp_hist", 4: "acc_hist"}[what]
        out = np.stack([getattr(b, h) for b in bks], 1)
        return out.astype(np.uint8) if what == 4 else out

    def set_block_state(self, layout, what, b0, b1, values):
        bks = self.layouts[layout][b0:b1]
        v = np.asarray(values)
        for j, b in enumerate(bks):
            if what == 0:
                b.ll = float(v[j])
            elif what == 1:
                b.llp = float(v[j])
            else:
                h = {2: "ll_hist", 3: "llp_hist", 4: "acc_hist"}[what]
                getattr(b, h)[...] = v[:, j]

    def mcmc_step(self, layout, b0, b1, mcmciter, salt=0, local=False):
        """dmt_mcmc_step: draw + accept with ONE key (disjoint normal / Exp(1) streams)."""
        it, ks = self._draw_key(mcmciter, salt, False)
        self._draw(layout, b0, b1, None, it, ks)
        self._accept(layout, b0, b1, mcmciter, None, it, ks, False)
        return self.fetch_ll(layout, b0, b1, mcmciter)

    def mcmc_run(self, layout, b0, b1, iter0, n_iter, salt=0, local=False):
        """dmt_mcmc_run: iteration it keyed by it (explicit) or by n_iter consecutive counter
        values that do not straddle a 2^32 boundary (RNG_AUTO)."""
        delta, ks = 0, salt
        if salt == RNG_AUTO:
            base = self.rng_ctr
            if (base & 0xFFFFFFFF) + n_iter > 1 << 32:
                base = (base | 0xFFFFFFFF) + 1
            self.rng_ctr, self.rng_pending = base + n_iter, False
            ks = auto_key(base)[1]
            delta = (base & 0xFFFFFFFF) - iter0
        out = np.empty((n_iter, 3))
        for i in range(n_iter):
            it = iter0 + i
            key = (it + delta) & 0xFFFFFFFF
            self._draw(layout, b0, b1, None, key, ks)
            self._accept(layout, b0, b1, it, None, key, ks, False)
            out[i] = self.fetch_ll(layout, b0, b1, it)
        return out

    def fetch_ll(self, layout, b0, b1, mcmciter=0, local=False):
        bks = self.layouts[layout][b0:b1]
        a = pairwise_tree([b.ll for b in bks])
        p = pairwise_tree([b.llp for b in bks])
        n = int(sum(bool(b.acc_hist[mcmciter - 1]) for b in bks)) if mcmciter > 0 else 0
        return a, p, n
